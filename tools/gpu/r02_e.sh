#!/bin/bash
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/debug_wheel_ranks.py > gpurun_out/debug_wheel.log 2>&1; echo rc=$?
grep -v "socket.cpp\|Gloo\]\|amdgpu.ids" gpurun_out/debug_wheel.log | grep -v "^\[ *[0-9.]*\] *[0-9]* " | head -150
