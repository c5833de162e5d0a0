#!/bin/bash
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/loop_prof.py > gpurun_out/loop_prof.log 2>&1; rc=$?; tail -4 gpurun_out/loop_prof.log; exit $rc
