#!/bin/bash
# Round 6, pass l: why the fused PH loop declines (engine.ph_loop_declined).
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fused_loop.py -k five > $O/tests.log 2>&1; r=$?; echo "tests rc=$r"; grep -E "AssertionError|phgpu|passed|failed" $O/tests.log | tail -8
