#!/bin/bash
# parallel setup for large patterns: parity tests (cm=10, cm=64, random long rows) + cm=64 setup time
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_wg.py tests/test_gpu_scale.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests_setup.log 2>&1
rc=$?; tail -3 gpurun_out/gputests_setup.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cm64s -o run -- python3 bench.py --cm 64 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_cm64s.log 2>&1
rc=$?; tail -1 gpurun_out/prof_cm64s.log | cut -c1-300; exit $rc
