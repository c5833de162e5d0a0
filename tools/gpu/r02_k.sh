#!/bin/bash
# path 4 with sliced-ELL passes: GPU tests of path 4 / UC, then the config 5 bench
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_uc.py -v -x --durations=0 -k "fix_nonants" --timeout 300 --timeout-method thread > gpurun_out/gputests_uc.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -12 gpurun_out/gputests_uc.log | cut -c1-400
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u bench.py --model uc --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_uc1000.log 2>&1
rc=$?; echo "uc bench rc=$rc"; tail -3 gpurun_out/bench_uc1000.log | cut -c1-1500
exit $rc
