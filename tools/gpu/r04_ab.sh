#!/bin/bash
# Round 4, pass ab: the split (cooperative) form of the streaming kernel -- path-4 GPU
# tests, then config 5 without / with the split of the longest scenarios.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -m gpu -v --timeout 150 --timeout-method thread tests/test_gpu_uc.py > gpurun_out/ab/tests.log 2>&1
r=$?; echo "tests rc=$r"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/ab/tests.log | tail -14; [ $r -eq 0 ] || exit $r
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],4), round(d["ms_per_step"],1), d["solver_iters_per_ph_iter"], d["all_optimal"])'
for T in 0 4; do
  PHGPU_STREAM_SPLIT=$T timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --model uc --steps 2 --warmup 1 > gpurun_out/ab/uc_$T.log 2>&1; r=$?; echo "uc T=$T rc=$r"; [ $r -eq 0 ] || exit $r
  grep '^{' gpurun_out/ab/uc_$T.log | python3 -c "$S"
done
