#!/bin/bash
# Round 4, pass ac: the split streaming form on a counter barrier -- split tests, then
# config 5 with the longest 1 / 4 scenarios split (kernel trace of the first).
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out/ac
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -m gpu -v --timeout 150 --timeout-method thread tests/test_gpu_uc.py -k split > gpurun_out/ac/tests.log 2>&1
r=$?; echo "tests rc=$r"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/ac/tests.log | tail -6; [ $r -eq 0 ] || exit $r
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],4), round(d["ms_per_step"],1), d["solver_iters_per_ph_iter"], d["all_optimal"])'
export PHGPU_STREAM_SPLIT=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ac/prof_t1 -o run -- python3 -u bench.py --no-cpu-baseline --model uc --steps 2 --warmup 1 > gpurun_out/ac/uc_1.log 2>&1; r=$?; echo "uc T=1 rc=$r"; [ $r -eq 0 ] || exit $r
grep '^{' gpurun_out/ac/uc_1.log | python3 -c "$S"
f=$(find gpurun_out/ac/prof_t1 -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cut -d, -f1-8 "$f" | head -8
export PHGPU_STREAM_SPLIT=4
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --model uc --steps 2 --warmup 1 > gpurun_out/ac/uc_4.log 2>&1; r=$?; echo "uc T=4 rc=$r"; [ $r -eq 0 ] || exit $r
grep '^{' gpurun_out/ac/uc_4.log | python3 -c "$S"
