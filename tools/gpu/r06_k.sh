#!/bin/bash
# Round 6, pass k: the fused PH loop (phgpu_ph_loop) on the GPU: its tests, the convergence
# tests, and the headline bench with and without it.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6k
mkdir -p $O
export TMPDIR=/tmp
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "mean_ms", round(d.get("ms_per_step_mean", d["ms_per_step"]),4), "median", round(d.get("ms_per_step_median", d["ms_per_step"]),4), "launch", round(d["roofline"]["launch_ms"],4), d["roofline"]["frac"], d["solver_iters_per_ph_iter"], (d.get("checks") or {}).get("all_ok"), d.get("fused_ph_loop"))'
b() { n=$1; shift; timeout -k 10 300 python3 -u bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || { tail -20 $O/$n.log; exit $r; }; grep '^{' $O/$n.log | python3 -c "$S"; }
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fused_loop.py tests/test_gpu_convergence.py tests/test_gpu_speculative.py > $O/tests.log 2>&1; r=$?; echo "tests rc=$r"; grep -E "PASSED|FAILED|passed|failed" $O/tests.log | tail -20; [ $r -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -20; exit 1; }
b s65536
b s65536_step --no-fused-loop
b s65536_k100 --steps 100
b s8192 --scens 8192
b cm10 --scens 1024 --cm 10
echo done
