#!/bin/bash
# Round 6, pass m: the cluster form of the streaming kernel (path 4, a batch smaller than
# the GPU): its UC test against the queue form and HiGHS, then the 125-scenario UC share
# (config 5 at N = 8) with and without it.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6m
mkdir -p $O
export TMPDIR=/tmp
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],4), "mean_ms", round(d.get("ms_per_step_mean", d["ms_per_step"]),1), "median", round(d.get("ms_per_step_median", d["ms_per_step"]),1), "launch", round(d["roofline"]["launch_ms"],1), d["roofline"]["frac"], d["solver_iters_per_ph_iter"], d.get("iter_ms"))'
b() { n=$1; shift; timeout -k 10 500 python3 -u bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || { tail -20 $O/$n.log; exit $r; }; grep '^{' $O/$n.log | python3 -c "$S"; }
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_uc.py -k "cluster or split or relaxation" > $O/tests.log 2>&1; r=$?; echo "tests rc=$r"; grep -E "PASSED|FAILED|passed|failed" $O/tests.log | tail -12; [ $r -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -20; exit 1; }
b uc125 --model uc --scens 125 --steps 3 --warmup 1
PHGPU_STREAM_CLUSTER=0 b uc125_queue --model uc --scens 125 --steps 3 --warmup 1
echo done
