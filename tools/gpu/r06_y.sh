#!/bin/bash
# Round 6, pass y: the cluster form with each cluster's workgroups on one XCD: UC cluster
# tests, then the 125-scenario share with and without (PHGPU_STREAM_XCD=0), alternating.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6y
mkdir -p $O
export TMPDIR=/tmp
S='import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"],4), "mean_ms", round(d.get("ms_per_step_mean", d["ms_per_step"]),1), "launch", round(r["launch_ms"],1), r.get("kernel"), r.get("workgroups_per_scenario"), d["solver_iters_per_ph_iter"])'
b() { n=$1; shift; timeout -k 10 500 python3 -u bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || { tail -20 $O/$n.log; exit $r; }; grep '^{' $O/$n.log | python3 -c "$S"; }
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 500 --timeout-method thread -m gpu tests/test_gpu_uc.py -k "cluster or split or relaxation" > $O/tests.log 2>&1; r=$?; echo "tests rc=$r"; tail -1 $O/tests.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit 1; }
for rep in 1 2; do
  b uc125_xcd_$rep --model uc --scens 125 --steps 2 --warmup 1
  PHGPU_STREAM_XCD=0 b uc125_seq_$rep --model uc --scens 125 --steps 2 --warmup 1
done
echo done
