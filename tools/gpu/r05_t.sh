#!/bin/bash
# Round 5, pass t (after s): config 5's warm-started PDHG restart criterion (beta_sufficient, default
# 0.2; farmer runs 0.6) on the UC bench, 2 timed PH iterations each.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5t
mkdir -p $O
export TMPDIR=/tmp
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],4), "median", round(d["ms_per_step"],1), "mean", round(d["ms_per_step_mean"],1), d["solver_iters_per_ph_iter"], d["all_optimal"])'
b() { n=$1; shift; timeout -k 10 390 python3 -u bench.py --no-cpu-baseline --model uc --steps 2 --warmup 1 "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || exit $r; grep '^{' $O/$n.log | python3 -c "$S"; }
b uc_b07 --solver-opt beta_sufficient=0.7
b uc_b08 --solver-opt beta_sufficient=0.8
b uc_b06 --solver-opt beta_sufficient=0.6
echo done
