#!/bin/bash
# Round 5, pass cc: config 5 with the KKT test every 256, and a longer step (eta_frac 0.999), around
# beta_sufficient 0.7; 2 timed PH iterations each.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5cc
mkdir -p $O
export TMPDIR=/tmp
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],4), "median", round(d["ms_per_step"],1), "mean", round(d["ms_per_step_mean"],1), d["solver_iters_per_ph_iter"], d["all_optimal"])'
b() { n=$1; shift; timeout -k 10 390 python3 -u bench.py --no-cpu-baseline --model uc --steps 2 --warmup 1 "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || exit $r; grep '^{' $O/$n.log | python3 -c "$S"; }
b uc_c256 --solver-opt beta_sufficient=0.7 --solver-opt check_every=256
b uc_c128_e999 --solver-opt beta_sufficient=0.7 --solver-opt check_every=128 --solver-opt eta_frac=0.999
echo done
