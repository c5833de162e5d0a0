#!/bin/bash
# Round 5, pass v: config 5 PH-solve options around beta_sufficient 0.7 (KKT check every 128, restart test
# every 32, artificial restart 0.5), 2 timed PH iterations each.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5v
mkdir -p $O
export TMPDIR=/tmp
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],4), "median", round(d["ms_per_step"],1), "mean", round(d["ms_per_step_mean"],1), d["solver_iters_per_ph_iter"], d["all_optimal"])'
b() { n=$1; shift; timeout -k 10 390 python3 -u bench.py --no-cpu-baseline --model uc --steps 2 --warmup 1 "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || exit $r; grep '^{' $O/$n.log | python3 -c "$S"; }
b uc_c128 --solver-opt beta_sufficient=0.7 --solver-opt check_every=128
b uc_r32 --solver-opt beta_sufficient=0.7 --solver-opt restart_every=32
b uc_art5 --solver-opt beta_sufficient=0.7 --solver-opt beta_artificial=0.5
echo done
