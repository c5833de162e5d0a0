#!/bin/bash
# Round 5, pass aa: farmer cm = 64 (65,536 scenarios, the workgroup PDHG) under the PDHG
# options that helped config 5 (KKT test every 128, beta_sufficient 0.7).
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5aa
mkdir -p $O
export TMPDIR=/tmp
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],2), "median", round(d["ms_per_step"],3), "mean", round(d["ms_per_step_mean"],3), d["solver_iters_per_ph_iter"], d["all_optimal"])'
b() { n=$1; shift; timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --cm 64 "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || exit $r; grep '^{' $O/$n.log | python3 -c "$S"; }
b def
b c128 --solver-opt check_every=128
b b07 --solver-opt beta_sufficient=0.7
b b07c128 --solver-opt beta_sufficient=0.7 --solver-opt check_every=128
b def2
echo done
