#!/bin/bash
# Round 5, pass bb: the 8,192 share (lane groups of 8) under the config-4 constants.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5bb
mkdir -p $O
export TMPDIR=/tmp
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "median", round(d["ms_per_step"],4), "mean", round(d["ms_per_step_mean"],4), d["solver_iters_per_ph_iter"], d["all_optimal"])'
b() { n=$1; d=$2; timeout -k 10 200 env PHGPU_IPM_DEFS="$d" python3 -u bench.py --no-cpu-baseline --scens 8192 > $O/$n.log 2>&1; r=$?; echo "$n [$d] rc=$r"; [ $r -eq 0 ] || exit $r; grep '^{' $O/$n.log | python3 -c "$S"; }
for rep in 1 2; do
  b def_$rep ""
  b both_$rep "IPM_SIG_MIN=0.003;IPM_WARM_T=0.3"
  b wt_$rep "IPM_WARM_T=0.3"
done
echo done
