#!/bin/bash
# Round 5, pass x: the interior point's centring floor and warm-start push (IPM_SIG_MIN 0.003,
# IPM_WARM_T 0.3 vs 0.01 / 0.1) on configs 4 and 3, twice each.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5x
mkdir -p $O
export TMPDIR=/tmp
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "median", round(d["ms_per_step"],4), "mean", round(d["ms_per_step_mean"],4), d["solver_iters_per_ph_iter"], d["all_optimal"])'
b() { n=$1; shift; timeout -k 10 300 "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || exit $r; grep '^{' $O/$n.log | python3 -c "$S"; }
D="IPM_SIG_MIN=0.003;IPM_WARM_T=0.3"
for rep in 1 2; do
  b air_def_$rep python3 -u bench.py --no-cpu-baseline --model aircond
  b air_new_$rep env PHGPU_IPM_DEFS="$D" python3 -u bench.py --no-cpu-baseline --model aircond
  b c3_def_$rep python3 -u bench.py --no-cpu-baseline
  b c3_new_$rep env PHGPU_IPM_DEFS="$D" python3 -u bench.py --no-cpu-baseline
done
echo done
