#!/bin/bash
# Round 5, pass z: config 2's subtree interior point under other constants (PHGPU_IPM_DEFS):
# the centring floor / warm-start push that helped config 4, and the Mehrotra corrector.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5z
mkdir -p $O
export TMPDIR=/tmp
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "median", round(d["ms_per_step"],4), "mean", round(d["ms_per_step_mean"],4), d["solver_iters_per_ph_iter"], d["all_optimal"], d.get("path6_last_solve_jam_handovers"))'
b() { n=$1; d=$2; timeout -k 10 200 env PHGPU_IPM_DEFS="$d" python3 -u bench.py --no-cpu-baseline --scens 1024 --cm 10 > $O/$n.log 2>&1; r=$?; echo "$n [$d] rc=$r"; [ $r -eq 0 ] || exit $r; grep '^{' $O/$n.log | python3 -c "$S"; }
for rep in 1 2; do
  b def_$rep ""
  b both_$rep "IPM_SIG_MIN=0.003;IPM_WARM_T=0.3"
  b wt_$rep "IPM_WARM_T=0.3"
  b smin_$rep "IPM_SIG_MIN=0.003"
  b mpc_$rep "IPM_MPC=1"
done
echo done
