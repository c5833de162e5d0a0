#!/bin/bash
# Round 6, pass s: A/B on one box of the one-lane kernel's data-first prologue
# (IPM_DATA_FIRST=1, the default) against the step-first order (=0), config 3 alternating.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6s
mkdir -p $O
export TMPDIR=/tmp
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "mean_ms", round(d.get("ms_per_step_mean", d["ms_per_step"]),4), "median", round(d.get("ms_per_step_median", d["ms_per_step"]),4), "launch", round(d["roofline"]["launch_ms"],4), d["solver_iters_per_ph_iter"]["max"], (d.get("checks") or {}).get("all_ok"))'
b() { n=$1; shift; timeout -k 10 300 python3 -u bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || { tail -20 $O/$n.log; exit $r; }; grep '^{' $O/$n.log | python3 -c "$S"; }
for rep in 1 2 3; do
  PHGPU_IPM_DEFS="IPM_DATA_FIRST=1" b df1_$rep
  PHGPU_IPM_DEFS="IPM_DATA_FIRST=0" b df0_$rep
done
for d in 1 0; do timeout -k 10 200 python3 -u tools/ipm_prof.py 65536 1 --defs "IPM_DATA_FIRST=$d" > $O/l1_df$d.log 2>&1 && tail -1 $O/l1_df$d.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["defs"], d["ms_per_step"], d["span_us"], d["seg_mean_us"]["pre_loop"], d["loop_us_per_trip"])'; done
echo done
