#!/bin/bash
# Round 6, pass b: the lane-group kernel's statistics atomics per wave instead of per group
# (A/B at the 8,192 share), its phase profile with wave lifetimes, the lane-group tests.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6b
mkdir -p $O
export TMPDIR=/tmp
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "mean_ms", round(d["ms_per_step"],4), "median_ms", round(d["ms_per_step_median"],4), "launch", round(d["roofline"]["launch_ms"],4), d["solver_iters_per_ph_iter"], d["all_optimal"])'
b() { n=$1; shift; timeout -k 10 200 python3 -u bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || { tail -20 $O/$n.log; exit $r; }; grep '^{' $O/$n.log | python3 -c "$S"; }
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ipm.py -k "stats or lane" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  b s8192_wave_$rep --scens 8192
  PHGPU_IPM_DEFS="IPM_ML_STATS_GROUP=1" b s8192_group_$rep --scens 8192
done
b s16384 --scens 16384
b s65536 --steps 40
timeout -k 10 200 python3 -u tools/ipm_prof.py 8192 8 > $O/prof_8192_L8.log 2>&1 && tail -1 $O/prof_8192_L8.log
timeout -k 10 200 python3 -u tools/ipm_prof.py 8192 16 > $O/prof_8192_L16.log 2>&1 && tail -1 $O/prof_8192_L16.log
echo done
