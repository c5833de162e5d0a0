#!/bin/bash
# Round 5, pass n: the empty fallback launch's dispatch cost against its grid (16 blocks,
# the default, vs 1 / 4), on the headline and config 2, twice each.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5n
mkdir -p $O
export TMPDIR=/tmp
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "median", round(d["ms_per_step"],4), "mean", round(d["ms_per_step_mean"],4), d["solver_iters_per_ph_iter"])'
b() { n=$1; shift; timeout -k 10 300 "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || exit $r; grep '^{' $O/$n.log | python3 -c "$S"; }
for rep in 1 2; do
  b c3_fb16_$rep python3 -u bench.py --no-cpu-baseline
  b c3_fb1_$rep env PHGPU_IPM_FB_BLOCKS=1 python3 -u bench.py --no-cpu-baseline
  b c3_fb4_$rep env PHGPU_IPM_FB_BLOCKS=4 python3 -u bench.py --no-cpu-baseline
done
b c2_fb16 python3 -u bench.py --no-cpu-baseline --scens 1024 --cm 10
b c2_fb1 env PHGPU_IPM_FB_BLOCKS=1 python3 -u bench.py --no-cpu-baseline --scens 1024 --cm 10
echo done
