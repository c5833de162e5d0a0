#!/bin/bash
# Round 5, pass e: lane groups of 2 (spills allowed) at 65,536 / 32,768 scenarios against the
# default one-lane kernel.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5e
mkdir -p $O
export TMPDIR=/tmp
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "median", round(d["ms_per_step"],4), "launch", round(d["roofline"]["launch_ms"],4), d["solver_iters_per_ph_iter"], d["all_optimal"])'
b() { n=$1; shift; timeout -k 10 300 python3 -u bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || exit $r; grep '^{' $O/$n.log | python3 -c "$S"; }
b s65536_L1 --scens 65536
PHGPU_IPM_LANES=2 PHGPU_IPM_SPILL_MAX=100000 b s65536_L2 --scens 65536
b s32768_L1 --scens 32768
PHGPU_IPM_LANES=2 PHGPU_IPM_SPILL_MAX=100000 b s32768_L2 --scens 32768
PHGPU_IPM_LANES=2 PHGPU_IPM_SPILL_MAX=100000 b s16384_L2 --scens 16384
echo done
