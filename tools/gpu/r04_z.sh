#!/bin/bash
# Round 4, pass z: whole GPU suite + smoke with the plan-dependent retry default, then the
# config-2 and config-3 benches and the opt-in cm = 64 subtree bench at 2048 scenarios.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out/z
export TMPDIR=/tmp
bash tools/gpu/r04_full.sh || exit $?
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), round(d["ms_per_step"],4), d["solver_iters_per_ph_iter"], d["all_optimal"], round(d["roofline"]["frac"],3))'
b() { n=$1; shift; timeout -k 10 240 python3 -u bench.py --no-cpu-baseline "$@" > gpurun_out/z/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || exit $r; grep '^{' gpurun_out/z/$n.log | python3 -c "$S"; }
b cfg2 --scens 1024 --cm 10
b cfg3 --steps 20 --warmup 5
PHGPU_IPM_WAVE=1 b cm64blk --cm 64 --scens 2048 --steps 10 --warmup 3
