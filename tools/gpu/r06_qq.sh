#!/bin/bash
# Round 6, pass qq: config 4 with the primal iterate in LDS as well (IPM_LDS_ISL=2: 132 -> 84 B
# of scratch offline, 156 KB of LDS) against the automatic choice (IPM_LDS_ISL=1), alternating.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6qq
mkdir -p $O
export TMPDIR=/tmp
run() { timeout -k 10 300 python3 -u bench.py --model aircond --bf 32,32,64 --no-cpu-baseline --check on > $O/$1.log 2>&1 || { echo "$1 failed"; tail -5 $O/$1.log; exit 1; }; echo "$1 $(grep '^{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("ms_per_step_median"), (d.get("checks") or {}).get("all_ok"))')"; }
run auto1
PHGPU_IPM_DEFS="IPM_LDS_ISL=2" run x1
run auto2
PHGPU_IPM_DEFS="IPM_LDS_ISL=2" run x2
echo done
