#!/bin/bash
# Round 6, pass ss: config 3 with the slack reciprocals in LDS (IPM_LDS_ISL=1 forced; the
# module spills nothing, 444 registers of which 188 AGPRs) against the default, alternating.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6ss
mkdir -p $O
export TMPDIR=/tmp
run() { timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > $O/$1.log 2>&1 || { echo "$1 failed"; tail -5 $O/$1.log; exit 1; }; echo "$1 $(grep '^{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("ms_per_step_median"), d["roofline"]["launch_ms"], (d.get("checks") or {}).get("all_ok"))')"; }
run def1
PHGPU_IPM_DEFS="IPM_LDS_ISL=1" run lds1
run def2
PHGPU_IPM_DEFS="IPM_LDS_ISL=1" run lds2
echo done
