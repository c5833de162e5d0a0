#!/bin/bash
# Round 4, closing pass: whole GPU suite + smoke, then the default bench line.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out/final2
export TMPDIR=/tmp
bash tools/gpu/r04_full.sh || exit $?
timeout -k 10 400 python3 -u bench.py > gpurun_out/final2/bench_default.log 2>&1; r=$?; echo "bench rc=$r"; [ $r -eq 0 ] || exit $r
grep '^{' gpurun_out/final2/bench_default.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), round(d["ms_per_step"],4), d["roofline"]["frac"], d["cpu_baseline"]["value"] if d.get("cpu_baseline") else None)'
