#!/bin/bash
# Round 6, closing pass 3: the other configurations' bench lines on this round's build.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6z3
mkdir -p $O
export TMPDIR=/tmp
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],2), "mean_ms", round(d.get("ms_per_step_mean", d["ms_per_step"]),4), "median", round(d.get("ms_per_step_median", d["ms_per_step"]),4), "launch", round(d["roofline"]["launch_ms"],4), d["roofline"]["frac"], d["solver_iters_per_ph_iter"], (d.get("checks") or {}).get("all_ok"))'
b() { n=$1; t=$2; shift 2; timeout -k 10 $t python3 -u bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || { tail -20 $O/$n.log; exit $r; }; grep '^{' $O/$n.log | python3 -c "$S"; }
b cfg2 300 --scens 1024 --cm 10
b cfg4 300 --model aircond
b s32768 200 --scens 32768
b s16384 200 --scens 16384
b s8192 200 --scens 8192
b cm64 400 --cm 64 --steps 10 --warmup 3
b gloo2 300 --gpus 2 --backend gloo
echo done
