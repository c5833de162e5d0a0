#!/bin/bash
# Round 4, pass ad: config 5 with two streaming workgroups per CU (every scenario in flight).
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out/ad
export TMPDIR=/tmp
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],4), round(d["ms_per_step"],1), d["solver_iters_per_ph_iter"], d["all_optimal"])'
PHGPU_STREAM_PER_CU=2 timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --model uc --steps 2 --warmup 1 > gpurun_out/ad/uc_pc2.log 2>&1; r=$?; echo "uc per_cu=2 rc=$r"; [ $r -eq 0 ] || exit $r
grep '^{' gpurun_out/ad/uc_pc2.log | python3 -c "$S"
PHGPU_STREAM_PER_CU=2 PHGPU_STREAM_SLOTS=1 timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --model uc --steps 2 --warmup 1 > gpurun_out/ad/uc_pc2_b1.log 2>&1; r=$?; echo "uc per_cu=2 B=1 rc=$r"; [ $r -eq 0 ] || exit $r
grep '^{' gpurun_out/ad/uc_pc2_b1.log | python3 -c "$S"
