#!/bin/bash
# Round 4, pass aa: config 4 (aircond 65,536) lanes per scenario A/B after the accuracy work.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out/aa
export TMPDIR=/tmp
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), round(d["ms_per_step"],4), round(d["time_split_ms"]["solve_launch"],4), d["solver_iters_per_ph_iter"], d["all_optimal"], d["roofline"]["kernel"], d["roofline"].get("lanes_per_scenario"))'
for L in default 1 2 8; do
  if [ $L = default ]; then unset PHGPU_IPM_LANES; else export PHGPU_IPM_LANES=$L; fi
  timeout -k 10 240 python3 -u bench.py --no-cpu-baseline --model aircond > gpurun_out/aa/air_$L.log 2>&1; r=$?; echo "L=$L rc=$r"; [ $r -eq 0 ] || exit $r
  grep '^{' gpurun_out/aa/air_$L.log | python3 -c "$S"
done
