#!/bin/bash
# Round 4, pass w: config 2 without the subtree kernel's cold retry (re-centring only).
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in "IPM_RETRY=0" "IPM_RECENTER=4"; do
  PHGPU_IPM_DEFS="$d" timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --scens 1024 --cm 10 > gpurun_out/w_b.log 2>&1
  echo "cfg2 [$d] rc=$?"; grep '^{' gpurun_out/w_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4), round(d['time_split_ms']['solve_launch'],4), d['solver_iters_per_ph_iter'], d['all_optimal'])"
  PHGPU_IPM_DEFS="$d" timeout -k 10 200 python3 -u tests/diag_ipm_cm64.py 8 1024 first 10 > gpurun_out/w_d.log 2>&1
  echo "diag [$d] rc=$?"; grep "^PH it" gpurun_out/w_d.log | cut -c1-130
done
