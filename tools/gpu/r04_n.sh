#!/bin/bash
# Round 4, pass n: complementarity stop in the lane-group kernel -- config 4 W, benches of
# the lane-group shares.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tests/diag_config4.py > gpurun_out/n_c4.log 2>&1
echo "diag rc=$?"; grep -v "amdgpu.ids" gpurun_out/n_c4.log | tail -8 | cut -c1-250
for a in "--model aircond" "--scens 8192" "--model aircond --bf 4,32,64"; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline $a > gpurun_out/n_b.log 2>&1
  echo "bench $a rc=$?"; grep '^{' gpurun_out/n_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4), round(d['time_split_ms']['solve_launch'],4), d['solver_iters_per_ph_iter'], d['all_optimal'], d['roofline']['kernel'])"
done
