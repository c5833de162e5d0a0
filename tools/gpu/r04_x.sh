#!/bin/bash
# Round 4, pass x: config 2 with re-centring only (no cold-retry code) at several budgets.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in "IPM_RETRY=0;IPM_RECENTER=4" "IPM_RETRY=0;IPM_RECENTER=8"; do
  PHGPU_IPM_DEFS="$d" timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --scens 1024 --cm 10 > gpurun_out/x_b.log 2>&1
  echo "cfg2 [$d] rc=$?"; grep '^{' gpurun_out/x_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4), round(d['time_split_ms']['solve_launch'],4), d['solver_iters_per_ph_iter'], d['all_optimal'])"
  PHGPU_IPM_DEFS="$d" timeout -k 10 200 python3 -u tests/diag_ipm_cm64.py 12 1024 first 10 > gpurun_out/x_d.log 2>&1
  echo "diag [$d] rc=$?"; grep "^PH it" gpurun_out/x_d.log | cut -c1-110
  PHGPU_IPM_DEFS="$d" timeout -k 10 300 python3 -u -m pytest -m gpu -q --timeout 120 --timeout-method thread tests/test_gpu_scale.py::test_config2_farmer1024_cm10_bound tests/test_gpu_scale.py::test_config2_ph_iterations_to_convergence tests/test_gpu_parity.py::test_farmer_cm10_parity tests/test_gpu_ipm_wave.py > gpurun_out/x_t.log 2>&1
  echo "tests [$d] rc=$?"; tail -1 gpurun_out/x_t.log
done
