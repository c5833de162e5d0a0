#!/bin/bash
# Round 4, pass v: the permlane-swap workgroup sums (correctness on the subtree-kernel tests,
# config 2 speed) against the readlane version.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
PHGPU_IPM_DEFS="IPM_PERMLANE=1" timeout -k 10 300 python3 -u -m pytest -m gpu -q --timeout 120 --timeout-method thread tests/test_gpu_ipm_wave.py tests/test_gpu_scale.py::test_config2_farmer1024_cm10_bound tests/test_gpu_parity.py::test_farmer_cm10_parity > gpurun_out/v_tests.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/v_tests.log
for d in "" "IPM_PERMLANE=1"; do
  PHGPU_IPM_DEFS="$d" timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --scens 1024 --cm 10 > gpurun_out/v_b.log 2>&1
  echo "cfg2 [$d] rc=$?"; grep '^{' gpurun_out/v_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4), round(d['time_split_ms']['solve_launch'],4), d['solver_iters_per_ph_iter'], d['all_optimal'])"
done
