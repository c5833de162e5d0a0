#!/bin/bash
# Round 4, pass y: re-centring-only default in the subtree kernel -- medium-path GPU tests,
# config 2 bench, the config-2 diagnostic.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out/y
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest -m gpu -q --timeout 150 --timeout-method thread tests/test_gpu_ipm_wave.py tests/test_gpu_wg.py tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_speculative.py > gpurun_out/y/tests.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/y/tests.log
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --scens 1024 --cm 10 > gpurun_out/y/cfg2.log 2>&1
echo "cfg2 rc=$?"; grep '^{' gpurun_out/y/cfg2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4), round(d['time_split_ms']['solve_launch'],4), d['solver_iters_per_ph_iter'], d['all_optimal'], round(d['roofline']['frac'],3))"
timeout -k 10 200 python3 -u tests/diag_ipm_cm64.py 12 1024 first 10 > gpurun_out/y/diag10.log 2>&1
echo "diag rc=$?"; grep "^PH it" gpurun_out/y/diag10.log | cut -c1-110
