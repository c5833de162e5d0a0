#!/bin/bash
# Round 4, pass q: x̄ partial / PH update over a nonant x scenario-block grid -- tests that
# cover the reductions, then config 2 / config 3 / config 4 benches.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python3 -u -m pytest -m gpu -q --timeout 200 --timeout-method thread"
timeout -k 10 700 $T tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_config4.py tests/test_gpu_speculative.py tests/test_gpu_readback.py tests/test_dist_engine.py > gpurun_out/q_tests.log 2>&1
echo "tests rc=$?"; tail -4 gpurun_out/q_tests.log
for a in "--scens 1024 --cm 10" "" "--model aircond"; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline $a > gpurun_out/q_b.log 2>&1
  echo "bench $a rc=$?"; grep '^{' gpurun_out/q_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4), round(d['time_split_ms']['solve_launch'],4), d['solver_iters_per_ph_iter'], d['all_optimal'])"
done
