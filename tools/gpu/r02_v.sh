#!/bin/bash
# deferred gripe readback: headline bench x2 + GPU parity subset
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_gripe$k.log 2>&1 || exit 1
  tail -1 gpurun_out/bench_gripe$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['time_split_ms'])"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_wheel.py tests/test_gpu_scale.py tests/test_gpu_uc.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests_gripe.log 2>&1
rc=$?; tail -2 gpurun_out/gputests_gripe.log; exit $rc
