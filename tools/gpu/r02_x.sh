#!/bin/bash
# speculative next solve: headline bench x2, UC PH test, full GPU suite
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_spec$k.log 2>&1 || exit 1
  tail -1 gpurun_out/bench_spec$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['time_split_ms'], d['all_optimal'])"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests_spec.log 2>&1
rc=$?; tail -3 gpurun_out/gputests_spec.log; exit $rc
