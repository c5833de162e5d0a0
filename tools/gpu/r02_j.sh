#!/bin/bash
# config 5 (UC, 1000 scenarios) bench, first full-scale run of path 4
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u bench.py --model uc --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_uc1000.log 2>&1
rc=$?; echo "uc bench rc=$rc"; tail -5 gpurun_out/bench_uc1000.log | cut -c1-3000
exit $rc
