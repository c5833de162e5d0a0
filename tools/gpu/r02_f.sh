#!/bin/bash
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/cm64_eps.py 1e-9 1e-9,1e-10,1e-11,1e-12 > gpurun_out/cm64_eps0.log 2>&1; echo rc=$?; grep eps gpurun_out/cm64_eps0.log
timeout -k 10 300 python -u -m pytest tests/test_wheel_ranks.py -v --timeout 280 --timeout-method thread > gpurun_out/wheel_ranks.log 2>&1; echo rc=$?; tail -3 gpurun_out/wheel_ranks.log
