#!/bin/bash
# PDHG option sweep on 64 UC scenarios (cold solves, eps 1e-6)
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/uc_sweep.py 64 '{}' '{"beta_sufficient": 0.1}' '{"beta_sufficient": 0.4}' \
  '{"beta_artificial": 0.2}' '{"beta_artificial": 1e9}' '{"omega0": 0.1}' '{"omega0": 10.0}' \
  '{"restart_every": 64}' '{"beta_necessary": 0.9}' > gpurun_out/uc_sweep.log 2>&1
rc=$?; cat gpurun_out/uc_sweep.log | grep cfg; exit $rc
