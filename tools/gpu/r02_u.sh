#!/bin/bash
# config 5 on two ranks sharing the GPU (engine-level test)
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_dist_uc.py -v -x --timeout 600 --timeout-method thread > gpurun_out/gputests_dist_uc.log 2>&1
rc=$?; tail -15 gpurun_out/gputests_dist_uc.log | cut -c1-300; exit $rc
