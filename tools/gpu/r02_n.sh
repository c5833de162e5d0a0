#!/bin/bash
# path 4 after balancing + early loads: timing, then the path-4 GPU tests
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
for S in 64 512; do
  timeout -k 10 200 python -u tools/uc_prof.py $S 2048 > gpurun_out/prof_S$S.log 2>&1 || exit 1
  tail -1 gpurun_out/prof_S$S.log
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_uc.py -x -q --timeout 300 --timeout-method thread -k "not ph_iterations" > gpurun_out/gputests_uc.log 2>&1
rc=$?; tail -3 gpurun_out/gputests_uc.log; exit $rc
