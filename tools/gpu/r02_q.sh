#!/bin/bash
# slot-blocked path 4: timing B=1 vs B=2, then the path-4 GPU tests (B=2 default)
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
for S in 64 512 1000; do
  for B in 1 2; do
    PHGPU_STREAM_SLOTS=$B timeout -k 10 200 python -u tools/uc_prof.py $S 2048 > gpurun_out/slots_B${B}_S$S.log 2>&1 || exit 1
    echo "B=$B $(tail -1 gpurun_out/slots_B${B}_S$S.log)"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_uc.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests_uc.log 2>&1
rc=$?; tail -3 gpurun_out/gputests_uc.log; exit $rc
