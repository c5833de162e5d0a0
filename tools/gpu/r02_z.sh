#!/bin/bash
# path 4 slots: B=2 vs B=4 at saturation
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
for S in 512 1000; do
  for B in 2 4; do
    PHGPU_STREAM_SLOTS=$B timeout -k 10 200 python -u tools/uc_prof.py $S 2048 > gpurun_out/slots4_B${B}_S$S.log 2>&1 || exit 1
    echo "B=$B $(tail -1 gpurun_out/slots4_B${B}_S$S.log)"
  done
done
