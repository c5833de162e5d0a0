#!/bin/bash
# A/B: path 4 one slice per step (exp/libphgpu_base.so) vs two interleaved slices (in-tree)
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
for S in 64 512; do
  PHGPU_LIB=$PWD/exp/libphgpu_base.so timeout -k 10 200 python -u tools/uc_prof.py $S 2048 > gpurun_out/ab_base_S$S.log 2>&1 || exit 1
  echo "base $(tail -1 gpurun_out/ab_base_S$S.log)"
  timeout -k 10 200 python -u tools/uc_prof.py $S 2048 > gpurun_out/ab_pair_S$S.log 2>&1 || exit 1
  echo "pair $(tail -1 gpurun_out/ab_pair_S$S.log)"
done
