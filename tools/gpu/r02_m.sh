#!/bin/bash
# experiment: gathers confined to an 8 KB window (wrong results, timing only)
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
for S in 64 512; do
  timeout -k 10 200 python -u tools/uc_prof.py $S 2048 > gpurun_out/exp_base_S$S.log 2>&1 || exit 1
  tail -1 gpurun_out/exp_base_S$S.log
  PHGPU_LIB=$PWD/exp/libphgpu_localgather.so timeout -k 10 200 python -u tools/uc_prof.py $S 2048 > gpurun_out/exp_lg_S$S.log 2>&1 || exit 1
  tail -1 gpurun_out/exp_lg_S$S.log
done
