#!/bin/bash
# Round 4, pass k: config 4 to convergence with and without the folded step.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python3 -u -m pytest -m gpu -v --timeout 200 --timeout-method thread"
PHGPU_FUSE_STEP=0 timeout -k 10 300 $T tests/test_gpu_config4.py -k iterations_to > gpurun_out/k_nofold.log 2>&1
echo "nofold rc=$?"; grep -E "PASSED|FAILED|^E  +Assert" gpurun_out/k_nofold.log | head -5
timeout -k 10 300 $T tests/test_gpu_config4.py -k iterations_to > gpurun_out/k_fold.log 2>&1
echo "fold rc=$?"; grep -E "PASSED|FAILED|^E  +Assert" gpurun_out/k_fold.log | head -5
