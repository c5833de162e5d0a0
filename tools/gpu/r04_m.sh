#!/bin/bash
# Round 4, pass m: bound snapping at store (lane groups, subtree) -- config 4 W, the config-4
# and speculative tests, config 2 tests.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 -u tests/diag_config4.py > gpurun_out/m_c4.log 2>&1
echo "diag rc=$?"; grep -v "amdgpu.ids" gpurun_out/m_c4.log | tail -8 | cut -c1-250
T="python3 -u -m pytest -m gpu -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_config4.py tests/test_gpu_speculative.py tests/test_gpu_scale.py tests/test_gpu_parity.py > gpurun_out/m_tests.log 2>&1
echo "tests rc=$?"; tail -6 gpurun_out/m_tests.log
