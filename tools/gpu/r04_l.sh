#!/bin/bash
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for e in 1e-9 1e-10; do
  timeout -k 10 200 python3 -u tests/diag_config4.py $e > gpurun_out/l_c4_$e.log 2>&1
  echo "eps $e rc=$?"; grep -v "amdgpu.ids" gpurun_out/l_c4_$e.log | tail -9 | cut -c1-300
done
