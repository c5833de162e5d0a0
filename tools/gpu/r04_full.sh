#!/bin/bash
# Round 4: the whole GPU suite, then smoke().
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/full_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -25 gpurun_out/full_gpu.log
if [ $rc -ge 124 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full_smoke.log 2>&1
echo "smoke rc=$?"
tail -3 gpurun_out/full_smoke.log
