#!/bin/bash
# Round 6, closing check on the final tree: the readback / config-4 / native-RCCL tests, smoke.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6z7
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_readback.py tests/test_gpu_config4.py tests/test_gpu_native_rccl.py > $O/tests.log 2>&1; r=$?; echo "tests rc=$r"; tail -1 $O/tests.log; [ $r -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit 1; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
echo done
