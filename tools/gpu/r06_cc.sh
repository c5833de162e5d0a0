#!/bin/bash
# Round 6, pass cc: the PH step's rank sums through the library's own RCCL communicator:
# its bit-for-bit test against torch.distributed, the loopback step times (library RCCL /
# torch RCCL / stand-in), the multi-rank tests.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6cc
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_native_rccl.py tests/test_gpu_loopback.py tests/test_gpu_dist_scale.py > $O/tests.log 2>&1; r=$?; echo "tests rc=$r"; grep -E "PASSED|FAILED|passed|failed" $O/tests.log | tail -8; [ $r -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -20; exit 1; }
MASTER_ADDR=127.0.0.1 MASTER_PORT=29551 timeout -k 10 400 python3 -u tools/fake_ranks.py 8 100 rccl > $O/rccl.log 2>&1; r=$?; echo "rccl rc=$r"; grep -E "loopback" $O/rccl.log | cut -c1-150; [ $r -eq 0 ] || { tail -20 $O/rccl.log; exit 1; }
echo done
