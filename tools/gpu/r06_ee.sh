#!/bin/bash
# Round 6, pass ee: two library RCCL communicators (one per issuing stream): the native-RCCL
# test, the multi-rank tests, the RCCL loopback three times.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6ee
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_native_rccl.py tests/test_gpu_loopback.py tests/test_gpu_dist_scale.py > $O/tests.log 2>&1; r=$?; echo "tests rc=$r"; tail -1 $O/tests.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit 1; }
for rep in 1 2 3; do MASTER_ADDR=127.0.0.1 MASTER_PORT=2958$rep timeout -k 10 400 python3 -u tools/fake_ranks.py 8 100 rccl > $O/rccl_$rep.log 2>&1; echo "rccl rc=$?"; grep -E "loopback" $O/rccl_$rep.log | cut -c1-110; done
echo done
