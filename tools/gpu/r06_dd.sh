#!/bin/bash
# Round 6, pass dd: k_xbar_final's chunk loads issued together: the tests on its paths and
# the multi-rank step times.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6dd
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_readback.py tests/test_gpu_loopback.py tests/test_gpu_dist_scale.py tests/test_gpu_native_rccl.py tests/test_variable_probability.py tests/test_gpu_config4.py > $O/tests.log 2>&1; r=$?; echo "tests rc=$r"; tail -1 $O/tests.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit 1; }
for rep in 1 2; do MASTER_ADDR=127.0.0.1 MASTER_PORT=2957$rep timeout -k 10 400 python3 -u tools/fake_ranks.py 8 100 rccl > $O/rccl_$rep.log 2>&1; echo "rccl rc=$?"; grep -E "loopback" $O/rccl_$rep.log | cut -c1-110; done
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --model aircond > $O/air.log 2>&1; echo "air rc=$?"; grep '^{' $O/air.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], (d.get("checks") or {}).get("all_ok"))'
echo done
