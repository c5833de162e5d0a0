#!/bin/bash
# Round 6, pass mm: k_ph_update's loads guarded per trip (a wave past S issues none): the RCCL
# loopback at the 8,192 share (3 runs), config 4's line, the update / readback tests.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6mm
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_readback.py tests/test_gpu_dist_scale.py > $O/tests.log 2>&1; r=$?; echo "tests rc=$r"; tail -1 $O/tests.log; [ $r -eq 0 ] || exit 1
for k in 1 2 3; do MASTER_ADDR=127.0.0.1 MASTER_PORT=2957$k timeout -k 10 300 python3 -u tools/fake_ranks.py 8 100 rccl > $O/rccl$k.log 2>&1 || { echo "rccl$k failed"; exit 1; }; grep -E "library" $O/rccl$k.log | cut -c1-110; done
timeout -k 10 300 python3 -u bench.py --model aircond --bf 32,32,64 --no-cpu-baseline --check on > $O/air.log 2>&1 || { echo "air failed"; exit 1; }; grep '^{' $O/air.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("config4", d["value"], d["ms_per_step"], d.get("ms_per_step_median"), (d.get("checks") or {}).get("all_ok"))'
echo done
