#!/bin/bash
# Round 6, pass kk: k_ph_update with a bounded grid (config 4's 1,536 blocks -> 252): the
# update / readback / aircond / distributed GPU tests, config 4 line and trace, the default line.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6kk
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_readback.py tests/test_gpu_config4.py tests/test_gpu_dist_scale.py tests/test_gpu_parity.py tests/test_gpu_convergence.py > $O/tests.log 2>&1; r=$?; echo "tests rc=$r"; tail -1 $O/tests.log; [ $r -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit 1; }
for k in 1 2; do timeout -k 10 300 python3 -u bench.py --model aircond --bf 32,32,64 --no-cpu-baseline --check on > $O/air$k.log 2>&1 || { echo "air$k failed"; tail -5 $O/air$k.log; exit 1; }; grep '^{' $O/air$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("config4", d["value"], d["ms_per_step"], d.get("ms_per_step_median"), d["roofline"]["frac"], (d.get("checks") or {}).get("all_ok"))'; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof4 -o run -- python3 -u bench.py --model aircond --bf 32,32,64 --no-cpu-baseline > $O/prof4.log 2>&1; echo "prof rc=$?"
timeout -k 10 400 python3 -u bench.py > $O/bench.log 2>&1; echo "bench rc=$?"; grep '^{' $O/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["cpu_baseline"]["value"], (d.get("checks") or {}).get("all_ok"))'
MASTER_ADDR=127.0.0.1 MASTER_PORT=29563 timeout -k 10 300 python3 -u tools/fake_ranks.py 8 100 rccl > $O/rccl.log 2>&1; echo "rccl rc=$?"; grep -E "library" $O/rccl.log | cut -c1-110
echo done
