#!/bin/bash
# Round 6, closing pass 6 (the final build): the whole GPU suite, smoke, the default bench
# line with its CPU baseline, the 8,192 share, 2 gloo ranks, the RCCL loopback.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6z6
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/ > $O/gputests.log 2>&1; r=$?; echo "tests rc=$r"; grep -E "passed|failed" $O/gputests.log | tail -2; [ $r -eq 0 ] || { grep -E "FAILED|Error" $O/gputests.log | head; exit 1; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
timeout -k 10 400 python3 -u bench.py > $O/bench.log 2>&1; echo "bench rc=$?"; grep '^{' $O/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"].get("traffic"), d["cpu_baseline"]["value"], (d.get("checks") or {}).get("all_ok"))'
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --scens 8192 > $O/s8192.log 2>&1; echo "s8192 rc=$?"; grep '^{' $O/s8192.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("ms_per_step_median"))'
timeout -k 10 400 python3 -u bench.py --gpus 2 --backend gloo --steps 10 > $O/g2.log 2>&1; echo "gloo2 rc=$?"; grep '^{' $O/g2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], (d.get("checks") or {}).get("all_ok"))'
MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 timeout -k 10 400 python3 -u tools/fake_ranks.py 8 100 rccl > $O/rccl.log 2>&1; echo "rccl rc=$?"; grep -E "loopback" $O/rccl.log | cut -c1-110
timeout -k 10 300 python3 -u bench.py --model aircond --bf 32,32,64 --no-cpu-baseline --check on > $O/c4.log 2>&1; echo "config4 rc=$?"; grep '^{' $O/c4.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], (d.get("checks") or {}).get("all_ok"))'
echo done
