#!/bin/bash
# Round 6, pass ii: the automatic LDS slack reciprocals (config 4): the aircond GPU tests, the
# config-4 bench line (self-checked) and its kernel trace, the default line.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6ii
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_config4.py tests/test_gpu_ipm.py tests/test_gpu_parity.py > $O/tests.log 2>&1; r=$?; echo "tests rc=$r"; tail -1 $O/tests.log; [ $r -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit 1; }
for k in 1 2; do timeout -k 10 300 python3 -u bench.py --model aircond --bf 32,32,64 --no-cpu-baseline --check on > $O/air$k.log 2>&1 || { echo "air$k failed"; tail -5 $O/air$k.log; exit 1; }; grep '^{' $O/air$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("config4", d["value"], d["ms_per_step"], d.get("ms_per_step_median"), d["roofline"]["frac"], (d.get("checks") or {}).get("all_ok"))'; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_air -o air -- python3 -u bench.py --model aircond --bf 32,32,64 --no-cpu-baseline --steps 10 > $O/air_prof.log 2>&1; echo "prof rc=$?"
timeout -k 10 400 python3 -u bench.py > $O/bench.log 2>&1; echo "bench rc=$?"; grep '^{' $O/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["cpu_baseline"]["value"], (d.get("checks") or {}).get("all_ok"))'
echo done
