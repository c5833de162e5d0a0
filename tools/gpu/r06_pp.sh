#!/bin/bash
# Round 6, pass pp: the one-launch local PH step for 30 nonants (config 2), its operands loaded together: readback / config-2
# tests, config 2 lines and trace, the default line.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6pp
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_readback.py tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_speculative.py tests/test_gpu_wg.py > $O/tests.log 2>&1; r=$?; echo "tests rc=$r"; tail -1 $O/tests.log; [ $r -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit 1; }
for k in 1 2; do timeout -k 10 300 python3 -u bench.py --scens 1024 --cm 10 --no-cpu-baseline --check on > $O/c2_$k.log 2>&1 || { echo "c2 $k failed"; tail -5 $O/c2_$k.log; exit 1; }; grep '^{' $O/c2_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("config2", d["value"], d["ms_per_step"], d.get("ms_per_step_median"), (d.get("checks") or {}).get("all_ok"))'; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2 -o run -- python3 -u bench.py --scens 1024 --cm 10 --no-cpu-baseline > $O/prof2.log 2>&1; echo "prof rc=$?"
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $O/bench.log 2>&1; echo "bench rc=$?"; grep '^{' $O/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], (d.get("checks") or {}).get("all_ok"))'
echo done
