#!/bin/bash
# Round 6, pass aa: the update kernels' statistics loads moved ahead of the conv exchange /
# ticket chain: the tests that read the statistics, bench lines, loopback.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6aa
mkdir -p $O
export TMPDIR=/tmp
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "mean_ms", round(d.get("ms_per_step_mean", d["ms_per_step"]),4), "median", round(d.get("ms_per_step_median", d["ms_per_step"]),4), "launch", round(d["roofline"]["launch_ms"],4), (d.get("checks") or {}).get("all_ok"))'
b() { n=$1; shift; timeout -k 10 300 python3 -u bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || { tail -20 $O/$n.log; exit $r; }; grep '^{' $O/$n.log | python3 -c "$S"; }
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_readback.py tests/test_gpu_speculative.py tests/test_gpu_loopback.py tests/test_gpu_ipm.py tests/test_variable_probability.py > $O/tests.log 2>&1; r=$?; echo "tests rc=$r"; tail -1 $O/tests.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit 1; }
for rep in 1 2; do b s8192_$rep --scens 8192; b s65536_$rep; done
b cfg2 --scens 1024 --cm 10
timeout -k 10 300 python3 -u tools/fake_ranks.py 8 100 > $O/fake8.log 2>&1 && grep -E "loopback|one rank" $O/fake8.log | cut -c1-120
echo done
