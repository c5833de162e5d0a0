#!/bin/bash
# Round 6, pass f: path-6 statistics spread over 32 copies (no same-line atomic queue at the
# end of the launch): the tests that read the statistics, then every share / config.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6f
mkdir -p $O
export TMPDIR=/tmp
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "mean_ms", round(d["ms_per_step"],4), "median_ms", round(d["ms_per_step_median"],4), "launch", round(d["roofline"]["launch_ms"],4), d["solver_iters_per_ph_iter"], d["all_optimal"], (d.get("checks") or {}).get("all_ok"))'
b() { n=$1; shift; timeout -k 10 300 python3 -u bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || { tail -20 $O/$n.log; exit $r; }; grep '^{' $O/$n.log | python3 -c "$S"; }
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ipm.py tests/test_gpu_readback.py tests/test_gpu_speculative.py tests/test_gpu_ipm_wave.py tests/test_gpu_loopback.py tests/test_variable_probability.py > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
b s65536
b s32768 --scens 32768
b s16384 --scens 16384
b s8192 --scens 8192
b cm10 --scens 1024 --cm 10
b air --model aircond
timeout -k 10 200 python3 -u tools/ipm_prof.py 8192 8 > $O/prof_l8.log 2>&1 && tail -1 $O/prof_l8.log
timeout -k 10 200 python3 -u tools/ipm_prof.py 65536 1 > $O/prof_l1.log 2>&1 && tail -1 $O/prof_l1.log
echo done
