#!/bin/bash
# Round 6, pass r: the one-lane kernel's scenario data loaded ahead of the folded PH step:
# tests, bench lines, prologue timeline, trace.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6r
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "mean_ms", round(d.get("ms_per_step_mean", d["ms_per_step"]),4), "median", round(d.get("ms_per_step_median", d["ms_per_step"]),4), "launch", round(d["roofline"]["launch_ms"],4), d["roofline"]["frac"], d["solver_iters_per_ph_iter"], (d.get("checks") or {}).get("all_ok"))'
b() { n=$1; shift; timeout -k 10 300 python3 -u bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || { tail -20 $O/$n.log; exit $r; }; grep '^{' $O/$n.log | python3 -c "$S"; }
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_readback.py tests/test_gpu_speculative.py tests/test_gpu_convergence.py tests/test_gpu_ipm.py tests/test_gpu_fused_loop.py tests/test_gpu_config4.py > $O/tests.log 2>&1; r=$?; echo "tests rc=$r"; tail -2 $O/tests.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit 1; }
b s65536
b s65536_b
b air --model aircond
timeout -k 10 200 python3 -u tools/ipm_prof.py 65536 1 > $O/l1.log 2>&1 && tail -1 $O/l1.log
echo done
