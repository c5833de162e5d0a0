#!/bin/bash
# Round 6, pass q: the PH step's latency chain (the folded step's partial loads in flight
# together, the scenario's W / rho / x loaded ahead of the x̄ sums, likewise in
# k_ph_update_local): tests, prologue timelines, traces, bench lines (8,192 share with the
# step folded into the lane-group kernel as the A/B).
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6q
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "mean_ms", round(d.get("ms_per_step_mean", d["ms_per_step"]),4), "median", round(d.get("ms_per_step_median", d["ms_per_step"]),4), "launch", round(d["roofline"]["launch_ms"],4), d["roofline"]["frac"], d["solver_iters_per_ph_iter"], (d.get("checks") or {}).get("all_ok"))'
b() { n=$1; shift; timeout -k 10 300 python3 -u bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || { tail -20 $O/$n.log; exit $r; }; grep '^{' $O/$n.log | python3 -c "$S"; }
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_readback.py tests/test_gpu_speculative.py tests/test_gpu_convergence.py tests/test_gpu_loopback.py tests/test_variable_probability.py > $O/tests.log 2>&1; r=$?; echo "tests rc=$r"; tail -2 $O/tests.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit 1; }
b s65536
b s8192 --scens 8192
PHGPU_FUSE_STEP=1 b s8192_fold --scens 8192
b cm10 --scens 1024 --cm 10
timeout -k 10 200 python3 -u tools/ipm_prof.py 65536 1 > $O/l1.log 2>&1 && tail -1 $O/l1.log
cd /tmp
for t in 8192 65536; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/t$t -o run -- python3 $R/bench.py --no-cpu-baseline --scens $t --steps 10 > $R/$O/t$t.log 2>&1 || { echo "trace $t failed"; exit 1; }
done
cd $R
for t in t8192 t65536; do f=$(find $O/$t -name "*kernel_trace.csv" | head -1); echo "== $t"; python3 tools/step_trace.py $f 2 | tail -8; done
echo done
