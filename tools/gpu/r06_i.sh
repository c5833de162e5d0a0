#!/bin/bash
# Round 6, pass i: wave-parallel statistics reads in the update kernels (the serial read of
# 32 copies took 8-10 us); A/B against round 5 on config 2 and the 8,192 share; UC PH test.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6i
mkdir -p $O
export TMPDIR=/tmp
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "mean_ms", round(d.get("ms_per_step_mean", d["ms_per_step"]),4), "median", round(d.get("ms_per_step_median", d["ms_per_step"]),4), "launch", round(d["roofline"]["launch_ms"],4), d["solver_iters_per_ph_iter"])'
b() { n=$1; dir=$2; shift; shift; timeout -k 10 300 python3 -u $dir/bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || { tail -20 $O/$n.log; exit $r; }; grep '^{' $O/$n.log | python3 -c "$S"; }
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 800 --timeout-method thread -m gpu tests/test_gpu_readback.py tests/test_gpu_loopback.py tests/test_gpu_speculative.py > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  b cm10_old_$rep ab_r05 --scens 1024 --cm 10
  b cm10_new_$rep . --scens 1024 --cm 10
  b s8192_old_$rep ab_r05 --scens 8192
  b s8192_new_$rep . --scens 8192
done
b s65536_new . 
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/tfake -o run -- python3 $GRAFT_REPO_ROOT/tools/fake_ranks.py 8 20 > $GRAFT_REPO_ROOT/$O/tfake.log 2>&1 || { echo "trace fake failed"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/tcm10 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --scens 1024 --cm 10 --steps 10 > $GRAFT_REPO_ROOT/$O/tcm10.log 2>&1 || { echo "trace cm10 failed"; exit 1; }
cd $GRAFT_REPO_ROOT
for t in tfake tcm10; do f=$(find $O/$t -name "*kernel_trace.csv" | head -1); echo "== $t"; python3 tools/step_trace.py $f 2 | tail -12; done
tail -2 $O/tfake.log
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 900 --timeout-method thread -m gpu tests/test_gpu_uc.py -k "ph_subproblems" > $O/uc_test.log 2>&1; echo "uc test rc=$?"; grep -E "passed|failed|Error|assert" $O/uc_test.log | head -8
echo done
