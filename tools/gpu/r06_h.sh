#!/bin/bash
# Round 6, pass h: A/B against the round-5 build (ab_r05/, not committed): config 2 and
# config 3, alternating, plus kernel traces (csv) of the current build.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6h
mkdir -p $O
export TMPDIR=/tmp
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "mean_ms", round(d.get("ms_per_step_mean", d["ms_per_step"]),4), "median", round(d.get("ms_per_step_median", d["ms_per_step"]),4), "launch", round(d["roofline"]["launch_ms"],4), d["solver_iters_per_ph_iter"])'
b() { n=$1; dir=$2; shift; shift; timeout -k 10 300 python3 -u $dir/bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || { tail -20 $O/$n.log; exit $r; }; grep '^{' $O/$n.log | python3 -c "$S"; }
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 800 --timeout-method thread -m gpu tests/test_gpu_uc.py -k "ph_subproblems" > $O/uc_test.log 2>&1; echo "uc test rc=$?"; tail -15 $O/uc_test.log
for rep in 1 2; do
  b cm10_old_$rep ab_r05 --scens 1024 --cm 10
  b cm10_new_$rep . --scens 1024 --cm 10
  b s65536_old_$rep ab_r05
  b s65536_new_$rep .
done
cd /tmp
for t in 8192 65536; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/t$t -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --scens $t --steps 10 > $GRAFT_REPO_ROOT/$O/t$t.log 2>&1 || { echo "trace $t failed"; exit 1; }
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/tfake -o run -- python3 $GRAFT_REPO_ROOT/tools/fake_ranks.py 8 20 > $GRAFT_REPO_ROOT/$O/tfake.log 2>&1 || { echo "trace fake failed"; exit 1; }
cd $GRAFT_REPO_ROOT
for t in t8192 tfake t65536; do f=$(find $O/$t -name "*kernel_trace.csv" | head -1); echo "== $t $f"; [ -n "$f" ] && python3 tools/step_trace.py $f 2 | tail -14; done
tail -3 $O/tfake.log
echo done
