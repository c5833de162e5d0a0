#!/bin/bash
# Round 6, pass g: kernel traces of one PH step (8,192 share one rank and loopback 8 ranks,
# config 3), the folded step in the lane-group kernel re-measured without the statistics
# queue, and the bench lines with per-iteration times.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6g
mkdir -p $O
export TMPDIR=/tmp
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "mean_ms", round(d["ms_per_step"],4), "median_ms", round(d["ms_per_step_median"],4), "launch", round(d["roofline"]["launch_ms"],4), d["solver_iters_per_ph_iter"], d["all_optimal"], (d.get("checks") or {}).get("all_ok"), d.get("iter_ms"))'
b() { n=$1; shift; timeout -k 10 300 python3 -u bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || { tail -20 $O/$n.log; exit $r; }; grep '^{' $O/$n.log | python3 -c "$S"; }
b s65536
b s8192 --scens 8192
PHGPU_FUSE_STEP=1 b s8192_fuse --scens 8192
b cm10 --scens 1024 --cm 10
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/t8192 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --scens 8192 --steps 10 > $GRAFT_REPO_ROOT/$O/t8192.log 2>&1 || { echo "trace 8192 failed"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/tfake -o run -- python3 $GRAFT_REPO_ROOT/tools/fake_ranks.py 8 20 > $GRAFT_REPO_ROOT/$O/tfake.log 2>&1 || { echo "trace fake failed"; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/t65536 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 10 > $GRAFT_REPO_ROOT/$O/t65536.log 2>&1 || { echo "trace 65536 failed"; exit 1; }
cd $GRAFT_REPO_ROOT
for t in t8192 tfake t65536; do f=$(find $O/$t -name "*kernel_trace.csv" | head -1); echo "== $t $f"; python3 tools/step_trace.py $f 2 | tail -14; done
tail -3 $O/tfake.log
echo done
