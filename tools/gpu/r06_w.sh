#!/bin/bash
# Round 6, pass w: the multi-rank conv readback polled instead of waited on: loopback /
# one-rank step times, the multi-rank tests, the loopback trace.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6w
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_loopback.py tests/test_gpu_dist_scale.py > $O/tests.log 2>&1; r=$?; echo "tests rc=$r"; tail -1 $O/tests.log; [ $r -eq 0 ] || { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit 1; }
timeout -k 10 300 python3 -u tools/fake_ranks.py 8 100 > $O/fake8.log 2>&1 && grep -E "loopback|one rank" $O/fake8.log
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/tfake -o run -- python3 $R/tools/fake_ranks.py 8 20 loopback > $R/$O/tfake.log 2>&1 || { echo "trace failed"; exit 1; }
cd $R
f=$(find $O/tfake -name "*kernel_trace.csv" | head -1); python3 tools/step_trace.py $f 2 | tail -10
timeout -k 10 400 python3 -u bench.py --gpus 2 --backend gloo --steps 10 > $O/g2.log 2>&1; echo "gloo2 rc=$?"; grep '^{' $O/g2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], (d.get("checks") or {}))'
echo done
