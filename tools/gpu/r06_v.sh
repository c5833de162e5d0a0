#!/bin/bash
# Round 6, pass v: the multi-rank step (loopback, 8 ranks at the 8,192 share): its kernel
# trace and its host profile.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6v
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
FAKE_PROF=1 timeout -k 10 300 python3 -u tools/fake_ranks.py 8 200 loopback > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
grep -v "^$" $O/prof.log | head -50
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/tfake -o run -- python3 $R/tools/fake_ranks.py 8 20 loopback > $R/$O/tfake.log 2>&1 || { echo "trace failed"; exit 1; }
cd $R
f=$(find $O/tfake -name "*kernel_trace.csv" | head -1); python3 tools/step_trace.py $f 2 | tail -20
echo done
