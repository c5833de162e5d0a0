#!/bin/bash
# Round 5, pass l: the multi-rank step path's own cost at the 8,192 and 32,768 shares
# (tools/fake_ranks.py: loopback communicator, no RCCL) against the folded one-rank step.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5l
mkdir -p $O
export TMPDIR=/tmp
step() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; tail -3 $O/$n.log; [ $r -eq 0 ] || exit $r; }
step fake8 300 python3 -u tools/fake_ranks.py 8 40
step fake2 300 python3 -u tools/fake_ranks.py 2 40
echo done
