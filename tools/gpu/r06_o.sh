#!/bin/bash
# Round 6, pass o: where the 8,192 share's lane-group iteration goes (IPM_PROF wave timelines,
# per-phase shader cycles), the one-lane timeline at 65,536, the loopback multi-rank step.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6o
mkdir -p $O
export TMPDIR=/tmp
p() { n=$1; shift; timeout -k 10 200 python3 -u tools/ipm_prof.py "$@" > $O/$n.log 2>&1; r=$?; [ $r -eq 0 ] || { echo "$n rc=$r"; tail -20 $O/$n.log; exit $r; }; echo "== $n"; tail -1 $O/$n.log; }
p l8_off 8192 8 --prof 0
p l8 8192 8
p l8_lv2 8192 8 --level 2
p l1 65536 1
timeout -k 10 300 python3 -u tools/fake_ranks.py 8 40 > $O/fake8.log 2>&1 && tail -4 $O/fake8.log
echo done
