#!/bin/bash
# Round 5, pass q: the whole GPU suite, smoke() and the default bench after the multi-rank step changes
# (after variable probabilities, the solve hooks and the speculation rule for extensions).
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5q
mkdir -p $O
export TMPDIR=/tmp
step() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; tail -2 $O/$n.log; [ $r -eq 0 ] || exit $r; }
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gputests.log 2>&1
r=$?; echo "pytest rc=$r"; tail -4 $O/gputests.log; [ $r -eq 0 ] || exit $r
step smoke 200 python3 -u -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python3 -u bench.py
echo done
