#!/bin/bash
# Round 5, pass r: the loopback multi-rank tests (one process, the multi-rank step path
# against the folded one-rank step).
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5r
mkdir -p $O
export TMPDIR=/tmp
step() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; tail -3 $O/$n.log; [ $r -eq 0 ] || exit $r; }
step tests 500 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_loopback.py
echo done
