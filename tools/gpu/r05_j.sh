#!/bin/bash
# Round 5, pass j: path 4's two-slice form (PHGPU_STREAM_PAIR=1): the path-4 tests with the
# bitwise pair-vs-single check, then config 5 alternating the two forms on one PH trajectory.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5j
mkdir -p $O
export TMPDIR=/tmp
step() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; tail -2 $O/$n.log; [ $r -eq 0 ] || exit $r; }
step tests 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_uc.py
step slots 900 python3 -u tools/uc_slots.py '[{}, {"PAIR": 1}, {}, {"PAIR": 1}]'
cp gpurun_out/uc_slots.npz $O/ 2>/dev/null
grep '^{' $O/slots.log
echo done
