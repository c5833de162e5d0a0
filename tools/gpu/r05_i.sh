#!/bin/bash
# Round 5, pass i: the per-scenario solve hooks and the W / x̄ writer-reader extensions (the
# writer now keeps the speculative solve).
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5i
mkdir -p $O
export TMPDIR=/tmp
step() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; tail -2 $O/$n.log; [ $r -eq 0 ] || exit $r; }
step tests 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_solve_hooks.py tests/test_wxbar.py
echo done
