#!/bin/bash
# Round 5, pass w: config 5 with the final recommended PH-solve options (beta_sufficient 0.7,
# KKT every 128): the UC tests and the bench line as the bench runs it.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5w
mkdir -p $O
export TMPDIR=/tmp
step() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; tail -2 $O/$n.log; [ $r -eq 0 ] || exit $r; }
step tests 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_uc.py -k "ph_iterations or lp_relaxation"
step uc 420 python3 -u bench.py --no-cpu-baseline --model uc --steps 2 --warmup 1
grep '^{' $O/uc.log > $O/uc_line.json
echo done
