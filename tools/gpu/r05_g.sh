#!/bin/bash
# Round 5, pass g: variable probabilities on the GPU, the reduction / readback tests and the
# 2-rank engine test (the step's generic path), the default bench.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5g
mkdir -p $O
export TMPDIR=/tmp
step() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; tail -2 $O/$n.log; [ $r -eq 0 ] || exit $r; }
step tests 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_variable_probability.py tests/test_gpu_readback.py tests/test_dist_engine.py tests/test_gpu_speculative.py
step bench 300 python3 -u bench.py --no-cpu-baseline
echo done
