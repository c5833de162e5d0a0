#!/bin/bash
# Round 5, pass y: per-handle interior-point tuning (phgpu_set_ipm_tuning, the aircond
# example's IPM_TUNING): the config-4 tests with it, the bench line of config 4.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5y
mkdir -p $O
export TMPDIR=/tmp
step() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; tail -2 $O/$n.log; [ $r -eq 0 ] || exit $r; }
step tests 700 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_config4.py tests/test_lib_exports.py
step air 300 python3 -u bench.py --no-cpu-baseline --model aircond
grep '^{' $O/air.log > $O/air_line.json
echo done
