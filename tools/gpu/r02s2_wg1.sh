#!/bin/bash
# Round 2 (session 2): one-wave workgroups without the LDS drain / barrier (config 2), and
# the workgroup-path GPU tests.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -1 "gpurun_out/$name.log" | cut -c1-200
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 -u bench.py --no-cpu-baseline"
step w_cfg2 300 $B --scens 1024 --cm 10
step w_tests 600 python -u -m pytest tests/test_gpu_wg.py tests/test_gpu_scale.py -x -v --timeout 300 --timeout-method thread
step w_cm64 400 $B --cm 64 --steps 5 --warmup 2
echo done
