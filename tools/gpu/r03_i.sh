#!/bin/bash
# Round 3, pass i: path-6 lane groups (k_solve_ipm_ml) -- tests, the bench
# (config 3 and the N=8 share) and a kernel trace of the default bench.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -3 "gpurun_out/$name.log" | cut -c1-600
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 -u bench.py --no-cpu-baseline"
T="python -u -m pytest -v --timeout 600 --timeout-method thread"
step i_tests 900 $T tests/test_gpu_ipm.py
step i_bench 300 $B
step i_bench_s8192 300 $B --scens 8192
PHGPU_IPM_LANES=4 step i_bench_s8192_L4 300 $B --scens 8192
PHGPU_IPM_LANES=16 step i_bench_s8192_L16 300 $B --scens 8192
step i_bench_s16384 300 $B --scens 16384
step i_bench_s32768 300 $B --scens 32768
echo done
