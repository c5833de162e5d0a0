#!/bin/bash
# Round 3, pass g: path 6 fixes -- its tests, the tests that failed in pass f, the bench
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
step g_tests 900 $T tests/test_gpu_ipm.py tests/test_xhat_eval.py "tests/test_gpu_scale.py::test_iter0_raises_on_an_infeasible_scenario"
step g_bench 300 $B
step g_bench_s8192 300 $B --scens 8192
step g_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/g_prof -o run -- python3 bench.py --no-cpu-baseline
echo done
