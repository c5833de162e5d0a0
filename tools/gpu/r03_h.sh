#!/bin/bash
# Round 3, pass h: solve statistics in the path-6 kernels -- path-6 tests, the bench
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
step h_tests 900 $T tests/test_gpu_ipm.py tests/test_gpu_speculative.py tests/test_gpu_parity.py
step h_bench 300 $B
step h_bench_s8192 300 $B --scens 8192
step h_prof 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/h_prof -o run -- python3 bench.py --no-cpu-baseline
echo done
