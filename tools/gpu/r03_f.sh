#!/bin/bash
# Round 3, pass f: path 6 (interior point) -- its parity tests, the bench on it vs the
# register path, the N=8 share, aircond, the convergence test, then the whole GPU suite.
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
step f_ipmtests 900 $T -x tests/test_gpu_ipm.py
step f_bench 300 $B
PHGPU_IPM=0 step f_bench_reg 300 $B
step f_bench_s8192 300 $B --scens 8192
step f_bench_air 300 $B --model aircond
step f_conv 900 $T tests/test_gpu_convergence.py tests/test_gpu_speculative.py
step f_gputests 1200 $T -m gpu tests
echo done
