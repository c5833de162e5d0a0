#!/bin/bash
# Round 3, pass d: path 5 (hipRTC pattern-specialised kernel) -- parity tests, then the
# bench on it against the default path (config 3, config 4, the N=8 share).
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -2 "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 bench.py --no-cpu-baseline"
T="python -u -m pytest -v --timeout 600 --timeout-method thread"
step d_jittests 600 $T tests/test_gpu_jit.py
step d_bench_def 300 $B
PHGPU_JIT=1 step d_bench_jit 300 $B
step d_bench_air_def 300 $B --model aircond
PHGPU_JIT=1 step d_bench_air_jit 300 $B --model aircond
step d_bench_s8192_def 300 $B --scens 8192
PHGPU_JIT=1 step d_bench_s8192_jit 300 $B --scens 8192
echo done
