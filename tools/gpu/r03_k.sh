#!/bin/bash
# Round 3, pass k: copy-free readbacks (x̄ clear in the partial kernel, conv and the
# solve statistics written to pinned host memory by the update kernel), aircond back on
# path 2, and the per-step trace.
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
T="python -u -m pytest -v -x --timeout 300 --timeout-method thread"
step k_tests 900 $T -m gpu tests/test_gpu_readback.py tests/test_gpu_speculative.py tests/test_gpu_convergence.py tests/test_dist_engine.py tests/test_gpu_parity.py tests/test_gpu_config4.py
step k_bench 300 $B
step k_s8192 300 $B --scens 8192
step k_air 300 $B --model aircond
step k_air8192 300 $B --model aircond --bf 4,32,64
step k_air8192_p2 300 env PHGPU_IPM=0 $B --model aircond --bf 4,32,64
step k_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/k_trace -o run -- python3 bench.py --no-cpu-baseline
step k_trace8192 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/k_trace8192 -o run -- python3 bench.py --no-cpu-baseline --scens 8192
echo done
