#!/bin/bash
# Round 3, pass l: one event marker per PH step (shared with the bench's solve-start event).
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -3 "gpurun_out/$name.log" | cut -c1-400
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 -u bench.py --no-cpu-baseline"
T="python -u -m pytest -v -x --timeout 300 --timeout-method thread"
step l_tests 900 $T -m gpu tests/test_gpu_readback.py tests/test_gpu_speculative.py tests/test_gpu_convergence.py tests/test_dist_engine.py tests/test_xhat_eval.py
step l_bench 300 $B
step l_s8192 300 $B --scens 8192
step l_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/l_trace -o run -- python3 bench.py --no-cpu-baseline
echo done
