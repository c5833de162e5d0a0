#!/bin/bash
# Round 3, pass w: one rank folds x̄ into the update launch (phgpu_ph_step_local).
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    grep '^{' "gpurun_out/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4), d.get('solver_iters_per_ph_iter'), d['time_split_ms'], d['all_optimal'])" 2>/dev/null || tail -3 "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 -u bench.py --no-cpu-baseline"
T="python -u -m pytest -v --timeout 600 --timeout-method thread"
step w_new 600 $T -x -m gpu tests/test_gpu_readback.py
step w_gputests 1200 $T -m gpu tests
step w_bench 300 $B
step w_bench2 300 $B
step w_s8192 300 $B --scens 8192
step w_s8192b 300 $B --scens 8192
step w_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/w_trace -o run -- python3 bench.py --no-cpu-baseline
echo done
