#!/bin/bash
# Round 3, pass o: sigma range [0.01, 0.05] -- GPU tests, then the warm start's first sigma.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    grep '^{' "gpurun_out/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), d['ms_per_step'], d['solver_iters_per_ph_iter'], d['time_split_ms']['solve_launch'], d['all_optimal'])" 2>/dev/null || tail -3 "gpurun_out/$name.log"
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 -u bench.py --no-cpu-baseline"
T="python -u -m pytest -v -x --timeout 300 --timeout-method thread"
step o_tests 1200 $T -m gpu tests/test_gpu_ipm.py tests/test_gpu_readback.py tests/test_gpu_speculative.py tests/test_gpu_convergence.py tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_xhat_eval.py tests/test_dist_engine.py tests/test_gpu_config4.py
step o_base 300 $B
step o_a08 300 env PHGPU_IPM_DEFS="IPM_WARM_A0=0.8" $B
step o_s8192 300 $B --scens 8192
step o_s8192_a08 300 env PHGPU_IPM_DEFS="IPM_WARM_A0=0.8" $B --scens 8192
step o_air8192 300 $B --model aircond --bf 4,32,64
step o_air8192_a08 300 env PHGPU_IPM_DEFS="IPM_WARM_A0=0.8" $B --model aircond --bf 4,32,64
echo done
