#!/bin/bash
# Round 3, pass p: lane-group kernel in load / iterate / store phases (no queue): GPU tests,
# lane sweeps at the per-rank shares.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    grep '^{' "gpurun_out/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), round(d['ms_per_step'],4), d['solver_iters_per_ph_iter'], round(d['time_split_ms']['solve_launch'],4), d['roofline']['lanes_per_scenario'], d['all_optimal'])" 2>/dev/null || tail -3 "gpurun_out/$name.log"
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 -u bench.py --no-cpu-baseline"
T="python -u -m pytest -v -x --timeout 300 --timeout-method thread"
step p_tests 900 $T -m gpu tests/test_gpu_ipm.py tests/test_gpu_config4.py tests/test_gpu_readback.py
for L in 8 4 16 2; do step p_s8192_l$L 300 env PHGPU_IPM_LANES=$L $B --scens 8192; done
for L in 1 4 8; do step p_s16384_l$L 300 env PHGPU_IPM_LANES=$L $B --scens 16384; done
for L in 1 2 4; do step p_s32768_l$L 300 env PHGPU_IPM_LANES=$L $B --scens 32768; done
for L in 1 2; do step p_s65536_l$L 300 env PHGPU_IPM_LANES=$L $B; done
step p_air8192 300 $B --model aircond --bf 4,32,64
step p_air16384_l4 300 env PHGPU_IPM_LANES=4 $B --model aircond --bf 8,32,64
step p_air16384_l8 300 env PHGPU_IPM_LANES=8 $B --model aircond --bf 8,32,64
echo done
