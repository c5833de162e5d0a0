#!/bin/bash
# Round 4, pass a: the folded PH step and the workgroup interior point -- their GPU tests,
# then the bench lines they change (config 3, the 8,192 share, config 2, cm = 64, config 4).
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    grep '^{' "gpurun_out/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4), round(d['time_split_ms']['solve_launch'],4), d['solver_iters_per_ph_iter'], d['all_optimal'])" 2>/dev/null || tail -4 "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
T="python3 -u -m pytest -m gpu -v --timeout 200 --timeout-method thread"
step a_wave 300 $T tests/test_gpu_ipm_wave.py
step a_fold 400 $T -x tests/test_gpu_speculative.py tests/test_gpu_readback.py tests/test_dist_engine.py
B="python3 -u bench.py --no-cpu-baseline"
step a_cfg3 300 $B
step a_s8192 300 $B --scens 8192
step a_cfg2 300 $B --scens 1024 --cm 10
step a_cm64 600 $B --cm 64 --steps 5 --warmup 2
step a_air 300 $B --model aircond
echo done
