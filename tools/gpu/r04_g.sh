#!/bin/bash
# Round 4, pass g: the subtree kernel with slack iterates, one-row root and retry -- config 2
# and cm = 64 parity, the cm = 64 diagnostic on scen0.., benches.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    grep '^{' "gpurun_out/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4), round(d['time_split_ms']['solve_launch'],4), d['solver_iters_per_ph_iter'], d['all_optimal'], d['roofline']['kernel'])" 2>/dev/null || tail -5 "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
T="python3 -u -m pytest -m gpu -v --timeout 100 --timeout-method thread"
step g_par 300 $T tests/test_gpu_scale.py::test_config2_farmer1024_cm10_bound tests/test_gpu_scale.py::test_config2_ph_iterations_to_convergence tests/test_gpu_parity.py::test_farmer_cm10_parity tests/test_gpu_wg.py::test_farmer_cm64_parity tests/test_gpu_ipm_wave.py
DIAG_DUMP=gpurun_out/g_worst step g_diag 120 python3 -u tests/diag_ipm_cm64.py 6 2048 first
B="python3 -u bench.py --no-cpu-baseline"
step g_cfg2 150 $B --scens 1024 --cm 10
step g_cm64a 150 $B --cm 64 --scens 2048 --steps 10 --warmup 3
step g_cm64b 200 $B --cm 64 --scens 8192 --steps 10 --warmup 3
step g_cfg3 150 $B
echo done
