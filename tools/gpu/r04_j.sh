#!/bin/bash
# Round 4, pass j: re-centring + cold retry; multi-wave IPMs opt-in -- GPU tests of path 6
# for medium scenarios, config 2 diagnostic and bench, cm = 64 on the automatic path.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    grep '^{' "gpurun_out/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4), round(d['time_split_ms']['solve_launch'],4), d['solver_iters_per_ph_iter'], d['all_optimal'], d['roofline']['kernel'])" 2>/dev/null || grep -v "^    scen" "gpurun_out/$name.log" | tail -9 | cut -c1-250
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
T="python3 -u -m pytest -m gpu -v --timeout 100 --timeout-method thread"
step j_par 400 $T tests/test_gpu_scale.py::test_config2_farmer1024_cm10_bound tests/test_gpu_scale.py::test_config2_ph_iterations_to_convergence tests/test_gpu_parity.py::test_farmer_cm10_parity tests/test_gpu_wg.py tests/test_gpu_ipm_wave.py
DIAG_DUMP=gpurun_out/j_w10 step j_d10 100 python3 -u tests/diag_ipm_cm64.py 8 1024 first 10
step j_cfg2 150 python3 -u bench.py --no-cpu-baseline --scens 1024 --cm 10
echo done
