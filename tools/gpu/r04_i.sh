#!/bin/bash
# Round 4, pass i: the retry with per-attempt accumulators -- config 2 (tests, diagnostic on
# scen0..1023, bench), cm = 64 diagnostic.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    grep '^{' "gpurun_out/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4), round(d['time_split_ms']['solve_launch'],4), d['solver_iters_per_ph_iter'], d['all_optimal'], d['roofline']['kernel'])" 2>/dev/null || grep -v "^    scen" "gpurun_out/$name.log" | tail -8 | cut -c1-250
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
T="python3 -u -m pytest -m gpu -v --timeout 100 --timeout-method thread"
step i_par 200 $T tests/test_gpu_scale.py::test_config2_farmer1024_cm10_bound tests/test_gpu_scale.py::test_config2_ph_iterations_to_convergence tests/test_gpu_parity.py::test_farmer_cm10_parity
DIAG_DUMP=gpurun_out/i_w10 step i_d10 100 python3 -u tests/diag_ipm_cm64.py 8 1024 first 10
step i_cfg2 150 python3 -u bench.py --no-cpu-baseline --scens 1024 --cm 10
DIAG_DUMP=gpurun_out/i_w64 step i_d64 120 python3 -u tests/diag_ipm_cm64.py 6 2048 first 64
echo done
