#!/bin/bash
# Round 4, pass f: the subtree kernel with slack iterates -- config 2 fixtures, cm = 64
# fixture parity, the cm = 64 diagnostic on scen0.. (ties, near-ties), config-2 bench.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -6 "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
T="python3 -u -m pytest -m gpu -v --timeout 100 --timeout-method thread"
step f_cfg2 300 $T tests/test_gpu_scale.py::test_config2_farmer1024_cm10_bound tests/test_gpu_scale.py::test_config2_ph_iterations_to_convergence tests/test_gpu_parity.py::test_farmer_cm10_parity tests/test_gpu_wg.py::test_farmer_cm64_parity
step f_diag 150 python3 -u tests/diag_ipm_cm64.py 6 2048 first
step f_bcfg2 150 python3 -u bench.py --no-cpu-baseline --scens 1024 --cm 10
echo done
