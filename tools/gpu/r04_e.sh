#!/bin/bash
# Round 4, pass e: config 2 on the subtree kernel (fixtures, convergence count, parity), the
# folded step at 40,000 scenarios, and the cm = 64 bench with a progress file.
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
step e_cfg2 300 $T tests/test_gpu_scale.py -k config2 tests/test_gpu_parity.py::test_farmer_cm10_parity
step e_fold 200 $T tests/test_gpu_speculative.py -k "folded and 40000"
step e_cm64b 170 python3 -u bench.py --no-cpu-baseline --cm 64 --scens 2048 --steps 10 --warmup 3
echo done
