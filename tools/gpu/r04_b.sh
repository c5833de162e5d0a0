#!/bin/bash
# Round 4, pass b: the folded step with the engine fix; the workgroup IPM at cm = 64 (four
# waves per scenario) under short limits.
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
T="python3 -u -m pytest -m gpu -v --timeout 100 --timeout-method thread"
step b_fold 200 $T -x tests/test_gpu_speculative.py -k folded
step b_wg64 150 $T -x tests/test_gpu_wg.py -k "cm64 and 1"
step b_cm64s 150 python3 -u bench.py --no-cpu-baseline --cm 64 --scens 2048 --steps 5 --warmup 2
echo done
