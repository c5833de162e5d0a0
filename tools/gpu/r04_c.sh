#!/bin/bash
# Round 4, pass c: the subtree interior point (jit_ipm_blk.hip.in) -- its GPU tests, the
# folded step, then config 2 and cm = 64 shares.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    grep '^{' "gpurun_out/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4), round(d['time_split_ms']['solve_launch'],4), d['solver_iters_per_ph_iter'], d['all_optimal'], d['roofline']['kernel'])" 2>/dev/null || tail -3 "gpurun_out/$name.log" | cut -c1-400
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
T="python3 -u -m pytest -m gpu -v --timeout 100 --timeout-method thread"
step c_blk 200 $T -x tests/test_gpu_ipm_wave.py
step c_fold 200 $T -x tests/test_gpu_speculative.py -k folded
step c_wg64 200 $T -x tests/test_gpu_wg.py -k "cm64 and blk"
B="python3 -u bench.py --no-cpu-baseline"
step c_cfg2 200 $B --scens 1024 --cm 10
step c_cm64s 200 $B --cm 64 --scens 2048 --steps 10 --warmup 3
step c_cm64m 200 $B --cm 64 --scens 16384 --steps 10 --warmup 3
echo done
