#!/bin/bash
# Round 3, pass n: path-6 variants on the GPU (env knobs, no code change): Mehrotra with the
# warm start (spills: threshold lifted), the warm start's first sigma, at 65,536 and 8,192.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    grep '^{' "gpurun_out/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']), d['ms_per_step'], d['solver_iters_per_ph_iter'], d['time_split_ms']['solve_launch'], d['roofline'].get('ipm'))" 2>/dev/null || tail -3 "gpurun_out/$name.log"
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 -u bench.py --no-cpu-baseline"
step n_base 300 $B
step n_meh 300 env PHGPU_IPM_MEHROTRA=1 PHGPU_IPM_SPILL_MAX=100000 $B
step n_a08 300 env PHGPU_IPM_DEFS="IPM_WARM_A0=0.8" $B
step n_a05 300 env PHGPU_IPM_DEFS="IPM_WARM_A0=0.5" $B
step n_s8192 300 $B --scens 8192
step n_s8192_a08 300 env PHGPU_IPM_DEFS="IPM_WARM_A0=0.8" $B --scens 8192
step n_s8192_l1 300 env PHGPU_IPM_LANES=1 $B --scens 8192
step n_s8192_l4 300 env PHGPU_IPM_LANES=4 $B --scens 8192
step n_s8192_l16 300 env PHGPU_IPM_LANES=16 $B --scens 8192
echo done
