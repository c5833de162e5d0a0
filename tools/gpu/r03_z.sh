#!/bin/bash
# Round 3, pass z: A/B of the fallback launch's grid (its dispatch costs even when empty).
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    grep '^{' "gpurun_out/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4), round(d['time_split_ms']['solve_launch'],4), d['all_optimal'])" 2>/dev/null || tail -3 "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 -u bench.py --no-cpu-baseline --steps 40"
for rep in 1 2; do
  for fb in 16 4 1; do
    step z_fb${fb}_$rep 300 env PHGPU_IPM_FB_BLOCKS=$fb $B
    step z_s8192_fb${fb}_$rep 300 env PHGPU_IPM_FB_BLOCKS=$fb $B --scens 8192
  done
done
step z_fail1 300 env PHGPU_IPM_FB_BLOCKS=1 PHGPU_IPM_MAXIT=3 python3 -u bench.py --no-cpu-baseline --scens 8192 --steps 3 --warmup 1
echo done
