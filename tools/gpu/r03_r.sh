#!/bin/bash
# Round 3, pass r: config 4 (aircond 65,536) on the phased lane-group IPM kernel.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    grep '^{' "gpurun_out/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4), d.get('solver'), d.get('solver_iters_per_ph_iter'), round(d['time_split_ms']['solve_launch'],4), d['roofline'].get('lanes_per_scenario'), d['all_optimal'])" 2>/dev/null || tail -2 "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 -u bench.py --no-cpu-baseline --model aircond"
for L in 4 8 16; do step r_air_l$L 300 env PHGPU_IPM_LANES=$L $B; done
step r_air32k_l4 300 env PHGPU_IPM_LANES=4 $B --bf 16,32,64
step r_air32k_l8 300 env PHGPU_IPM_LANES=8 $B --bf 16,32,64
step r_farmer_l4 300 env PHGPU_IPM_LANES=4 python3 -u bench.py --no-cpu-baseline
echo done
