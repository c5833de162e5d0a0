#!/bin/bash
# Round 3, pass u: A/B of compile-time knobs of the IPM modules (no code change): the KKT
# gate and the scheduler strategy.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    grep '^{' "gpurun_out/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4), d.get('solver_iters_per_ph_iter'), round(d['time_split_ms']['solve_launch'],4), d['all_optimal'])" 2>/dev/null || tail -3 "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 -u bench.py --no-cpu-baseline --steps 40"
for rep in 1 2; do
  step u_base_$rep 300 $B
  step u_gate3_$rep 300 env PHGPU_IPM_DEFS="IPM_KKT_GATE=3" $B
  step u_ilp_$rep 300 env PHGPU_JIT_OPTS="-mllvm -amdgpu-sched-strategy=max-ilp" $B
  step u_s8192_base_$rep 300 $B --scens 8192
  step u_s8192_gate3_$rep 300 env PHGPU_IPM_DEFS="IPM_KKT_GATE=3" $B --scens 8192
  step u_s8192_ilp_$rep 300 env PHGPU_JIT_OPTS="-mllvm -amdgpu-sched-strategy=max-ilp" $B --scens 8192
done
echo done
