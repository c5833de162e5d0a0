#!/bin/bash
# Round 4, pass r: farmer cm = 64 on its automatic path (workgroup PDHG) -- the per-rank
# shares of an 8-GPU run and PMC bytes / issue counters of the 65,536-scenario launch.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out/r
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/r/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    grep '^{' "gpurun_out/r/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],2), round(d['ms_per_step'],4), d.get('solver_iters_per_ph_iter'), round(d['time_split_ms']['solve_launch'],4), d['roofline'].get('kernel'), round(d['roofline']['frac'],3), d['roofline'].get('hbm'), d['all_optimal'])" 2>/dev/null || tail -2 "gpurun_out/r/$name.log" | cut -c1-300
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 -u bench.py --no-cpu-baseline --cm 64 --steps 10 --warmup 3"
for S in 32768 16384 8192; do step cm64_$S 300 $B --scens $S; done
P="python3 -u bench.py --no-cpu-baseline --cm 64 --steps 3 --warmup 1"
step pmcf 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r/pmcf -o run -- $P
step pmcw 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r/pmcw -o run -- $P
step sqa 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/r/sqa -o run -- $P
echo done
