#!/bin/bash
# Round 4, pass p (measurement): default bench with its CPU baseline, the per-rank shares,
# config 2 / 4, cm = 64; PMC bytes and issue counters of config 3 and config 2; kernel traces.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out/p
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/p/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    grep '^{' "gpurun_out/p/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4), d.get('solver_iters_per_ph_iter'), d['time_split_ms'], d['roofline'].get('kernel'), round(d['roofline']['frac'],3), d['all_optimal'])" 2>/dev/null || tail -2 "gpurun_out/p/$name.log" | cut -c1-300
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 -u bench.py --no-cpu-baseline"
step bench 400 python3 -u bench.py
for S in 32768 16384 8192; do step s$S 200 $B --scens $S; done
step cfg2 200 $B --scens 1024 --cm 10
step air 200 $B --model aircond
step air8192 200 $B --model aircond --bf 4,32,64
step cm64 300 $B --cm 64 --steps 10 --warmup 3
P="python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
P2="$P --scens 1024 --cm 10"
for cfg in 3 2; do
  if [ $cfg = 3 ]; then C="$P"; else C="$P2"; fi
  step pmcf$cfg 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/p/pmcf$cfg -o run -- $C
  step pmcw$cfg 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/p/pmcw$cfg -o run -- $C
  step sqa$cfg 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/p/sqa$cfg -o run -- $C
  step sqb$cfg 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_ANY --output-format csv -d gpurun_out/p/sqb$cfg -o run -- $C
done
step trace3 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p/trace3 -o run -- python3 bench.py --no-cpu-baseline
step trace2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p/trace2 -o run -- python3 bench.py --no-cpu-baseline --scens 1024 --cm 10
echo done
