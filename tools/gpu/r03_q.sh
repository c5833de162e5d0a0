#!/bin/bash
# Round 3, pass q: the state to report -- whole GPU suite, smoke, default bench (with its
# CPU baseline), every config, per-share PMC bytes for the changed lane-group kernel, a
# kernel trace and SQ counters of the headline kernel.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    grep '^{' "gpurun_out/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],4), round(d['ms_per_step'],4), d.get('solver'), d.get('solver_iters_per_ph_iter'), d['time_split_ms'], d['roofline'].get('kernel'), round(d['roofline']['frac'],3))" 2>/dev/null || tail -2 "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 -u bench.py --no-cpu-baseline"
step q_gputests 1200 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu tests
step q_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step q_bench 400 python3 -u bench.py
for S in 32768 16384 8192; do step q_s$S 300 $B --scens $S; done
step q_air 300 $B --model aircond
step q_air8192 300 $B --model aircond --bf 4,32,64
step q_cfg2 300 $B --scens 1024 --cm 10
step q_cm64 300 $B --cm 64 --steps 5 --warmup 2
step q_gloo2 300 $B --gpus 2 --backend gloo --steps 10
P="python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
for S in 16384 8192; do
  step q_pmcf_$S 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/q_pmcf_$S -o run -- $P --scens $S
  step q_pmcw_$S 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/q_pmcw_$S -o run -- $P --scens $S
done
step q_sqa 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/q_sqa -o run -- $P
step q_sqb 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_ANY --output-format csv -d gpurun_out/q_sqb -o run -- $P
step q_sqa8 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/q_sqa8 -o run -- $P --scens 8192
step q_sqb8 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_ANY --output-format csv -d gpurun_out/q_sqb8 -o run -- $P --scens 8192
step q_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/q_trace -o run -- python3 bench.py --no-cpu-baseline
step q_trace8192 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/q_trace8192 -o run -- python3 bench.py --no-cpu-baseline --scens 8192
step q_uc 1000 $B --model uc --steps 2 --warmup 1
echo done
