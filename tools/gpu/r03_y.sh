#!/bin/bash
# Round 3, pass y (final): whole GPU suite, smoke, default bench (with its CPU baseline),
# the shares and config 4, PMC bytes / issue counters and a kernel trace of config 3.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    grep '^{' "gpurun_out/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4), d.get('solver_iters_per_ph_iter'), d['time_split_ms'], d['roofline'].get('lanes_per_scenario'), round(d['roofline']['frac'],3), d['roofline'].get('traffic'), d['all_optimal'])" 2>/dev/null || tail -2 "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 -u bench.py --no-cpu-baseline"
step y_gputests 1200 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu tests
step y_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step y_bench 400 python3 -u bench.py
for S in 32768 16384 8192; do step y_s$S 300 $B --scens $S; done
step y_air 300 $B --model aircond
step y_cfg2 300 $B --scens 1024 --cm 10
step y_gloo2 300 $B --gpus 2 --backend gloo --steps 10
P="python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
step y_pmcf 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/y_pmcf -o run -- $P
step y_pmcw 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/y_pmcw -o run -- $P
step y_sqa 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/y_sqa -o run -- $P
step y_sqb 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_ANY --output-format csv -d gpurun_out/y_sqb -o run -- $P
step y_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/y_trace -o run -- python3 bench.py --no-cpu-baseline
step y_trace8192 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/y_trace8192 -o run -- python3 bench.py --no-cpu-baseline --scens 8192
echo done
