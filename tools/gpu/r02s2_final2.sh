#!/bin/bash
# Round 2 (session 2) second measurement pass on HEAD (farmer with its recommended
# PH-solve option): GPU suite, smoke, benches (config 3 with
# the CPU baseline, configs 2 / 4, cm=64, the 8,192 share), kernel-trace stats and PMC
# passes (HBM bytes, SQ issue) of the config 3 solve kernel.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -1 "gpurun_out/$name.log" | cut -c1-200
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 bench.py --no-cpu-baseline"
step h_gputests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step h_smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step h_bench_cfg3 400 python -u bench.py
step h_bench_cfg2 300 $B --scens 1024 --cm 10
step h_bench_air 300 $B --model aircond
step h_bench_s8192 300 $B --scens 8192
step h_bench_cm64 400 $B --cm 64 --steps 5 --warmup 2
step h_bench_gloo2 300 python3 -u bench.py --gpus 2 --backend gloo --no-cpu-baseline --steps 10
step h_prof_cfg3 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/h_prof_cfg3 -o run -- $B --steps 20 --warmup 5
step h_pmc_fetch 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/h_pmc_fetch -o run -- $B --steps 3 --warmup 1
step h_pmc_write 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/h_pmc_write -o run -- $B --steps 3 --warmup 1
step h_pmc_sqa 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/h_pmc_sqa -o run -- $B --steps 3 --warmup 1
step h_pmc_sqb 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_ANY --output-format csv -d gpurun_out/h_pmc_sqb -o run -- $B --steps 3 --warmup 1
echo done
