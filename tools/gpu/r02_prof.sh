#!/bin/bash
# Round 2 measurement pass: GPU tests, smoke, benches (headline + configs 2/4 + cm=64),
# kernel-trace stats and PMC passes (HBM bytes, SQ issue) for the headline and cm=64.
# Each GPU step has its own limit; a timeout / abort / signal ends the script.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -2 "gpurun_out/$name.log" | cut -c1-400
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 bench.py --no-cpu-baseline"
step gputests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_farmer65536_cm1 300 python -u bench.py
step bench_farmer1024_cm10 300 $B --scens 1024 --cm 10
step bench_aircond65536 300 $B --model aircond
step bench_farmer65536_cm64 400 $B --cm 64 --steps 5 --warmup 2
step bench_gloo2 300 python -u bench.py --gpus 2 --backend gloo --no-cpu-baseline --steps 10
step prof_cm1 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cm1 -o run -- $B --steps 20 --warmup 5
step prof_cm64 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cm64 -o run -- $B --cm 64 --steps 3 --warmup 1
step prof_cfg2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cfg2 -o run -- $B --scens 1024 --cm 10 --steps 20 --warmup 5
step pmc_fetch_cm1 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_cm1 -o run -- $B --steps 3 --warmup 1
step pmc_write_cm1 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_cm1 -o run -- $B --steps 3 --warmup 1
step pmc_fetch_cm64 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_cm64 -o run -- $B --cm 64 --steps 3 --warmup 1
step pmc_write_cm64 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_cm64 -o run -- $B --cm 64 --steps 3 --warmup 1
step pmc_sqa_cm1 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmc_sqa_cm1 -o run -- $B --steps 3 --warmup 1
step pmc_sqb_cm1 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_sqb_cm1 -o run -- $B --steps 3 --warmup 1
step pmc_sqa_cm64 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmc_sqa_cm64 -o run -- $B --cm 64 --steps 3 --warmup 1
step pmc_sqb_cm64 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_sqb_cm64 -o run -- $B --cm 64 --steps 3 --warmup 1
echo done
