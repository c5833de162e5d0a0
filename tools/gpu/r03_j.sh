#!/bin/bash
# Round 3, pass j: the tree with path 6 as the default -- whole GPU suite, smoke, the
# default bench (with its CPU baseline), PMC passes of the path-6 kernel (HBM bytes and
# the issue side), a kernel trace, a 2-rank gloo rehearsal and aircond.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -3 "gpurun_out/$name.log" | cut -c1-500
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 -u bench.py --no-cpu-baseline"
T="python -u -m pytest -v --timeout 600 --timeout-method thread"
P="python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
step j_gputests 1200 $T -m gpu tests
step j_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step j_bench 400 python3 -u bench.py
step j_pmc_fetch 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/j_pmc_fetch -o run -- $P
step j_pmc_write 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/j_pmc_write -o run -- $P
step j_pmc_sqa 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/j_pmc_sqa -o run -- $P
step j_pmc_sqb 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_ANY --output-format csv -d gpurun_out/j_pmc_sqb -o run -- $P
step j_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/j_trace -o run -- python3 bench.py --no-cpu-baseline
step j_gloo2 300 $B --gpus 2 --backend gloo --steps 10
step j_air 300 $B --model aircond
step j_s8192 300 $B --scens 8192
echo done
