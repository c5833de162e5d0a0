# GPU validation: parity tests, default lane plan at 65,536 / 8,192 scenarios, bench,
# kernel-trace stats, PMC passes (HBM bytes, SQ issue)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gputests.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/kbench.py 65536 1 0 > gpurun_out/kb_s65536.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/kbench.py 8192 1 0 > gpurun_out/kb_s8192.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || exit $?
python tools/trace_summary.py gpurun_out/prof/run_kernel_trace.csv 20 gpurun_out/prof/solve_dispatches.json >> gpurun_out/prof.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmc_sqa -o run -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_sqa.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_sqb -o run -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_sqb.log 2>&1 || exit $?
