# occupancy variants (kbench) + SQ PMC passes of the bench's solve kernel
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for W in 2 3 4; do
  PHGPU_LIB=variants/libphgpu_w$W.so timeout -k 10 200 python -u tools/kbench.py 65536 1 0 > gpurun_out/kb_w$W.log 2>&1 || exit $?
done
SQA=SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_ACTIVE_INST_VALU,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_INST_LDS,GRBM_GUI_ACTIVE
SQB=SQ_INSTS_VALU_FMA_F64,SQ_INSTS_VALU_ADD_F64,SQ_INSTS_VALU_MUL_F64,SQ_INSTS_VALU_TRANS_F64,SQ_ACTIVE_INST_LDS,SQ_WAIT_ANY,SQ_LDS_BANK_CONFLICT,SQ_WAVES,GRBM_GUI_ACTIVE
timeout -s KILL 120 rocprofv3 --pmc $(echo $SQA | tr , ' ') --output-format csv -d gpurun_out/pmc_sqa -o run -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_sqa.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc $(echo $SQB | tr , ' ') --output-format csv -d gpurun_out/pmc_sqb -o run -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_sqb.log 2>&1 || exit $?
python tools/pmc_sq_summary.py gpurun_out/pmc_sq_summary.json gpurun_out/pmc_sqa/run_counter_collection.csv gpurun_out/pmc_sqb/run_counter_collection.csv > gpurun_out/pmc_sq.log 2>&1
PHGPU_DIST_BACKEND=gloo timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/bench2.log 2>&1
echo "bench2 rc=$?" >> gpurun_out/bench2.log
