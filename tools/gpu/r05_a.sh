#!/bin/bash
# Round 5, pass a: the 2-rank headline-scale parity tests (gloo ranks sharing the GPU), the
# split form with a wrapping barrier counter, config 3 under rocprofv3 (teardown), the
# path-6 iteration dump, SQ passes of the 8,192 share and of config 4.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5a
mkdir -p $O
export TMPDIR=/tmp
step() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; tail -3 $O/$n.log; [ $r -eq 0 ] || exit $r; }
step dist 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_dist_scale.py
step split 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_uc.py -k "split_matches"
step prof3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof3 -o run -- python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5
step iters 200 python3 -u tools/dump_ipm_iters.py 65536 30
cp gpurun_out/ipm_iters_S65536.npz $O/ 2>/dev/null
P="python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
for cfg in s8192 air; do
  if [ $cfg = s8192 ]; then C="$P --scens 8192"; else C="$P --model aircond"; fi
  step sqa_$cfg 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d $O/sqa_$cfg -o run -- $C
  step sqb_$cfg 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_ANY --output-format csv -d $O/sqb_$cfg -o run -- $C
done
echo done
