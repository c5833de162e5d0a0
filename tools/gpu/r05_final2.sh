#!/bin/bash
# Round 5, closing pass, part 2: PMC byte and issue passes of configs 3 / 2 / 4 and the 8,192 share,
# the other configurations' bench lines, lane groups of 2 at 32,768 / 16,384 scenarios.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5f
mkdir -p $O
export TMPDIR=/tmp
step() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; tail -2 $O/$n.log; [ $r -eq 0 ] || exit $r; }
P="python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
for cfg in c3 c2 c4 s8192; do
  case $cfg in c3) C="$P";; c2) C="$P --scens 1024 --cm 10";; c4) C="$P --model aircond";; s8192) C="$P --scens 8192";; esac
  step pmcf_$cfg 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf_$cfg -o run -- $C
  step pmcw_$cfg 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw_$cfg -o run -- $C
  step sqa_$cfg 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d $O/sqa_$cfg -o run -- $C
  step sqb_$cfg 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_ANY --output-format csv -d $O/sqb_$cfg -o run -- $C
done
B="python3 -u bench.py --no-cpu-baseline"
step b_cfg2 300 $B --scens 1024 --cm 10
step b_cfg4 300 $B --model aircond
step b_s32768 200 $B --scens 32768
step b_s16384 200 $B --scens 16384
step b_s8192 200 $B --scens 8192
step b_cm64 400 $B --cm 64 --steps 10 --warmup 3
step b_gloo2 300 $B --gpus 2 --backend gloo
step b_gloo2_serial 300 $B --gpus 2 --backend gloo --no-conv-overlap
PHGPU_IPM_LANES=2 PHGPU_IPM_SPILL_MAX=100000 step b_s32768_L2 200 $B --scens 32768
PHGPU_IPM_LANES=2 PHGPU_IPM_SPILL_MAX=100000 step b_s16384_L2 200 $B --scens 16384
echo done
