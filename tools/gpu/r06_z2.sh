#!/bin/bash
# Round 6, closing pass 2: the default bench line with its CPU baseline, its kernel trace
# (--stats), PMC byte and issue passes of config 3 and the 8,192 share.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6z2
mkdir -p $O
export TMPDIR=/tmp
step() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || { tail -5 $O/$n.log; exit $r; }; }
step bench 400 python3 -u bench.py
grep '^{' $O/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["cpu_baseline"]["value"], (d.get("checks") or {}).get("all_ok"))'
step prof3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof3 -o run -- python3 -u bench.py --no-cpu-baseline
grep '^{' $O/prof3.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("profiled:", d["value"], d["roofline"]["launch_ms"])'
P="python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
for cfg in c3 s8192; do
  case $cfg in c3) C="$P";; s8192) C="$P --scens 8192";; esac
  step pmcf_$cfg 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf_$cfg -o run -- $C
  step pmcw_$cfg 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw_$cfg -o run -- $C
  step sqa_$cfg 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d $O/sqa_$cfg -o run -- $C
  step sqb_$cfg 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_ANY --output-format csv -d $O/sqb_$cfg -o run -- $C
done
echo done
