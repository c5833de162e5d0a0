#!/bin/bash
# Round 6, pass jj: config 4 (aircond 32x32x64) with the LDS slack reciprocals: its kernel trace
# (--stats) and the PMC byte and issue passes.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6jj
mkdir -p $O
export TMPDIR=/tmp
step() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || { tail -5 $O/$n.log; exit $r; }; }
A="--model aircond --bf 32,32,64 --no-cpu-baseline"
step prof4 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof4 -o run -- python3 -u bench.py $A
grep '^{' $O/prof4.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("profiled:", d["value"], d["roofline"]["launch_ms"])'
C="python3 -u bench.py $A --steps 3 --warmup 1"
step pmcf_c4 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf_c4 -o run -- $C
step pmcw_c4 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw_c4 -o run -- $C
step sqa_c4 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d $O/sqa_c4 -o run -- $C
step sqb_c4 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_ANY --output-format csv -d $O/sqb_c4 -o run -- $C
echo done
