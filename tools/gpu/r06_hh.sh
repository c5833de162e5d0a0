#!/bin/bash
# Round 6, pass hh: config 4 (aircond 32x32x64) with the one-lane module's slack reciprocals in
# LDS (IPM_LDS_ISL, 132 B of spills per lane offline against 516) vs as before; self-checked.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6hh
mkdir -p $O
export TMPDIR=/tmp
run() { timeout -k 10 300 python3 -u bench.py --model aircond --bf 32,32,64 --no-cpu-baseline --check on > $O/$1.log 2>&1 || { echo "$1 failed"; tail -5 $O/$1.log; exit 1; }; echo "$1"; grep '^{' $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("ms_per_step_median"), d["roofline"]["frac"], (d.get("checks") or {}).get("all_ok"))'; }
run base1
PHGPU_IPM_DEFS="IPM_LDS_ISL=1" run lds1
run base2
PHGPU_IPM_DEFS="IPM_LDS_ISL=1" run lds2
PHGPU_IPM_DEFS="IPM_LDS_ISL=1" timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_config4.py tests/test_gpu_ipm.py > $O/tests_lds.log 2>&1; echo "tests(lds) rc=$?"; tail -2 $O/tests_lds.log
echo done
