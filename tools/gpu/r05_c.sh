#!/bin/bash
# Round 5, pass c: the subtree kernel's floor acceptance (config 2 tests + bench, mean and
# median step), the config-2 fixture's face-invariant check; aircond 65,536 on one lane
# with its spills allowed, against the lane-group default.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5c
mkdir -p $O
export TMPDIR=/tmp
step() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; tail -2 $O/$n.log; [ $r -eq 0 ] || exit $r; }
step tests 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_speculative.py tests/test_gpu_ipm_wave.py "tests/test_gpu_parity.py::test_farmer_cm10_parity" tests/test_gpu_scale.py -k "not register_path and not headline_instance and not infeasible"
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "median", round(d["ms_per_step"],4), "mean", round(d["ms_per_step_mean"],4), d["solver_iters_per_ph_iter"], d["all_optimal"], d.get("path6_last_solve_jam_handovers"), d.get("path6_last_solve_recentrings"))'
b() { n=$1; shift; timeout -k 10 300 python3 -u bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || exit $r; grep '^{' $O/$n.log | python3 -c "$S"; }
b cfg2 --scens 1024 --cm 10 --steps 60
b air --model aircond
PHGPU_IPM_LANES=1 PHGPU_IPM_SPILL_MAX=100000 b air_L1 --model aircond
echo done
