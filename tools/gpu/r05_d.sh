#!/bin/bash
# Round 5, pass d: config 4 on the one-lane module (tests + bench), the 2-rank headline-scale
# tests again, config 2's per-step jam diagnostic, config 5 with the Iter0 continuation.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5d
mkdir -p $O
export TMPDIR=/tmp
step() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; tail -2 $O/$n.log; [ $r -eq 0 ] || exit $r; }
step tests 900 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_config4.py tests/test_gpu_dist_scale.py tests/test_gpu_ipm.py "tests/test_gpu_convergence.py::test_config3_iterations_to_convergence[6-1e-09-1e-05]" tests/test_gpu_readback.py tests/test_gpu_speculative.py
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "median", round(d["ms_per_step"],4), "mean", round(d["ms_per_step_mean"],4), d["solver_iters_per_ph_iter"], d["all_optimal"], d.get("iter0_not_optimal"), d.get("iter0_continuation_solves"), d.get("trivial_bound"))'
b() { n=$1; shift; timeout -k 10 600 python3 -u bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || exit $r; grep '^{' $O/$n.log | python3 -c "$S"; }
b air --model aircond
step jams 300 python3 -u tools/diag_jams.py 60
b uc --model uc --steps 2 --warmup 1
echo done
