#!/bin/bash
# Round 5, pass b: subtree-kernel jam hand-over (honest statuses) on the GPU tests of the
# workgroup kernels and config 2; the speculative / fold tests; config 2 bench; the 8,192
# share at L = 8 and L = 16.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5b
mkdir -p $O
export TMPDIR=/tmp
step() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; tail -2 $O/$n.log; [ $r -eq 0 ] || exit $r; }
step tests 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_speculative.py tests/test_gpu_ipm_wave.py tests/test_gpu_wg.py "tests/test_gpu_parity.py::test_farmer_cm10_parity" tests/test_gpu_scale.py -k "not register_path and not headline_instance"
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), round(d["ms_per_step"],4), d["solver_iters_per_ph_iter"], d["all_optimal"], d.get("path6_last_solve_jam_handovers"), d.get("path6_last_solve_recentrings"))'
b() { n=$1; shift; timeout -k 10 240 python3 -u bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || exit $r; grep '^{' $O/$n.log | python3 -c "$S"; }
b cfg2 --scens 1024 --cm 10
b cfg2b --scens 1024 --cm 10 --steps 60
b s8192 --scens 8192
PHGPU_IPM_LANES=16 b s8192_L16 --scens 8192
PHGPU_IPM_LANES=4 b s8192_L4 --scens 8192
echo done
