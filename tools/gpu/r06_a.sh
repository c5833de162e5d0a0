#!/bin/bash
# Round 6, pass a: ADVICE fixes on the GPU, bench self-check (1 rank, 2 gloo ranks, and a
# perturbed rho that must fail), the 8,192-share baseline.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_variable_probability.py tests/test_solve_hooks.py > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > $O/b1.log 2>&1 || { echo "b1 rc=$?"; tail -20 $O/b1.log; exit 1; }
grep '^{' $O/b1.log
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --scens 8192 > $O/b8192.log 2>&1 || { echo "b8192 rc=$?"; tail -20 $O/b8192.log; exit 1; }
grep '^{' $O/b8192.log
timeout -k 10 400 python3 -u bench.py --gpus 2 --backend gloo --steps 10 > $O/g2.log 2>&1 || { echo "g2 rc=$?"; tail -20 $O/g2.log; exit 1; }
grep '^{' $O/g2.log
timeout -k 10 400 python3 -u bench.py --gpus 2 --backend gloo --steps 4 --rho 1.02 --check on > $O/g2_bad.log 2>&1
r=$?; echo "perturbed rho rc=$r (expect non-zero)"
grep "checks" $O/g2_bad.log | tail -2
echo done1
# lane-group phase profile (IPM_PROF) at the 8,192 share
for L in 8 16 4; do
  timeout -k 10 200 python3 -u tools/ipm_prof.py 8192 $L > $O/prof_8192_L$L.log 2>&1 || { echo "prof L=$L rc=$?"; tail -20 $O/prof_8192_L$L.log; exit 1; }
  tail -1 $O/prof_8192_L$L.log
done
timeout -k 10 200 python3 -u tools/ipm_prof.py 8192 8 --prof 0 > $O/prof_8192_L8_off.log 2>&1 && tail -1 $O/prof_8192_L8_off.log
echo done2
