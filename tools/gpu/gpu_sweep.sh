# termination-check interval sweep (check_every = 16 / 32 / 64 PDHG iterations)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for S in 65536 8192; do
  for CE in 64 32 16; do
    timeout -k 10 200 python -u tools/kbench.py $S 1 0 check_every=$CE > gpurun_out/sweep_s${S}_ce${CE}.log 2>&1 || exit $?
  done
done
