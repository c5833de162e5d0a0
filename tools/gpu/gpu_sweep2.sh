# restart-test interval sweep (restart_every = 8 / 16 / 32 PDHG iterations, check_every 64)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for S in 65536 8192; do
  for RE in 16 32 8; do
    timeout -k 10 200 python -u tools/kbench.py $S 1 0 restart_every=$RE > gpurun_out/sweep_s${S}_re${RE}.log 2>&1 || exit $?
  done
done
