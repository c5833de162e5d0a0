# parity tests, then bench with the longest-first queue order on / off (farmer 65,536 cm=1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gputests.log 2>&1 || exit $?
for O in 1 0; do
  PHGPU_ORDER=$O timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_order$O.log 2>&1 || exit $?
done
PHGPU_ORDER=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --scens 8192 --no-cpu-baseline > gpurun_out/bench_s8192_order1.log 2>&1 || exit $?
PHGPU_ORDER=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --scens 8192 --no-cpu-baseline > gpurun_out/bench_s8192_order0.log 2>&1 || exit $?
