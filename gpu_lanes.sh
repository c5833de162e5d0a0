# bench at pinned lane counts (farmer 65,536 cm=1)
set -o pipefail
mkdir -p gpurun_out
for L in 4 8; do
  PHGPU_LANES=$L timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_L$L.log 2>&1 || exit $?
done
