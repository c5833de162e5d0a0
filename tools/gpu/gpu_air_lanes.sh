# aircond 65,536 (config 4): lanes-per-scenario sweep through bench.py (PHGPU_LANES pins L)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for L in 4 8 16; do
  PHGPU_LANES=$L timeout -k 10 300 python -u bench.py --model aircond --bf 32,32,64 --steps 10 --warmup 3 > gpurun_out/bench_aircond_L$L.log 2>&1 || exit $?
done
