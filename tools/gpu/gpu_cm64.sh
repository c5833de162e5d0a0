# HBM-bound variant (SURVEY 8(d) cfg3 cm=64: 67.6 KB per scenario, 4.4 GB of scenario data):
# farmer 65,536 scenarios cm=64 on the global-memory kernel; bench, kernel trace, FETCH/WRITE
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --scens 65536 --cm 64 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_farmer65536_cm64.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cm64 -o run -- python -u bench.py --scens 65536 --cm 64 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_cm64.log 2>&1 || exit $?
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_cm64 -o run -- python -u bench.py --scens 65536 --cm 64 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch_cm64.log 2>&1 || exit $?
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_cm64 -o run -- python -u bench.py --scens 65536 --cm 64 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write_cm64.log 2>&1 || exit $?
