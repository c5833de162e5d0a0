# configs 2 and 4 on the current kernels: bench lines + kernel-trace stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --scens 1024 --cm 10 --steps 10 --warmup 3 --cpu-sample 64 > gpurun_out/bench_farmer1024_cm10.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cm10 -o run -- python -u bench.py --scens 1024 --cm 10 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_cm10.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --model aircond --bf 32,32,64 --steps 10 --warmup 3 > gpurun_out/bench_aircond65536.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_air -o run -- python -u bench.py --model aircond --bf 32,32,64 --steps 10 --warmup 3 > gpurun_out/prof_air.log 2>&1 || exit $?
