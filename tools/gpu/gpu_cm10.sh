# config 2 (farmer cm=10, 1,024 scenarios): parity tests, kernel micro-bench, bench, rocprof
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gputests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/kbench.py 1024 10 0 > gpurun_out/kb_s1024_cm10.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --scens 1024 --cm 10 --steps 10 --warmup 3 --cpu-sample 64 > gpurun_out/bench_farmer1024_cm10.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cm10 -o run -- python -u bench.py --scens 1024 --cm 10 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_cm10.log 2>&1 || exit $?
