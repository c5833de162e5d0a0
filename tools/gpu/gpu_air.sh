# parity tests + aircond config-4 bench and kernel trace (multi-node x̄ merge)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gputests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --model aircond --bf 32,32,64 --steps 10 --warmup 3 > gpurun_out/bench_aircond65536.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_air -o run -- python -u bench.py --model aircond --bf 32,32,64 --steps 10 --warmup 3 > gpurun_out/prof_air.log 2>&1 || exit $?
