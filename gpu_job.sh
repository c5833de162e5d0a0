set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
echo "tests rc=$?" >> gpurun_out/gputests.log
timeout -k 10 200 python -u tools/diag_iter0.py 65536 > gpurun_out/diag.log 2>&1
echo "diag rc=$?" >> gpurun_out/diag.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1
echo "bench rc=$?" >> gpurun_out/bench.log
