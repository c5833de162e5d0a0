set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
echo "tests rc=$?" >> gpurun_out/gputests.log
timeout -k 10 300 python -u tools/kbench.py 65536 1 2,4,8,16 > gpurun_out/kbench.log 2>&1
echo "kbench rc=$?" >> gpurun_out/kbench.log
