# parity tests, then the lane-count sweep of the chunked register kernel (kbench)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gputests.log 2>&1 || exit $?
for S in 8192 16384 32768 65536; do
  timeout -k 10 200 python -u tools/kbench.py $S 1 4,8,16,32 > gpurun_out/kb_s$S.log 2>&1 || exit $?
done
PHGPU_LIB=variants/libphgpu_w3.so timeout -k 10 200 python -u tools/kbench.py 65536 1 4,8 > gpurun_out/kb_w3.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/kbench.py 65536 64 0 > gpurun_out/kb_cm64.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/kbench.py 1024 10 0 > gpurun_out/kb_cm10.log 2>&1 || exit $?
