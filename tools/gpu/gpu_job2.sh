mkdir -p gpurun_out
timeout -k 10 200 python -u tools/diag_random.py > gpurun_out/diag_random.log 2>&1
