mkdir -p gpurun_out
timeout -k 10 200 python -u tools/kbench.py 65536 1 4,8 > gpurun_out/kb1.log 2>&1
timeout -k 10 200 python -u tools/kbench.py 65536 1 8 check_every=32 > gpurun_out/kb2.log 2>&1
timeout -k 10 200 python -u tools/kbench.py 65536 1 8 check_every=32,restart_every=8 > gpurun_out/kb3.log 2>&1
timeout -k 10 200 python -u tools/kbench.py 8192 1 8,16 > gpurun_out/kb4.log 2>&1
timeout -k 10 200 python -u tools/kbench.py 1024 10 16,32,64 > gpurun_out/kb5.log 2>&1
