# non-headline configs: aircond multistage at 65,536 scenarios (config 4), farmer cm=10 at
# 1,024 scenarios (config 2), and a 2-rank gloo rehearsal of the N>1 bench path on one GPU
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --model aircond --bf 32,32,64 --steps 10 --warmup 3 > gpurun_out/bench_aircond65536.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_air -o run -- python -u bench.py --model aircond --bf 32,32,64 --steps 10 --warmup 3 > gpurun_out/prof_air.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --scens 1024 --cm 10 --steps 10 --warmup 3 --cpu-sample 64 > gpurun_out/bench_farmer1024_cm10.log 2>&1 || exit $?
PHGPU_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/bench_gloo2.log 2>&1 || exit $?
