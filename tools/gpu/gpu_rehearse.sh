# functional rehearsal of the N>1 bench path on a 1-GPU box (gloo, ranks share cuda:0):
# farmer 4 ranks (16,384 scenarios each, the N=4 lane plan) and aircond 2 ranks (multi-node x̄)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
PHGPU_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --steps 5 --warmup 2 > gpurun_out/bench_gloo4.log 2>&1 || exit $?
PHGPU_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 2 --model aircond --bf 32,32,64 --steps 5 --warmup 2 > gpurun_out/bench_gloo2_aircond.log 2>&1 || exit $?
