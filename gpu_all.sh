# GPU validation: parity tests, then the bench + profiles, then a 2-rank rehearsal of the
# multi-rank path on the one GPU (gloo between the ranks, both ranks on cuda:0)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/gputests.log; [ $rc -eq 0 ] || exit $rc
bash gpu_bench.sh || exit $?
PHGPU_DIST_BACKEND=gloo timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/bench2.log 2>&1
echo "bench2 rc=$?" >> gpurun_out/bench2.log
