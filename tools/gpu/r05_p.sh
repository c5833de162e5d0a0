#!/bin/bash
# Round 5, pass o (and p: the next x̄ reduced ahead of the convergence test): the speculative solve launched before the side-stream conv work (several
# ranks): the multi-rank tests, loopback timings and trace, the 2-rank gloo bench line.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5p
mkdir -p $O
export TMPDIR=/tmp
step() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; tail -3 $O/$n.log; [ $r -eq 0 ] || exit $r; }
step tests 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dist_engine.py tests/test_gpu_dist_scale.py tests/test_gpu_readback.py tests/test_gpu_convergence.py tests/test_gpu_speculative.py
step fake 300 python3 -u tools/fake_ranks.py 8 40
step trace8 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace8 -o run -- python3 -u tools/fake_ranks.py 8 40 loopback
step gloo2 300 python3 -u bench.py --gpus 2 --backend gloo --no-cpu-baseline
echo done
