#!/bin/bash
# Round 5, pass m: the multi-rank step path after dropping node_buf's clear for one-node
# trees: loopback timings, a kernel trace of the loopback 8,192 share, the reduction tests.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5m
mkdir -p $O
export TMPDIR=/tmp
step() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; tail -3 $O/$n.log; [ $r -eq 0 ] || exit $r; }
step tests 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_readback.py tests/test_dist_engine.py tests/test_gpu_dist_scale.py
step fake8 300 python3 -u tools/fake_ranks.py 8 40
step trace8 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace8 -o run -- python3 -u tools/fake_ranks.py 8 40 loopback
echo done
