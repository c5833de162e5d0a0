#!/bin/bash
# Round 6, pass tt: the N = 2 share (32,768) over RCCL loopback with lane groups of 2 (its
# module spills 428 B per lane) against one lane, alternating.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6tt
mkdir -p $O
export TMPDIR=/tmp
run() { MASTER_ADDR=127.0.0.1 MASTER_PORT=29581 timeout -k 10 300 python3 -u tools/fake_ranks.py 2 60 rccl > $O/$1.log 2>&1 || { echo "$1 failed"; tail -5 $O/$1.log; exit 1; }; echo "$1 $(grep -E 'library' $O/$1.log | cut -c1-120)"; }
run l1a
PHGPU_IPM_LANES=2 run l2a
run l1b
PHGPU_IPM_LANES=2 run l2b
echo done
