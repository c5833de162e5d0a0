#!/bin/bash
# Round 6, pass gg: the N = 2 share (32,768 scenarios) over real RCCL loopback with the one-lane
# IPM launched in 256-, 128- and 64-thread workgroups (PHGPU_IPM_BLK; no folded step there).
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6gg
mkdir -p $O
export TMPDIR=/tmp
for b in 256 64 128 256 64; do PHGPU_IPM_BLK=$b MASTER_ADDR=127.0.0.1 MASTER_PORT=29571 timeout -k 10 300 python3 -u tools/fake_ranks.py 2 60 rccl > $O/b$b.log 2>&1 || { echo "b=$b failed"; tail -5 $O/b$b.log; exit 1; }; echo "b=$b"; grep -E "library" $O/b$b.log | cut -c1-130; done
echo done
