#!/bin/bash
# Round 6, pass ff: the multi-rank step at each rank share over real RCCL collectives (loopback
# N = 2, 4, 8): the per-rank step an N-GPU run pays before the collectives' own latency.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6ff
mkdir -p $O
export TMPDIR=/tmp
for n in 2 4 8; do MASTER_ADDR=127.0.0.1 MASTER_PORT=2959$n timeout -k 10 500 python3 -u tools/fake_ranks.py $n 60 rccl > $O/rccl_$n.log 2>&1; echo "N=$n rc=$?"; grep -E "loopback" $O/rccl_$n.log | cut -c1-120; done
echo done
