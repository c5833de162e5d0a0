#!/bin/bash
# Round 5, pass h: config 5's queue-kernel slot layouts on one warm PH trajectory
# (tools/uc_slots.py): 1 workgroup per CU (default), 2 per CU, 2 per CU with the T longest
# scenarios split over the whole GPU first.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r5h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u tools/uc_slots.py '[{}, {"PER_CU": 2}, {"PER_CU": 2, "SPLIT": 8}, {"PER_CU": 2, "SPLIT": 16}, {}]' > $O/slots.log 2>&1
r=$?; echo "slots rc=$r"; tail -8 $O/slots.log; cp gpurun_out/uc_slots.npz $O/ 2>/dev/null; exit $r
