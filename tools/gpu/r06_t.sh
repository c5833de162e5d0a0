#!/bin/bash
# Round 6, pass t: where the host's time per PH iteration goes (cProfile of iterk_loop) at the
# 8,192 share and at config 3.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6t
mkdir -p $O
export TMPDIR=/tmp
for S in 8192 65536; do timeout -k 10 300 python3 -u tools/host_prof.py $S 200 > $O/host_$S.log 2>&1 || { echo "host $S failed"; tail -20 $O/host_$S.log; exit 1; }; head -45 $O/host_$S.log | grep -v "^$"; done
echo done
