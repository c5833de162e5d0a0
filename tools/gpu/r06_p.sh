#!/bin/bash
# Round 6, pass p: kernel traces of the 8,192 share and config 3 (the dispatches of one PH step
# and the gaps between them).
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6p
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for t in 8192 65536; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/t$t -o run -- python3 $R/bench.py --no-cpu-baseline --scens $t --steps 10 > $R/$O/t$t.log 2>&1 || { echo "trace $t failed"; exit 1; }
done
cd $R
for t in t8192 t65536; do f=$(find $O/$t -name "*kernel_trace.csv" | head -1); echo "== $t"; python3 tools/step_trace.py $f 2 | tail -16; done
echo done
