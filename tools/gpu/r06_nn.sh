#!/bin/bash
# Round 6, pass nn: config 2 (farmer 1,024, cm=10) kernel trace.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6nn
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2 -o run -- python3 -u bench.py --scens 1024 --cm 10 --no-cpu-baseline > $O/prof2.log 2>&1; echo "prof rc=$?"; grep '^{' $O/prof2.log | cut -c1-200
echo done
