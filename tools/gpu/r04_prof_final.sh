#!/bin/bash
# Round 4: kernel-trace statistics of the default bench command (final build), configs 3 and 2.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out/pf
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pf/cfg3 -o run -- python3 -u bench.py --no-cpu-baseline > gpurun_out/pf/cfg3.log 2>&1; r=$?; echo "cfg3 rc=$r"; [ $r -eq 0 ] || exit $r
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pf/cfg2 -o run -- python3 -u bench.py --no-cpu-baseline --scens 1024 --cm 10 > gpurun_out/pf/cfg2.log 2>&1; r=$?; echo "cfg2 rc=$r"; [ $r -eq 0 ] || exit $r
