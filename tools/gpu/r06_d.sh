#!/bin/bash
# Round 6, pass d: per-wave timelines (plain stores, IPM_PROF=1) of the one-lane and
# lane-group kernels; the lane-group phase split (IPM_PROF=2).
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6d
mkdir -p $O
export TMPDIR=/tmp
p() { n=$1; shift; timeout -k 10 200 python3 -u tools/ipm_prof.py "$@" > $O/$n.log 2>&1; r=$?; [ $r -eq 0 ] || { echo "$n rc=$r"; tail -20 $O/$n.log; exit $r; }; tail -1 $O/$n.log; }
p l8 8192 8
p l8_off 8192 8 --prof 0
p l1 65536 1
p l1_off 65536 1 --prof 0
p l4 16384 4
p l1_32k 32768 1
p l8_lv2 8192 8 --level 2
echo done
