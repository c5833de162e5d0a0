#!/bin/bash
# Round 4, pass h: dump the worst cm = 64 PH subproblems (scen0..2047) for a host replay.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out/h
export TMPDIR=/tmp
DIAG_DUMP=gpurun_out/h/worst timeout -k 10 120 python3 -u tests/diag_ipm_cm64.py 4 2048 first > gpurun_out/h/diag.log 2>&1
echo rc=$?
tail -12 gpurun_out/h/diag.log | cut -c1-200
