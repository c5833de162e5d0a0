#!/bin/bash
# Round 4, pass d: why cm = 64 PH subproblems miss the oracle by 1e-5 on path 6, and where
# the cm = 64 bench stalls (both workgroup kernels).
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -12 "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
step d_diag 150 python3 -u tests/diag_ipm_cm64.py 12
echo done
