#!/bin/bash
# Round 2 (session 2): verify k_reg_prep (fused histogram + PH-state transpose).
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -1 "gpurun_out/$name.log" | cut -c1-200
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 -u bench.py --no-cpu-baseline"
step i_gputests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
PHGPU_REG_REC=1 step i_gputests_rec 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
echo done
