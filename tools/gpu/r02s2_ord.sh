#!/bin/bash
# Round 2 (session 2): queue-order study (exact vs previous-iteration predictor), record-mode
# load overhead at a fixed iteration count.
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
step ord_rec 200 python -u tools/kbench_order.py 65536
PHGPU_REG_REC=0 step ord_norec 200 python -u tools/kbench_order.py 65536
PHGPU_REG_REC=1 step kb_fixed224_rec 200 python -u tools/kbench.py 65536 1 0 eps_rel=0.0,max_iter=224
echo done
