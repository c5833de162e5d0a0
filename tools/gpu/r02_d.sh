#!/bin/bash
# Round 2, pass D: wheel on separate ranks, cm=64 accuracy vs eps, full GPU suite.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -6 "gpurun_out/$name.log"
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
step wheel_ranks 300 python -u -m pytest tests/test_wheel_ranks.py -v --timeout 280 --timeout-method thread
step cm64_eps 300 python -u tools/cm64_eps.py 1e-9,3e-10,1e-10,3e-11
step gputests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
echo done
