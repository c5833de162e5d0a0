#!/bin/bash
# Round 2 (session 2) end-of-session check on the final tree: GPU suite, smoke, default bench.
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
step e_gputests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step e_smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step e_bench 400 python -u bench.py
echo done
