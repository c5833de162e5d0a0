#!/bin/bash
# Post-records validation: full GPU suite, smoke, headline bench.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -3 "gpurun_out/$name.log" | cut -c1-600
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
step gputests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_farmer65536_cm1 300 python -u bench.py
step bench_farmer65536_cm64 400 python3 bench.py --no-cpu-baseline --cm 64 --steps 5 --warmup 2
echo done
