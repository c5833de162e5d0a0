#!/bin/bash
# Round 3, first pass: GPU suite, smoke, default bench, the N=8 share, config 4.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -1 "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 bench.py --no-cpu-baseline"
step a_gputests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step a_smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step a_bench 400 python -u bench.py
step a_bench_s8192 300 $B --scens 8192
step a_bench_air 300 $B --model aircond
echo done
