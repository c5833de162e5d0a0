#!/bin/bash
# Round 2 (session 2): fused primal step (one FMA after the A^T y gather), tree dot for
# 4-entry rows: benches, GPU suite.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -2 "gpurun_out/$name.log" | cut -c1-250
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
step bench_cfg3 300 python -u bench.py --no-cpu-baseline
step bench_s8192 300 python -u bench.py --scens 8192 --no-cpu-baseline
step bench_air 300 python -u bench.py --model aircond --no-cpu-baseline
step kb_8192 200 python -u tools/kbench.py 8192 1
step gputests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
echo done
