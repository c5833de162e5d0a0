#!/bin/bash
# Round 2 (session 2): farmer's recommended PH-solve options (beta_sufficient 0.6) on the
# farmer configs, GPU suite (the headline test runs with them).
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -1 "gpurun_out/$name.log" | cut -c1-160
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 -u bench.py --no-cpu-baseline"
step g_cfg3 300 $B
step g_cfg2 300 $B --scens 1024 --cm 10
step g_s8192 300 $B --scens 8192
step g_cm64 400 $B --cm 64 --steps 5 --warmup 2
step g_cm64_def 400 $B --cm 64 --steps 5 --warmup 2 --default-solver-options
step g_gputests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
echo done
