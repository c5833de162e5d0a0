#!/bin/bash
# Round 2, pass A: GPU tests (incl. headline-scale parity), bench N=1, gloo 2-rank
# rehearsal, rocprof kernel stats.  Each GPU step has its own time limit; a timeout,
# abort or signal ends the script (test failures, rc 1, do not).
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -3 "gpurun_out/$name.log"
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
step gputests 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step bench_n1 300 python -u bench.py
step bench_gloo2 300 python -u bench.py --gpus 2 --backend gloo --no-cpu-baseline --steps 10
step rocprof_stats 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_a -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5
echo done
