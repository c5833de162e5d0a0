#!/bin/bash
# Round 2 (session 2): per-step overheads trimmed (multi-block status count, one PH-state
# record transpose, no dual output in the loop); iteration-count dump; GPU suite.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -3 "gpurun_out/$name.log" | cut -c1-400
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
step dump 200 python -u tools/dump_iters.py 65536 40
step bench_cfg3 300 python -u bench.py --no-cpu-baseline
step bench_s8192 300 python -u bench.py --scens 8192 --no-cpu-baseline
step prof_ovh 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ovh -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5
step gputests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
echo done
