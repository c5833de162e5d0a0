#!/bin/bash
# Round 2, pass B: the workgroup-per-scenario kernel (config 2 and farmer cm = 64), all GPU
# tests, benches, kernel stats.  Each GPU step has its own time limit; a timeout, abort or
# signal ends the script (test failures, rc 1, do not).
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
step wgtests 300 python -u -m pytest tests/test_gpu_wg.py -v --timeout 120 --timeout-method thread
step gputests 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step bench_cfg2 300 python -u bench.py --scens 1024 --cm 10 --no-cpu-baseline
step bench_cm64 400 python -u bench.py --scens 65536 --cm 64 --steps 5 --warmup 2 --no-cpu-baseline
step prof_cm1 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cm1 -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5
step prof_cm64 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cm64 -o run -- python3 bench.py --scens 65536 --cm 64 --steps 3 --warmup 1 --no-cpu-baseline
echo done
