#!/bin/bash
# Round 2 (session 2) closing check on HEAD: GPU suite, smoke, the driver's default bench
# (config 3 with the CPU baseline), config 4, kernel-trace stats of config 2.
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
step z_gputests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step z_smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step z_bench 400 python -u bench.py
step z_bench_air 300 python3 -u bench.py --no-cpu-baseline --model aircond
step z_prof_cfg2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/z_prof_cfg2 -o run -- python3 bench.py --no-cpu-baseline --scens 1024 --cm 10 --steps 20 --warmup 5
echo done
