#!/bin/bash
# Round 2 (session 2): EMA queue predictor, fused PH-state transpose, parallel status count,
# self-resetting order bins: benches, kernel stats, GPU suite.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -2 "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
step bench_cfg3 300 python -u bench.py --no-cpu-baseline
PHGPU_REG_REC=0 step bench_cfg3_norec 300 python -u bench.py --no-cpu-baseline
step bench_air 300 python -u bench.py --model aircond --no-cpu-baseline
step bench_s8192 300 python -u bench.py --scens 8192 --no-cpu-baseline
step prof_ema2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ema2 -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5
step gputests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
echo done
