#!/bin/bash
# Round 4, pass u (final measurement): the path-6 medium-scenario tests, then the default
# bench with its CPU baseline, config 2 / 4 and the 8,192 share, kernel traces of configs 2 / 3.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out/u
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/u/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    grep '^{' "gpurun_out/u/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4), d.get('solver_iters_per_ph_iter'), round(d['time_split_ms']['solve_launch'],4), d['roofline'].get('kernel'), round(d['roofline']['frac'],3), d['all_optimal'], d.get('cpu_baseline'))" 2>/dev/null || tail -3 "gpurun_out/u/$name.log" | cut -c1-300
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
step tests 400 python3 -u -m pytest -m gpu -q --timeout 120 --timeout-method thread tests/test_gpu_ipm_wave.py tests/test_gpu_wg.py tests/test_gpu_scale.py tests/test_gpu_parity.py
step bench 400 python3 -u bench.py
B="python3 -u bench.py --no-cpu-baseline"
step cfg2 200 $B --scens 1024 --cm 10
step s8192 200 $B --scens 8192
step air 200 $B --model aircond
step trace3 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/u/trace3 -o run -- python3 bench.py --no-cpu-baseline
step trace2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/u/trace2 -o run -- python3 bench.py --no-cpu-baseline --scens 1024 --cm 10
echo done
