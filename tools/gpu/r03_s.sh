#!/bin/bash
# Round 3, pass s: config 4 on lane groups of 4 by default (its one-lane IPM module spills):
# the config-4 / IPM GPU tests, the bench, PMC bytes and a kernel trace.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    grep '^{' "gpurun_out/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4), d.get('solver'), d.get('solver_iters_per_ph_iter'), d['time_split_ms'], d['roofline'].get('kernel'), d['roofline'].get('lanes_per_scenario'), round(d['roofline']['frac'],3), d['roofline'].get('traffic'), d['all_optimal'])" 2>/dev/null || tail -2 "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 -u bench.py --no-cpu-baseline --model aircond"
T="python -u -m pytest -v -x --timeout 600 --timeout-method thread"
step s_tests 1000 $T -m gpu tests/test_gpu_config4.py tests/test_gpu_ipm.py tests/test_gpu_speculative.py tests/test_gpu_parity.py tests/test_xhat_eval.py tests/test_dist_engine.py
step s_air 300 $B
P="python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --model aircond"
step s_pmcf 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/s_pmcf -o run -- $P
step s_pmcw 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/s_pmcw -o run -- $P
step s_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s_trace -o run -- python3 bench.py --no-cpu-baseline --model aircond
step s_air_again 300 $B
echo done
