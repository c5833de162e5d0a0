#!/bin/bash
# Round 3, pass v: the new GPU tests, then the full suite, smoke and the default bench.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    grep '^{' "gpurun_out/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4), d.get('solver_iters_per_ph_iter'), d['time_split_ms'], d['roofline'].get('lanes_per_scenario'), round(d['roofline']['frac'],3), d['roofline'].get('traffic'), d['all_optimal'])" 2>/dev/null || tail -3 "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 -u bench.py --no-cpu-baseline"
T="python -u -m pytest -v --timeout 600 --timeout-method thread"
step v_new 600 $T -x -m gpu tests/test_gpu_ipm.py -k "warm or lane_policy"
step v_gputests 1200 $T -m gpu tests
step v_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step v_bench 400 python3 -u bench.py
step v_s8192 300 $B --scens 8192
step v_air 300 $B --model aircond
echo done
