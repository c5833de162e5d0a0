#!/bin/bash
# Round 3, pass e (session 2): verify HEAD -- new parity tests, full GPU suite, smoke,
# path-5 (hipRTC) tests, default bench, path-5 benches, gloo 2-rank rehearsal, kernel trace.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -2 "gpurun_out/$name.log" | cut -c1-400
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
(cat /sys/fs/cgroup/cpu.max; nproc; echo "OMP=$OMP_NUM_THREADS") > gpurun_out/e_cgroup.log 2>&1
B="python3 -u bench.py --no-cpu-baseline"
T="python -u -m pytest -v --timeout 600 --timeout-method thread"
step e_gputests 1200 $T -m gpu tests
step e_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step e_bench 400 python -u bench.py
PHGPU_JIT=1 step e_bench_jit 300 $B
step e_bench_s8192 300 $B --scens 8192
PHGPU_JIT=1 step e_bench_s8192_jit 300 $B --scens 8192
step e_bench_air 300 $B --model aircond
PHGPU_JIT=1 step e_bench_air_jit 300 $B --model aircond
step e_bench_gloo2 300 $B --gpus 2 --backend gloo --steps 10
echo done
