#!/bin/bash
# Round 3, pass b: the new parity tests (config 3 to convergence, config 4 on the bench
# instance, speculative-solve invisibility, final Lagrangian bound on separate ranks),
# the full GPU suite, the bench's new fields, a gloo 2-rank rehearsal line, aircond Iter0
# diagnostics, and the box's cgroup CPU quota.
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
(cat /sys/fs/cgroup/cpu.max; nproc; echo "OMP=$OMP_NUM_THREADS") > gpurun_out/b_cgroup.log 2>&1
B="python3 bench.py --no-cpu-baseline"
T="python -u -m pytest -v --timeout 600 --timeout-method thread"
step b_newtests 900 $T tests/test_gpu_convergence.py tests/test_gpu_config4.py tests/test_gpu_speculative.py tests/test_wheel_ranks.py
step b_gputests 900 $T -m gpu tests
step b_bench 400 python -u bench.py
step b_bench_gloo2 300 python3 -u bench.py --gpus 2 --backend gloo --no-cpu-baseline --steps 10
step b_diag_air 300 python -u tools/diag_air_iter0.py
echo done
