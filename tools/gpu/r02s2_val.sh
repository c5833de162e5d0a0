#!/bin/bash
# Round 2 (session 2): A/B of the LDS hand-off (in-order, no drain vs drain), a fixed
# iteration-count run (imbalance), then GPU tests, smoke and benches on HEAD.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -4 "gpurun_out/$name.log" | cut -c1-600
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
step kb_nowait 200 python -u tools/kbench.py 65536 1
PHGPU_LIB=$PWD/variants/libphgpu_wait.so step kb_wait 200 python -u tools/kbench.py 65536 1
step kb_nowait_8192 200 python -u tools/kbench.py 8192 1
PHGPU_LIB=$PWD/variants/libphgpu_wait.so step kb_wait_8192 200 python -u tools/kbench.py 8192 1
step kb_fixed224 200 python -u tools/kbench.py 65536 1 0 eps_rel=0.0,max_iter=224
step gputests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_farmer65536_cm1 300 python -u bench.py
step bench_s8192 300 python -u bench.py --scens 8192 --no-cpu-baseline
echo done
