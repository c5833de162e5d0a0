#!/bin/bash
# Round 2 (session 2): record mode + longest-first queue for the register path.
# A/B kbench (PHGPU_REG_REC=0 vs default), benches, then the GPU suite with record mode forced.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -4 "gpurun_out/$name.log" | cut -c1-700
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
step kb_rec 200 python -u tools/kbench.py 65536 1
PHGPU_REG_REC=0 step kb_norec 200 python -u tools/kbench.py 65536 1
step bench_cfg3 300 python -u bench.py --no-cpu-baseline
PHGPU_REG_REC=0 step bench_cfg3_norec 300 python -u bench.py --no-cpu-baseline
step bench_air 300 python -u bench.py --model aircond --no-cpu-baseline
step bench_s8192 300 python -u bench.py --scens 8192 --no-cpu-baseline
PHGPU_REG_REC=1 step gputests_rec 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
echo done
