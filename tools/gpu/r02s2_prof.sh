#!/bin/bash
# Round 2 (session 2): kernel-trace stats of the headline bench in record mode and scenario
# order (separates the solve kernel from the record transposes and the queue-order kernels).
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -3 "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 bench.py --no-cpu-baseline --steps 20 --warmup 5"
step prof_rec 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rec -o run -- $B
PHGPU_REG_REC=0 step prof_norec 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_norec -o run -- $B
echo done
