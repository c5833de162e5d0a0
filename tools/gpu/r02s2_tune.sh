#!/bin/bash
# Round 2 (session 2): tuning A/B on config 3 -- 3 waves / SIMD (spills) and the KKT
# check interval with the longest-first queue.
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
B="python -u bench.py --no-cpu-baseline"
step t_base 300 $B
PHGPU_LIB=$PWD/variants/libphgpu_w3.so step t_w3 300 $B
step t_chk32 300 $B --solver-opt check_every=32
step t_chk128 300 $B --solver-opt check_every=128
step t_base_air 300 $B --model aircond
step t_chk32_air 300 $B --model aircond --solver-opt check_every=32
echo done
