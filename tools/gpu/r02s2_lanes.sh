#!/bin/bash
# Round 2 (session 2): lane count re-check under record mode / longest-first queue.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 -u bench.py --no-cpu-baseline"
PHGPU_LANES=16 step l_air16 300 $B --model aircond
PHGPU_LANES=4 step l_air4 300 $B --model aircond
PHGPU_LANES=8 step l_cfg3_8 300 $B
PHGPU_LANES=16 step l_cfg3_16 300 $B
echo done
