#!/bin/bash
# Round 2 (session 2): restart-parameter sweep of the PH solves on config 3 (Halpern
# restart criteria: sufficient / necessary decay, artificial restart fraction).
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -1 "gpurun_out/$name.log" | cut -c1-160
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 -u bench.py --no-cpu-baseline"
step b_base 300 $B
step b_bs01 300 $B --solver-opt beta_sufficient=0.1
step b_bs03 300 $B --solver-opt beta_sufficient=0.3
step b_bn06 300 $B --solver-opt beta_necessary=0.6
step b_bn09 300 $B --solver-opt beta_necessary=0.9
step b_ba02 300 $B --solver-opt beta_artificial=0.2
step b_ba05 300 $B --solver-opt beta_artificial=0.5
echo done
