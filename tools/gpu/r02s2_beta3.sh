#!/bin/bash
# Round 2 (session 2): restart-parameter sweep, third pass: beta_sufficient 0.5-0.8 on
# configs 3 and 4 and the 8,192 share.
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
step d_bs06 300 $B --solver-opt beta_sufficient=0.6
step d_bs07 300 $B --solver-opt beta_sufficient=0.7
step d_bs08 300 $B --solver-opt beta_sufficient=0.8
step d_bs05bn09 300 $B --solver-opt beta_sufficient=0.5 --solver-opt beta_necessary=0.9
step d_air_bs05 300 $B --model aircond --solver-opt beta_sufficient=0.5
step d_air_bs07 300 $B --model aircond --solver-opt beta_sufficient=0.7
step d_s8192_bs05 300 $B --scens 8192 --solver-opt beta_sufficient=0.5
step d_s8192_bs07 300 $B --scens 8192 --solver-opt beta_sufficient=0.7
step d_cfg2_base 300 $B --scens 1024 --cm 10
step d_cfg2_bs05 300 $B --scens 1024 --cm 10 --solver-opt beta_sufficient=0.5
echo done
