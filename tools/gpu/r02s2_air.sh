#!/bin/bash
# Round 2 (session 2): restart-parameter sweep for aircond (config 4) and one UC (config 5)
# run with beta_sufficient 0.4 on the PH solves.
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
B="python3 -u bench.py --no-cpu-baseline --model aircond"
step a_bs01 300 $B --solver-opt beta_sufficient=0.1
step a_bs015 300 $B --solver-opt beta_sufficient=0.15
step a_ba05 300 $B --solver-opt beta_artificial=0.5
step a_ba07 300 $B --solver-opt beta_artificial=0.7
step a_bn09 300 $B --solver-opt beta_necessary=0.9
step a_bn07 300 $B --solver-opt beta_necessary=0.7
step u_bs04 900 python3 -u bench.py --no-cpu-baseline --model uc --scens 1000 --steps 2 --warmup 1 --solver-opt beta_sufficient=0.4
echo done
