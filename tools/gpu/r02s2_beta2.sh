#!/bin/bash
# Round 2 (session 2): restart-parameter sweep, second pass (config 3, config 4, 8,192 share).
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
step c_bs04 300 $B --solver-opt beta_sufficient=0.4
step c_bs05 300 $B --solver-opt beta_sufficient=0.5
step c_ba01 300 $B --solver-opt beta_artificial=0.1
step c_ba015 300 $B --solver-opt beta_artificial=0.15
step c_bs03ba02 300 $B --solver-opt beta_sufficient=0.3 --solver-opt beta_artificial=0.2
step c_bs04ba02 300 $B --solver-opt beta_sufficient=0.4 --solver-opt beta_artificial=0.2
step c_bs03ba015 300 $B --solver-opt beta_sufficient=0.3 --solver-opt beta_artificial=0.15
step c_air_base 300 $B --model aircond
step c_air_bs03ba02 300 $B --model aircond --solver-opt beta_sufficient=0.3 --solver-opt beta_artificial=0.2
step c_s8192_base 300 $B --scens 8192
step c_s8192_bs03ba02 300 $B --scens 8192 --solver-opt beta_sufficient=0.3 --solver-opt beta_artificial=0.2
echo done
