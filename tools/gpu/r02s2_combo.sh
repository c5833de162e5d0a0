#!/bin/bash
# Round 2 (session 2): farmer's recommended option combined with the artificial-restart /
# necessary-decay changes (config 3, config 2, 8,192 share).
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
step k_base 300 $B
step k_ba02 300 $B --solver-opt beta_artificial=0.2
step k_ba025 300 $B --solver-opt beta_artificial=0.25
step k_bn09 300 $B --solver-opt beta_necessary=0.9
step k_cfg2_ba02 300 $B --scens 1024 --cm 10 --solver-opt beta_artificial=0.2
step k_s8192_ba02 300 $B --scens 8192 --solver-opt beta_artificial=0.2
echo done
