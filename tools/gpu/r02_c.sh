#!/bin/bash
# Round 2, pass C: cm=64 parity on the well-conditioned fixture set + near-tie check,
# lane sweep at the N=8 share (8,192 scenarios), WPS sweep at cm=64.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -4 "gpurun_out/$name.log"
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
step wgtests 300 python -u -m pytest tests/test_gpu_wg.py -v --timeout 120 --timeout-method thread
step lanes8192 300 python -u tools/kbench.py 8192 1 8,16,32,64
step lanes65536 300 python -u tools/kbench.py 65536 1 4,8
step wps_cm64_4 300 env PHGPU_WPS=4 python -u tools/kbench.py 16384 64
step wps_cm64_8 300 env PHGPU_WPS=8 python -u tools/kbench.py 16384 64
step wps_cm64_2 300 env PHGPU_WPS=2 python -u tools/kbench.py 16384 64
echo done
