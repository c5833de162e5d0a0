#!/bin/bash
# Round 2 (session 2): path 4 with the slice metadata loaded one slice ahead: per-iteration
# time on 512 UC scenarios, path-4 GPU tests.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -2 "gpurun_out/$name.log" | cut -c1-200
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
step pf_prof 300 python -u tools/uc_prof.py 512 2048
step pf_prof64 300 python -u tools/uc_prof.py 64 2048
step pf_tests 900 python -u -m pytest tests/test_gpu_uc.py tests/test_dist_uc.py -x -v --timeout 300 --timeout-method thread
echo done
