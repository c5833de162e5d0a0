#!/bin/bash
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -2 "gpurun_out/$name.log" | cut -c1-600
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 bench.py --no-cpu-baseline"
step wgtests 300 python -u -m pytest tests/test_gpu_wg.py tests/test_gpu_parity.py tests/test_xhat_eval.py -v --timeout 120 --timeout-method thread
step bench_cm64 400 $B --cm 64 --steps 5 --warmup 2
step bench_cfg2 300 $B --scens 1024 --cm 10
step pmc_fetch_cm64 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_cm64b -o run -- $B --cm 64 --steps 3 --warmup 1
step pmc_write_cm64 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_cm64b -o run -- $B --cm 64 --steps 3 --warmup 1
echo done
