#!/bin/bash
# round-2 measurement pass after path 4: GPU suite, smoke, headline bench, config 5 bench
# (with its CPU baseline), kernel trace of config 5, PMC bytes of path 4
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
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
step gputests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_farmer65536_cm1 300 python -u bench.py
step bench_uc1000 900 python -u bench.py --model uc --steps 2 --warmup 1
step prof_uc 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_uc -o run -- python3 bench.py --model uc --steps 1 --warmup 0 --no-cpu-baseline
step pmc_fetch_uc 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_uc -o run -- python3 tools/uc_prof.py 512 2048
step pmc_write_uc 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_uc -o run -- python3 tools/uc_prof.py 512 2048
echo done
