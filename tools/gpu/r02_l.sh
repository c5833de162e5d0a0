#!/bin/bash
# path 4 profile: concurrency sweep + PMC bytes per scenario-iteration (fixed 4096 iterations)
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ne 0 ]; then exit $rc; fi
}
for S in 1 16 64 256 512 1000; do step ucprof_S$S 300 python -u tools/uc_prof.py $S 2048; done
step pmc_fetch_uc 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_uc -o run -- python3 tools/uc_prof.py 512 2048
step pmc_write_uc 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_uc -o run -- python3 tools/uc_prof.py 512 2048
step pmc_sq_uc 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/pmc_sq_uc -o run -- python3 tools/uc_prof.py 512 2048
echo done
