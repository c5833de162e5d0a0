#!/bin/bash
# Round 2 (session 2): path 4 with fp32 gathered vectors (PHGPU_STREAM_F32=1) vs fp64:
# per-iteration time at 512 scenarios, cold iteration counts on 64, path-4 GPU tests;
# config 3 bench after reverting the side-stream snapshot.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -3 "gpurun_out/$name.log" | cut -c1-250
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
step v_bench_cfg3 300 python3 -u bench.py --no-cpu-baseline
step p_f64 300 python -u tools/uc_prof.py 512 2048
PHGPU_STREAM_F32=1 step p_f32 300 python -u tools/uc_prof.py 512 2048
step s_f64 300 python -u tools/uc_sweep.py 64
PHGPU_STREAM_F32=1 step s_f32 300 python -u tools/uc_sweep.py 64
PHGPU_STREAM_F32=1 step t_f32 600 python -u -m pytest tests/test_gpu_uc.py -x -v --timeout 300 --timeout-method thread
echo done
