#!/bin/bash
# Round 3, pass m: the IPM warm start (PH solves start from the last x / y) -- GPU tests,
# benches at the N=1 / 2 / 4 / 8 per-rank shares, and PMC byte passes for each share.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2; shift 2
    echo "=== $name (limit ${secs}s)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -2 "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
B="python3 -u bench.py --no-cpu-baseline"
T="python -u -m pytest -v -x --timeout 300 --timeout-method thread"
step m_tests 1200 $T -m gpu tests/test_gpu_ipm.py tests/test_gpu_readback.py tests/test_gpu_speculative.py tests/test_gpu_convergence.py tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_xhat_eval.py tests/test_dist_engine.py
step m_bench 300 $B
for S in 32768 16384 8192; do
  step m_s$S 300 $B --scens $S
done
step m_air8192 300 $B --model aircond --bf 4,32,64
P="python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline"
for S in 65536 32768 16384 8192; do
  step m_pmcf_$S 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/m_pmcf_$S -o run -- $P --scens $S
  step m_pmcw_$S 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/m_pmcw_$S -o run -- $P --scens $S
done
step m_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/m_trace -o run -- python3 bench.py --no-cpu-baseline
echo done
