set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1
echo "bench rc=$?" >> gpurun_out/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof.log 2>&1
echo "prof rc=$?" >> gpurun_out/prof.log
python tools/trace_summary.py gpurun_out/prof/run_kernel_trace.csv 10 gpurun_out/prof/solve_dispatches.json >> gpurun_out/prof.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1
echo "pmc fetch rc=$?" >> gpurun_out/pmc_fetch.log
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1
echo "pmc write rc=$?" >> gpurun_out/pmc_write.log
