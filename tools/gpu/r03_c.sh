#!/bin/bash
# Round 3, pass c: where the bench's extra 2.7 ms per step comes from (host profile).
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/prof_bench_loop.py > gpurun_out/c_prof.log 2>&1
echo "rc=$?"
grep "===" gpurun_out/c_prof.log
