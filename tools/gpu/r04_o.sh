#!/bin/bash
# Round 4, pass o: the 8,192 share with / without the folded step and the complementarity stop.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline "$@" > gpurun_out/o_b.log 2>&1
  echo "bench $* [$PHGPU_FUSE_STEP|$PHGPU_IPM_DEFS] rc=$?"; grep '^{' gpurun_out/o_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4), round(d['time_split_ms']['solve_launch'],4), d['solver_iters_per_ph_iter'], d['all_optimal'])"
}
run --scens 8192
PHGPU_FUSE_STEP=0 run --scens 8192
PHGPU_IPM_DEFS="IPM_XACC=0" run --scens 8192
PHGPU_FUSE_STEP=0 PHGPU_IPM_DEFS="IPM_XACC=0" run --scens 8192
run
PHGPU_FUSE_STEP=0 run
