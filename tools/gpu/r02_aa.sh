#!/bin/bash
# longest-first queue for the register path: A/B on config 3, the 8,192 share and config 4, then parity tests
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 300 "$@" > gpurun_out/$name.log 2>&1 || exit 1
  echo "$name $(tail -1 gpurun_out/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), round(d["ms_per_step"],4), d["time_split_ms"])')"
}
B="python3 bench.py --no-cpu-baseline"
run ord0_cfg3 env PHGPU_ORDER=0 $B
run ord1_cfg3 $B
run ord0_s8192 env PHGPU_ORDER=0 $B --scens 8192
run ord1_s8192 $B --scens 8192
run ord0_air env PHGPU_ORDER=0 $B --model aircond
run ord1_air $B --model aircond
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_xhat_eval.py tests/test_dist_engine.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests_order.log 2>&1
rc=$?; tail -2 gpurun_out/gputests_order.log; exit $rc
