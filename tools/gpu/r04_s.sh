#!/bin/bash
# Round 4, pass s: two gloo ranks sharing the GPU (config 3 and config 2), the all-reduce split.
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out/s
export TMPDIR=/tmp
for a in "" "--scens 1024 --cm 10"; do
  timeout -k 10 400 python3 -u bench.py --gpus 2 --backend gloo --steps 10 --no-cpu-baseline $a > gpurun_out/s/gloo2.log 2>&1
  echo "gloo2 $a rc=$?"; grep '^{' gpurun_out/s/gloo2.log | tee -a gpurun_out/s/gloo2_lines.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), round(d['ms_per_step'],4), d['time_split_ms'], d['all_optimal'])"
done
