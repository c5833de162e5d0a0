#!/bin/bash
# N=8 share (8,192 farmer scenarios per GPU): solve time vs check / restart periods
cd "$(dirname "$0")/../.." || exit 1
mkdir -p gpurun_out
for X in "" "check_every=32" "check_every=32,restart_every=8" "check_every=16,restart_every=8"; do
  timeout -k 10 120 python -u tools/kbench.py 8192 1 16 $X > gpurun_out/n8_$X.log 2>&1 || exit 1
  echo "[$X] $(tail -1 gpurun_out/n8_$X.log)"
done
