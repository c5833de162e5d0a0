#!/bin/bash
# Round 6, pass x: the empty fallback launch with one workgroup instead of 16 (its dispatch
# cost is paid every PH iteration), A/B alternating; the perturbed-rho self-check on 2 ranks.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6x
mkdir -p $O
export TMPDIR=/tmp
S='import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "mean_ms", round(d.get("ms_per_step_mean", d["ms_per_step"]),4), "median", round(d.get("ms_per_step_median", d["ms_per_step"]),4), "launch", round(d["roofline"]["launch_ms"],4))'
b() { n=$1; shift; timeout -k 10 300 python3 -u bench.py --no-cpu-baseline "$@" > $O/$n.log 2>&1; r=$?; echo "$n rc=$r"; [ $r -eq 0 ] || { tail -20 $O/$n.log; exit $r; }; grep '^{' $O/$n.log | python3 -c "$S"; }
for rep in 1 2; do
  b s8192_fb16_$rep --scens 8192
  PHGPU_IPM_FB_BLOCKS=1 b s8192_fb1_$rep --scens 8192
  b s65536_fb16_$rep
  PHGPU_IPM_FB_BLOCKS=1 b s65536_fb1_$rep
done
timeout -k 10 400 python3 -u bench.py --gpus 2 --backend gloo --steps 4 --rho 1.02 --check on > $O/g2_bad.log 2>&1
echo "perturbed rho rc=$? (expect 3)"; grep '^{' $O/g2_bad.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d.get("checks") or {}; print({k: c.get(k) for k in ("world_size","all_ok","conv_ok","xbar_ok","W_ok")})'
echo done
