#!/bin/bash
# Round 6, pass n: config 5's traffic re-measured on this round's path-4 kernels (PMC
# FETCH_SIZE / WRITE_SIZE, separate passes, of a cold capped solve: the queue form at 1,000
# scenarios and the cluster form at the 125-scenario share), then the 1,000-scenario bench
# line with its CPU baseline and the 125 share's line; first the split / cluster tests and the
# (pass n2: the 125 share's PMC again, the 1,000 line; two slices per wave trip measured slower.)
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6n
mkdir -p $O profiles/r06
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
S='import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"],4), "mean_ms", round(d.get("ms_per_step_mean", d["ms_per_step"]),1), "launch", round(r["launch_ms"],1), "frac", r["frac"], "traffic", r.get("traffic"), r.get("kernel"), d["solver_iters_per_ph_iter"], "cpu", (d.get("cpu_baseline") or {}).get("value"))'
for sc in "125 2048 125"; do
  set -- $sc
  cd /tmp
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pf$1 -o run -- python3 $R/tools/uc_prof.py $1 $2 $3 > $R/$O/pf$1.log 2>&1 || { echo "pmc fetch $1 failed"; tail -5 $R/$O/pf$1.log; exit 1; }
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pw$1 -o run -- python3 $R/tools/uc_prof.py $1 $2 $3 > $R/$O/pw$1.log 2>&1 || { echo "pmc write $1 failed"; tail -5 $R/$O/pw$1.log; exit 1; }
  cd $R
  f=$(find $O/pf$1 -name "*counter_collection.csv" | head -1); w=$(find $O/pw$1 -name "*counter_collection.csv" | head -1)
  python3 tools/uc_pmc.py $f $w $O/pf$1.log $O/pmc_summary_uc$1.json $1 $2 | tail -8 || exit 1
  cp $O/pmc_summary_uc$1.json profiles/r06/
  grep "S=" $O/pf$1.log
done
timeout -k 10 900 python3 -u bench.py --model uc --steps 2 --warmup 1 > $O/uc1000.log 2>&1; r=$?; echo "uc1000 rc=$r"; [ $r -eq 0 ] || { tail -20 $O/uc1000.log; exit 1; }
grep '^{' $O/uc1000.log | python3 -c "$S"
timeout -k 10 600 python3 -u bench.py --model uc --scens 125 --steps 3 --warmup 1 --no-cpu-baseline > $O/uc125.log 2>&1; r=$?; echo "uc125 rc=$r"; [ $r -eq 0 ] || { tail -20 $O/uc125.log; exit 1; }
grep '^{' $O/uc125.log | python3 -c "$S"
echo done
