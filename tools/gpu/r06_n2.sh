#!/bin/bash
# Round 6, pass n2: the 1,000-scenario UC line with its CPU baseline and the 125 share's line,
# then (last: rocprofv3 crashes at the exit of a process that made a cooperative launch, after
# writing its output) the 125 share's PMC WRITE_SIZE pass.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6n2
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
S='import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["value"],4), "mean_ms", round(d.get("ms_per_step_mean", d["ms_per_step"]),1), "launch", round(r["launch_ms"],1), "frac", r["frac"], "traffic", r.get("traffic"), r.get("kernel"), d["solver_iters_per_ph_iter"], "cpu", (d.get("cpu_baseline") or {}).get("value"))'
timeout -k 10 900 python3 -u bench.py --model uc --steps 2 --warmup 1 > $O/uc1000.log 2>&1; r=$?; echo "uc1000 rc=$r"; [ $r -eq 0 ] || { tail -20 $O/uc1000.log; exit 1; }
grep '^{' $O/uc1000.log | python3 -c "$S"
timeout -k 10 600 python3 -u bench.py --model uc --scens 125 --steps 3 --warmup 1 --no-cpu-baseline > $O/uc125.log 2>&1; r=$?; echo "uc125 rc=$r"; [ $r -eq 0 ] || { tail -20 $O/uc125.log; exit 1; }
grep '^{' $O/uc125.log | python3 -c "$S"
cd /tmp
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pw125 -o run -- python3 $R/tools/uc_prof.py 125 2048 125 > $R/$O/pw125.log 2>&1
echo "pmc write 125 rc=$? (a crash at exit after the output is written is the profiler's)"
grep "S=" $R/$O/pw125.log
echo done
