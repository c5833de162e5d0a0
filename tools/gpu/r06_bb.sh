#!/bin/bash
# Round 6, pass bb: RCCL collectives inside the engine's multi-rank path (one-rank nccl group
# under the loopback communicator): step time and the trace of one step.
cd "$(dirname "$0")/../.." || exit 1
O=gpurun_out/r6bb
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u tools/fake_ranks.py 8 100 rccl > $O/rccl.log 2>&1; r=$?; echo "rccl rc=$r"; grep -E "loopback" $O/rccl.log | cut -c1-160; [ $r -eq 0 ] || { tail -20 $O/rccl.log; exit 1; }
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/trccl -o run -- python3 $R/tools/fake_ranks.py 8 20 rccl > $R/$O/trccl.log 2>&1 || { echo "trace failed"; tail -5 $R/$O/trccl.log; exit 1; }
cd $R
f=$(find $O/trccl -name "*kernel_trace.csv" | head -1); python3 - $f <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda d: int(d["Start_Timestamp"]))
names = {}
for d in rows:
    k = d["Kernel_Name"][:60]; names.setdefault(k, []).append((int(d["End_Timestamp"]) - int(d["Start_Timestamp"])) / 1e3)
for k, v in sorted(names.items(), key=lambda kv: -len(kv[1]))[:12]:
    print(f"{len(v):6d} {sum(v)/len(v):8.2f} us  {k}")
PY
echo done
