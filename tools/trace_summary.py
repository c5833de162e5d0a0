"""Per-dispatch durations of the solve kernel from a rocprofv3 --kernel-trace csv.

The --stats average mixes the cold Iter0 LP launch and the warmup PH launches with the
timed ones; bench.py times the last K launches (K = --steps).  This prints the mean of
the last K solve dispatches so the two can be compared like for like.
usage: python tools/trace_summary.py run_kernel_trace.csv K out.json"""
import csv
import json
import sys

path, k, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
rows = [r for r in csv.DictReader(open(path)) if "k_solve" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
name = rows[-1]["Kernel_Name"].split("(")[0] if rows else None
res = {"kernel": name, "dispatches_ms": dur, "timed_last_k": k,
       "mean_ms_last_k": sum(dur[-k:]) / max(1, len(dur[-k:])),
       "mean_ms_all": sum(dur) / max(1, len(dur)),
       "vgpr": rows[-1]["VGPR_Count"] if rows else None,
       "lds_bytes": rows[-1]["LDS_Block_Size"] if rows else None,
       "scratch": rows[-1]["Scratch_Size"] if rows else None,
       "grid": rows[-1]["Grid_Size_X"] if rows else None,
       "workgroup": rows[-1]["Workgroup_Size_X"] if rows else None}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
