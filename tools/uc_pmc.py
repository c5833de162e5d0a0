"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of tools/uc_prof.py (one cold
path-4 solve of S UC scenarios capped at K PDHG iterations) into the per-scenario-iteration
byte summary bench.py reads for config 5 (profiles/<round>/pmc_summary_uc<S>.json).

    python tools/uc_pmc.py FETCH_CSV WRITE_CSV UC_PROF_LOG OUT_JSON S K

The solve kernel is every dispatch whose name starts with "void k_solve_stream" (the queue
form k_solve_stream<2>, or the cluster form k_solve_stream<1, true> for a batch smaller
than the GPU); the scenario-iterations come from uc_prof.py's log line.  gfx950 correction
(MI355X_MICROARCH.md): FETCH_SIZE counts half of wide streaming reads, so the read bytes lie
in [FETCH_SIZE, 2 FETCH_SIZE]; WRITE_SIZE is exact.
"""
import collections
import csv
import json
import re
import sys

fetch_csv, write_csv, log, out_json, S, K = sys.argv[1:7]
m = re.search(r"scenario-iterations (\d+)", open(log).read())
units = int(m.group(1))
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for path, ctr in [(fetch_csv, "FETCH_SIZE"), (write_csv, "WRITE_SIZE")]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if k.startswith("void k_solve_stream") or k.startswith("k_solve_stream"):
            tot[k.split("(")[0]][ctr] += float(r["Counter_Value"]) * 1024.0
assert len(tot) == 1, dict(tot)
kname, c = next(iter(tot.items()))
if not kname.startswith("void "):
    kname = "void " + kname
rd = c["FETCH_SIZE"] / units
wr = c["WRITE_SIZE"] / units
out = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) of tools/uc_prof.py {S} {K}: one cold "
                 f"solve of {S} UC scenarios capped at {K} PDHG iterations = {units} scenario-iterations",
       "kernel": kname, "scenario_iterations": units,
       "bytes_per_scenario_iter": {"read_lower": rd, "read_upper": 2 * rd, "write": wr, "total_upper": 2 * rd + wr},
       "note": "path 4 streams the same bytes every iteration, so bytes per scenario-iteration carry over to the "
               "config 5 bench (x scenario-iterations per launch)"}
json.dump(out, open(out_json, "w"), indent=1)
print(json.dumps(out, indent=1))
