"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into profiles/<round>/pmc_summary_*.json."""
import csv, collections, json, sys
fetch_csv, write_csv, out_json, config = sys.argv[1:5]
out = {"command": "rocprofv3 --pmc {FETCH_SIZE|WRITE_SIZE} --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline",
       "config": config, "units": "KB per dispatch as reported by rocprofv3",
       "gfx950_correction": "FETCH_SIZE reads 1/2 of wide coalesced streaming reads (MI355X_MICROARCH.md HBM section): read bytes in [FETCH_SIZE, 2*FETCH_SIZE]*1024; WRITE_SIZE exact for 16-B stores",
       "kernels": {}}
for path, ctr in [(fetch_csv, "FETCH_SIZE"), (write_csv, "WRITE_SIZE")]:
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        # the first dispatch of the solve kernel is the cold Iter0 LP; report iterk separately
        d = {"dispatches": len(v), "mean_KB": sum(v) / len(v), "max_KB": max(v)}
        if len(v) > 1:
            d["mean_KB_after_first"] = sum(v[1:]) / (len(v) - 1)
        out["kernels"].setdefault(k, {})[ctr] = d
solve = [k for k in out["kernels"] if "k_solve" in k]
for k in solve:
    f = out["kernels"][k]["FETCH_SIZE"]
    w = out["kernels"][k]["WRITE_SIZE"]
    fr = f.get("mean_KB_after_first", f["mean_KB"]) * 1024
    wr = w.get("mean_KB_after_first", w["mean_KB"]) * 1024
    out.setdefault("solve_traffic_bytes_per_launch", {})[k] = {"read_lower": fr, "read_upper": 2 * fr, "write": wr,
                                                              "total_upper": 2 * fr + wr}
json.dump(out, open(out_json, "w"), indent=1)
print(json.dumps(out.get("solve_traffic_bytes_per_launch"), indent=1))
