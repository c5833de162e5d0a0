"""Pack the reference's UC data for the GPU box (where /root/reference does not exist).

Parses paperruns/larger_uc/RootNode.dat with the model's own reader and stores the
parsed parameters and sets as uc_data/rootnode.json, and packs the wind bounds of
paperruns/larger_uc/1000scenarios_wind/Node1..1000.dat -- the only scenario data --
into uc_data/wind_1000scen.npz (lo/hi [node, gen, t]).  Both hold exactly what reading
the .dat files gives (tests/test_uc.py compares them with the files when
/root/reference is present).
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy-1_amd"))
from mpisppy_amd.utils.datfile import load_dat, dump_data  # noqa: E402

SRC = "/root/reference/paperruns/larger_uc"
DST = os.path.join(ROOT, "mpi-sppy-1_amd", "mpisppy_amd", "examples", "uc_data")


def main():
    os.makedirs(DST, exist_ok=True)
    p, s = load_dat(os.path.join(SRC, "RootNode.dat"))
    with open(os.path.join(DST, "rootnode.json"), "w") as f:
        json.dump(dump_data(p, s), f, separators=(",", ":"))
    wdir = os.path.join(SRC, "1000scenarios_wind")
    nodes = sorted(int(f[4:-4]) for f in os.listdir(wdir) if f.startswith("Node") and f.endswith(".dat"))
    p0, s0 = load_dat(os.path.join(SRC, "RootNode.dat"))
    T = int(p0["NumTimePeriods"])
    gens = sorted({g for (g, _) in load_dat(os.path.join(wdir, f"Node{nodes[0]}.dat"))[0]["MaxNondispatchablePower"]})
    lo = np.zeros((len(nodes), len(gens), T))
    hi = np.zeros((len(nodes), len(gens), T))
    for k, nd in enumerate(nodes):
        p, _ = load_dat(os.path.join(wdir, f"Node{nd}.dat"))
        for i, g in enumerate(gens):
            for t in range(T):
                lo[k, i, t] = p["MinNondispatchablePower"][(g, t + 1)]
                hi[k, i, t] = p["MaxNondispatchablePower"][(g, t + 1)]
    np.savez_compressed(os.path.join(DST, "wind_1000scen.npz"), node=np.array(nodes, dtype=np.int64),
                        gens=np.array(gens), lo=lo, hi=hi)
    print(f"packed {len(nodes)} nodes x {len(gens)} nondispatchable x {T} periods into {DST}")


if __name__ == "__main__":
    main()
