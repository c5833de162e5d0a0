"""Queue-order study of the register path's persistent kernel: list
scheduling of per-scenario PDHG iteration counts on the resident scenario groups, in
iteration units (a wave runs its groups in lockstep, so a launch lasts about as long as
its latest-finishing group).  Input: the counts of consecutive PH iterations dumped by
tools/dump_iters.py (profiles/r02/s2/iters_S65536.npz: farmer cm=1, 40 PH iterations).

    python tools/sim_queue.py [npz] [resident groups = 32768]"""
import heapq
import sys

import numpy as np


def makespan(order, dur, G):
    fin = list(dur[order[:G]])
    heapq.heapify(fin)
    for s in order[G:]:
        heapq.heappush(fin, heapq.heappop(fin) + dur[s])
    return max(fin)


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "profiles/r02/s2/iters_S65536.npz"
    G = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
    z = np.load(path)
    it = z["iters"].astype(np.int64) * int(z["unit"])
    K, S = it.shape
    lpt = lambda key: np.argsort(-key, kind="stable")  # noqa: E731
    res = {"scenario order": [], "previous count": [], "EMA 0.3 (kernel)": [], "exact (oracle)": [],
           "lower bound": []}
    ema = it[0].astype(np.int64)
    for k in range(1, K):
        d = it[k].astype(float)
        if k >= 3:
            res["scenario order"].append(makespan(np.arange(S), d, G))
            res["previous count"].append(makespan(lpt(it[k - 1]), d, G))
            res["EMA 0.3 (kernel)"].append(makespan(lpt(ema), d, G))
            res["exact (oracle)"].append(makespan(lpt(it[k]), d, G))
            res["lower bound"].append(max(d.max(), d.sum() / G))
        ema = (7 * ema + 3 * it[k] + 5) // 10  # the kernel's update (solve_reg.inc)
    base = np.mean(res["scenario order"])
    for k, v in res.items():
        print(f"{k:18s} mean makespan {np.mean(v):7.1f} iterations ({np.mean(v) / base - 1:+.1%})")


if __name__ == "__main__":
    main()
