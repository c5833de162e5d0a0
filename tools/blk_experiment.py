"""CPU experiments on the subtree interior point (TOOL ONLY): PH on farmer cm = 10 (config
2's instance by default) with the generated k_solve_ipm_blk compiled for the host
(tests/ipm_wave_host.py), x̄ / W in numpy, warm starts as the GPU loop passes them.  Prints
per PH iteration the IPM iteration counts (mean / max / tail), fallbacks, jam hand-overs
and re-centrings (stats[6] / stats[7]), and the worst nonant error against the exact
farmer oracle's proximal solve (oracle/farmer_vec.py).

    python tools/blk_experiment.py [--S 1024] [--cm 10] [--iters 6] [-D NAME=VALUE ...]
"""
import argparse
import os
import re
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy-1_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--S", type=int, default=1024)
    ap.add_argument("--cm", type=int, default=10)
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--lanes", type=int, default=64, help="threads per scenario (64 WPS)")
    ap.add_argument("--sub", type=int, default=0, help="solve only every k-th scenario (x̄ from the oracle)")
    ap.add_argument("-D", action="append", default=[])
    ap.add_argument("--tmpl", default=None)
    ap.add_argument("--save", default=None)
    ap.add_argument("--trace", type=int, default=0, help="trace the slowest scenario of this PH iteration")
    ap.add_argument("--cold", action="store_true", help="every PH solve starts cold (no x_in / y_in)")
    a = ap.parse_args()
    import ipm_wave_host
    import mpisppy_amd._lib as L
    from mpisppy_amd.examples import farmer
    from oracle import farmer_vec as fv
    names = farmer.scenario_names_creator(a.S)
    b = farmer.batch_creator(names, crops_multiplier=a.cm, num_scens=a.S)
    src, _ = L.ipm_source(b, a.lanes)
    if a.tmpl:
        tmpl = open(a.tmpl).read()
        k = src.index("// jit_ipm_blk.hip.in --")
        src = src[:k] + tmpl
    for d in a.D:
        name, val = (d.split("=", 1) + ["1"])[:2]
        line = f"#define {name} {val}\n"
        src, n = re.subn(rf"^#define {name} .*\n", line, src, count=1, flags=re.M)
        if not n:
            src = line + src
    orig = L.ipm_source
    L.ipm_source = lambda batch, lanes=1: (src, None)  # noqa: E731
    nn, nc = b.nn, b.nonant_col
    # W / x̄ of each PH iteration from the exact oracle over all S scenarios (what the GPU
    # run reproduces to ~1e-8); the emulated kernel solves the subset every --sub-th
    # scenario, warm-started from its own previous solve as on the GPU
    oph = fv.FarmerVecPH(names, a.cm)
    oph.iter0()
    sub = np.arange(0, a.S, max(1, a.sub))
    bs = b.subset(sub) if hasattr(b, "subset") else farmer.batch_creator([names[i] for i in sub], crops_multiplier=a.cm,
                                                                         num_scens=a.S)
    S = len(sub)
    rho = np.ones((S, nn))
    try:
        t0 = time.time()
        st8 = []
        x, y, obj, bound, st, it = ipm_wave_host.solve(bs, lanes=a.lanes, eps_rel=1e-10, stats=st8)
        print(f"iter0 ({S} scenarios) {time.time() - t0:.1f}s mean {it[st == 0].mean():.2f} max {it.max()} "
              f"fail {(st != 0).sum()}", flush=True)
        allit = []
        for k in range(a.iters):
            oph.iterk_loop(1)
            W, xbar = oph.W[sub], oph.xbar[sub]
            st8 = []
            t0 = time.time()
            xprev, yprev = x, y
            x, y, obj, bound, st, it = ipm_wave_host.solve(bs, lanes=a.lanes, W=W, rho=rho, xbar=xbar,
                                                           x_in=None if a.cold else x, y_in=None if a.cold else y,
                                                           stats=st8)
            xv = oph.x[sub]
            ok = st == 0
            err = np.abs(x[:, nc] - xv).max(1)
            h = np.bincount(it[ok])
            allit.append(it.copy())
            tail = " ".join(f"{v}:{h[v]}" for v in range(max(0, len(h) - 6), len(h)) if h[v])
            print(f"ph{k + 1} {time.time() - t0:.1f}s mean {it[ok].mean():.2f} max {it[ok].max()} "
                  f"fail {(~ok).sum()} jam {int(st8[0][6])} recentre {int(st8[0][7])} "
                  f"max|x-oracle| (solved) {err[ok].max():.2e}  tail {tail}", flush=True)
            if a.trace == k + 1:
                i = int(np.argmax(st != 0)) if (st != 0).any() else int(np.argmax(it))
                tsrc = "#include <stdio.h>\n#define WTRACE(...) if (threadIdx.x == 0) printf(__VA_ARGS__)\n" + src
                L.ipm_source = lambda batch, lanes=1: (tsrc, None)  # noqa: E731
                one = farmer.batch_creator([names[sub[i]]], crops_multiplier=a.cm, num_scens=a.S)
                print("trace of", names[sub[i]], "iterations", int(it[i]), flush=True)
                ipm_wave_host.solve(one, lanes=a.lanes, W=W[i:i + 1], rho=rho[i:i + 1], xbar=xbar[i:i + 1], x_in=xprev[i:i + 1],
                                    y_in=yprev[i:i + 1])
                L.ipm_source = lambda batch, lanes=1: (src, None)  # noqa: E731
            # a scenario left to the fallback continues from the oracle's solution (the PDHG's)
            x[np.ix_(~ok, nc)] = xv[~ok]
        if a.save:
            np.save(a.save, np.array(allit))
    finally:
        L.ipm_source = orig


if __name__ == "__main__":
    main()
