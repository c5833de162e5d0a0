"""CPU experiments on the path-6 kernel (TOOL ONLY): run PH on a farmer batch with the
generated IPM kernel compiled for the host (tests/ipm_host.py), x̄ / W in numpy, and
report the IPM iteration counts of every PH iteration (mean / max / histogram tail) and
the distance of x to a reference run.  A template file other than the library's can be
passed to try kernel variants without rebuilding the library.

    python tools/ipm_experiment.py [--S 2048] [--iters 8] [--tmpl path] [--eps-tight 1e-13]
                                   [-D NAME=VALUE ...]
"""
import argparse
import re
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy-1_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--S", type=int, default=2048)
    ap.add_argument("--model", choices=["farmer", "aircond"], default="farmer")
    ap.add_argument("--bf", default="8,8,16")
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--tmpl", default=os.path.join(ROOT, "mpi-sppy-1_amd", "csrc", "jit_ipm.hip.in"))
    ap.add_argument("--eps-tight", type=float, default=1e-13)
    ap.add_argument("--eps", type=float, default=1e-9)
    ap.add_argument("-D", action="append", default=[])
    ap.add_argument("--save", default=None)
    ap.add_argument("--ref", default=None)
    ap.add_argument("--warm", action="store_true", help="pass the previous x / y as x_in / y_in")
    ap.add_argument("--worst", type=int, default=0, help="print the slowest scenarios of this PH iteration")
    ap.add_argument("--trace", default=None, help="K:S -- print scenario S's iterations in PH iteration K")
    a = ap.parse_args()
    import ipm_host
    import mpisppy_amd._lib as L
    from mpisppy_amd.examples import farmer
    if a.model == "farmer":
        b = farmer.batch_creator(farmer.scenario_names_creator(a.S), crops_multiplier=1, num_scens=a.S)
    else:
        from mpisppy_amd.examples import aircond
        from bench import AIRCOND_KW
        bf = [int(v) for v in a.bf.split(",")]
        b = aircond.batch_creator(aircond.scenario_names_creator(int(np.prod(bf))), branching_factors=bf,
                                  **AIRCOND_KW)
        a.S = b.S
    src, _ = L.ipm_source(b)
    tmpl = open(a.tmpl).read()
    src = src[:src.index("// jit_ipm.hip.in --")] + tmpl
    for d in a.D:  # -D NAME=VALUE: replace the preamble's definition or add one
        name, val = (d.split("=", 1) + ["1"])[:2]
        line = f"#define {name} {val}\n"
        src, n = re.subn(rf"^#define {name} .*\n", line, src, count=1, flags=re.M)
        if not n:
            k = src.index("\n", src.index("#define IPM_GAM")) + 1  # (tests/ipm_host.py starts there)
            src = src[:k] + line + src[k:]
    orig = L.ipm_source
    L.ipm_source = lambda batch, lanes=1: (src, None)  # noqa: E731
    tk, ts = (int(v) if v != "all" else -2 for v in a.trace.split(":")) if a.trace else (-1, -1)
    k = src.index("\n", src.index("#define IPM_GAM")) + 1
    cond = "true" if ts == -2 else f"s == {ts}"
    tsrc = src[:k] + f"#define WTRACE(...) if ({cond}) printf(__VA_ARGS__)\n" + src[k:]
    try:
        nn = b.nn
        nc = b.nonant_col
        prob = b.prob
        rho = np.ones((a.S, nn))
        x, y, obj, bound, st, it = ipm_host.solve(b, eps_rel=a.eps, eps_tight=a.eps_tight)
        rows = [("iter0", it, st)]
        xs = [x]
        W = np.zeros((a.S, nn))
        for k in range(a.iters):
            xbar = np.zeros((a.S, nn))
            for kk in range(nn):  # x̄ per tree node of the nonant's depth (phbase.py:54-79)
                g = b.node_of[:, b.nonant_depth[kk]]
                num = np.bincount(g, prob * x[:, nc[kk]])
                den = np.bincount(g, prob)
                xbar[:, kk] = (num / np.where(den > 0, den, 1))[g]
            W = W + rho * (x[:, nc] - xbar)
            L.ipm_source = (lambda batch, lanes=1: (tsrc, None)) if k + 1 == tk else (lambda batch, lanes=1: (src, None))
            x, y, obj, bound, st, it = ipm_host.solve(b, W=W, rho=rho, xbar=xbar, eps_rel=a.eps,
                                                      eps_tight=a.eps_tight,
                                                      x_in=x if a.warm else None, y_in=y if a.warm else None)
            rows.append((f"ph{k + 1}", it, st))
            xs.append(x)
    finally:
        L.ipm_source = orig
    ref = np.load(a.ref) if a.ref else None
    for (name, it, st), k in zip(rows, range(len(rows))):
        ok = st == 0
        h = np.bincount(it[ok], minlength=1)
        tail = " ".join(f"{v}:{h[v]}" for v in range(max(0, len(h) - (99 if os.environ.get("FULLHIST") else 6)), len(h)) if h[v])
        dx = ""
        if ref is not None:
            dx = f"  max|x-ref| {np.abs(xs[k] - ref[k]).max():.2e}"
        wm = it[: len(it) // 64 * 64].reshape(-1, 64).max(1).mean() if len(it) >= 64 else float(it.max())
        print(f"{name:6s} mean {it[ok].mean():5.2f} max {it[ok].max():3d} wave-max {wm:5.2f} fail {int((~ok).sum()):4d}  tail {tail}{dx}")
    if a.worst:
        name, it, st = rows[a.worst]
        order = np.argsort(-it)[:8]
        print("slowest of", name, [(int(k), int(it[k])) for k in order])
    if a.save:
        np.save(a.save, np.stack(xs))


if __name__ == "__main__":
    main()
