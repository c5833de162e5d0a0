"""Generate the configuration-scale farmer fixtures (tests/golden/farmer_scale.json).

Run:  python tests/golden/make_golden_scale.py        (~20 minutes, one core)
      python tests/golden/make_golden_scale.py --cm10 (config 2's set only)
      python tests/golden/make_golden_scale.py --conv (farmer_conv.json: config 3 run to
                                                       convergence, ~30 minutes)

Source: oracle/farmer_vec.py, the vectorised exact restatement of farmer.py:85-224 and
PHBase.Iter0 / iterk_loop (phbase.py:758-979).  It is pinned by tests/test_oracle_scale.py:
its Iter0 LP matches scipy's HiGHS and its PH subproblem matches lpqp.farmer_prox_exact
(which reproduces the reference's w_test_data fixtures) on samples of every set below.

Sets (SURVEY.md 8(c) "golden vectors to commit"):
  farmer65536_cm1   config 3: scen0..scen65535, cm=1, rho=1 -- trivial bound, Iter0
                    objectives and W after 5 PH iterations on every 64th scenario, x̄ and
                    conv of each of the 5 iterations, E[obj] after 5
  farmer1024_cm10   config 2: scen0..scen1023, cm=10 -- trivial bound, sampled Iter0 objectives,
                    x̄ / conv of 5 PH iterations, W of every 8th scenario and E[obj] after them;
                    "breaks": the PH iteration at which iterk_loop stops for conv < 1e-2 and
                    1e-3 (phbase.py:925-934), with x̄ at that iteration and its neighbours
  farmer2048_cm64   the HBM-scale variant of config 3 at test size: the first 2048
                    well-conditioned scenarios from scen3 on, cm=64, 5 PH iterations.
                    scen0..2 are skipped (with cm > 1 their crop copies tie exactly, so
                    their Iter0 LP optimum is a face and only the objective is
                    solver-independent), and so are the ~1.3% whose Iter0 LP has a near-tie
                    (lp_margin < 1e-2: two crops' yields within ~1e-4, e.g. scen411 at 2e-4),
                    where a first-order method needs ~1/margin iterations to pick the vertex
  farmer_cm64_neartie  Iter0 objectives of the near-tied scenarios below 1e-3 margin among
                    scen3..scen6002 (objective-only parity)
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import farmer_vec as fv  # noqa: E402
from oracle.farmer_vec import FarmerVecPH  # noqa: E402


def well_conditioned(start, count, cm, margin=1e-2):
    names, lo = [], start
    while len(names) < count:
        chunk = [f"scen{i}" for i in range(lo, lo + 2 * count)]
        bp, sl, _ = fv.pieces(fv.yields(chunk, cm), cm)
        mg = fv.lp_margin(bp, sl, 500.0 * cm)
        names += [nm for nm, g in zip(chunk, mg) if g >= margin]
        lo += 2 * count
    return names[:count]


def run(names, cm, iters, stride, num_scens=None):
    t0 = time.time()
    ph = FarmerVecPH(names, cm, rho=1.0, num_scens=num_scens)
    tb = ph.iter0()
    sample = list(range(0, len(names), stride))
    out = {"names_first": names[0], "names_last": names[-1], "S": len(names), "crops_multiplier": cm,
           "rho": 1.0, "trivial_bound": tb, "sample": sample,
           "iter0_obj": ph.iter0_obj[sample].tolist(), "iter0_x": ph.iter0_x[sample].tolist()}
    if iters:
        ph.iterk_loop(iters)
        out["ph_iters"] = iters
        out["conv"] = [h["conv"] for h in ph.history]
        out["xbar"] = [h["xbar"].tolist() for h in ph.history]
        out["W"] = ph.W[sample].tolist()
        out["x"] = ph.x[sample].tolist()
        out["Eobj"] = ph.Eobjective()
    print(f"{len(names)} scen cm={cm}: tb {tb:.10f}  ({time.time() - t0:.1f}s)", flush=True)
    return out


CONV_THRESH = (1e-2, 3e-3, 1e-3)


def run_to_convergence(S=65536, limit=4000, stride=64):
    """farmer_conv.json: config 3 (scen0..scen65535, cm=1, rho=1) run by iterk_loop until
    conv < 1e-3 (phbase.py:925-934).  For every threshold of CONV_THRESH: the PH iteration
    at which the loop breaks, and x̄ plus the W of every ``stride``-th scenario at that
    iteration and its two neighbours (so a run that breaks one iteration off is compared
    against its own iteration); the whole conv trajectory."""
    t0 = time.time()
    ph = FarmerVecPH([f"scen{i}" for i in range(S)], 1, rho=1.0)
    tb = ph.iter0()
    sample = list(range(0, S, stride))
    conv, hit, kept, prev = [], {}, {thr: {} for thr in CONV_THRESH}, None
    it = 0
    while it < limit:
        it += 1
        xb = ph.compute_xbar()                                   # phbase.py:909
        ph.W += ph.rho * (ph.x - ph.xbar)                        # :913
        c = float(np.abs(ph.x - ph.xbar).sum() / (ph.S * ph.K))  # :916
        conv.append(c)
        snap = (xb.tolist(), ph.W[sample].tolist())
        for thr in CONV_THRESH:
            if thr in hit and it == hit[thr] + 1:
                kept[thr][it] = snap
            if thr not in hit and c < thr:
                hit[thr] = it
                kept[thr][it] = snap
                if prev is not None:
                    kept[thr][it - 1] = prev
        prev = snap
        if len(hit) == len(CONV_THRESH) and it > hit[CONV_THRESH[-1]]:
            break
        ph.x, ph.obj = fv.prox(ph.bp, ph.sl, ph.f0, ph.W, ph.xbar, ph.rho, ph.total)   # :941
        if it % 100 == 0:
            print(f"  iteration {it}: conv {c:.6g} ({time.time() - t0:.0f}s)", flush=True)
    out = {"S": S, "crops_multiplier": 1, "rho": 1.0, "trivial_bound": tb, "sample": sample,
           "conv": conv, "breaks": {}}
    for thr in CONV_THRESH:
        out["breaks"][repr(thr)] = {"iteration": hit[thr],
                                    "xbar": {str(j): v[0] for j, v in sorted(kept[thr].items())},
                                    "W": {str(j): v[1] for j, v in sorted(kept[thr].items())}}
    print(f"{S} scen to conv < {CONV_THRESH[-1]}: breaks {hit} ({time.time() - t0:.0f}s)", flush=True)
    with open(os.path.join(HERE, "farmer_conv.json"), "w") as f:
        json.dump(out, f)


def breaks(names, cm, thresholds=(1e-2, 1e-3), limit=3000):
    """PH iteration counts of iterk_loop's break for each threshold, x̄ around each."""
    ph = FarmerVecPH(names, cm, rho=1.0)
    ph.iter0()
    ph.iterk_loop(limit, convthresh=min(thresholds))
    conv = [h["conv"] for h in ph.history]
    out = {}
    for thr in thresholds:
        it = next(i + 1 for i, c in enumerate(conv) if c < thr)
        out[repr(thr)] = {"iteration": it,
                          "xbar": {str(j): ph.history[j - 1]["xbar"].tolist()
                                   for j in (it - 1, it, it + 1) if 1 <= j <= len(conv)}}
    return {"conv": conv, "breaks": out}


def main():
    if "--conv" in sys.argv:
        return run_to_convergence()
    if "--cm10" in sys.argv:  # regenerate config 2's set only
        path = os.path.join(HERE, "farmer_scale.json")
        out = json.load(open(path))
        out["farmer1024_cm10"] = run([f"scen{i}" for i in range(1024)], 10, 5, 8)
        out["farmer1024_cm10"].update(breaks([f"scen{i}" for i in range(1024)], 10))
        with open(path, "w") as f:
            json.dump(out, f)
        return
    out = {}
    out["farmer65536_cm1"] = run([f"scen{i}" for i in range(65536)], 1, 5, 64)
    out["farmer1024_cm10"] = run([f"scen{i}" for i in range(1024)], 10, 5, 8)
    out["farmer1024_cm10"].update(breaks([f"scen{i}" for i in range(1024)], 10))
    names64 = well_conditioned(3, 2048, 64)
    out["farmer2048_cm64"] = run(names64, 64, 5, 16)
    out["farmer2048_cm64"]["names"] = names64
    chunk = [f"scen{i}" for i in range(3, 6003)]
    bp, sl, f0 = fv.pieces(fv.yields(chunk, 64), 64)
    mg = fv.lp_margin(bp, sl, 500.0 * 64)
    tied = [nm for nm, g in zip(chunk, mg) if g < 1e-3]
    _, obj = fv.iter0_lp(*fv.pieces(fv.yields(tied, 64), 64), 500.0 * 64)
    out["farmer_cm64_neartie"] = {"names": tied, "margin": [float(g) for g in mg[mg < 1e-3]],
                                  "iter0_obj": obj.tolist()}
    with open(os.path.join(HERE, "farmer_scale.json"), "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
