"""Per-phase cycle profile of the lane-group interior point (TOOL ONLY, diagnostics).

Builds the path-6 module with IPM_PROF=1 (jit_ipm_ml.hip.in: s_memtime at the phase
boundaries of the iteration loop, summed per wave), runs farmer PH on S scenarios with L
lanes per scenario, and prints the mean cycles per loop trip of each phase over the timed
PH iterations, with the plain module's step time beside it.

    python tools/ipm_prof.py S L [--iters 10] [--defs "IPM_X=..;"]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy-1_amd"))
sys.path.insert(0, ROOT)

PHASES = ["slacks+mu", "Ax+Aty+pq", "kkt", "assembly", "factor", "rhs+solve", "dx+dw", "step+update"]


def run(S, L, iters, defs, prof, level=1):
    os.environ["PHGPU_IPM_LANES"] = str(L)
    if prof:
        os.environ["PHGPU_IPM_PROF"] = "1"
    d = (defs + ";" if defs else "") + (f"IPM_PROF={level}" if prof else "")
    if d:
        os.environ["PHGPU_IPM_DEFS"] = d
    else:
        os.environ.pop("PHGPU_IPM_DEFS", None)
    import torch
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer
    opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": 5, "defaultPHrho": 1.0, "convthresh": -1.0,
            "verbose": False, "display_progress": False, "toc": False, "device": "cuda:0",
            "batch_creator": farmer.batch_creator, "iterk_solver_options": dict(farmer.PDHG_ITERK_OPTIONS)}
    ph = PH(opts, farmer.scenario_names_creator(S), farmer.scenario_creator,
            scenario_creator_kwargs={"crops_multiplier": 1, "num_scens": S})
    ph.PH_Prep()
    ph.Iter0()
    ph.iterk_loop()
    e = ph.engine
    info = e.ipm_info()
    ph.options["PHIterLimit"] = iters
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ph.iterk_loop()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    p = e.ipm_prof() if prof else None
    e.close()
    return dt, p, info


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("S", type=int)
    ap.add_argument("L", type=int)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--defs", default="")
    ap.add_argument("--prof", type=int, default=1)
    ap.add_argument("--level", type=int, default=1)
    a = ap.parse_args()
    dt, p, info = run(a.S, a.L, a.iters, a.defs, a.prof, a.level)
    out = {"S": a.S, "L": a.L, "ms_per_step": 1e3 * dt, "lanes": info["lanes"], "kernel": info["kernel"],
           "scratch": info["scratch_bytes"], "defs": a.defs, "prof": bool(a.prof)}
    if p is not None:
        import numpy as np
        nw = int(np.ceil(a.S * max(1, int(info["lanes"])) / 64.0))
        r = p[:nw].astype(np.float64)
        ok = r[:, 5] > 0
        r = r[ok]
        t0 = r[:, 0].min()
        us = lambda v: round(float(v) / 100.0, 2)  # noqa: E731  (100 MHz ticks)
        seg = {"entry_delay": r[:, 0] - t0, "pre_loop": r[:, 1] - r[:, 0], "loop": r[:, 2] - r[:, 1],
               "stores": r[:, 3] - r[:, 2], "stats": r[:, 4] - r[:, 3], "epilogue": r[:, 5] - r[:, 4],
               "life": r[:, 5] - r[:, 0]}
        out["waves"] = int(ok.sum())
        out["span_us"] = us(r[:, 5].max() - t0)
        out["seg_mean_us"] = {k: us(v.mean()) for k, v in seg.items()}
        out["seg_max_us"] = {k: us(v.max()) for k, v in seg.items()}
        crit = int(np.argmax(r[:, 5]))
        out["critical_wave"] = {"wave": crit, "trips": int(r[crit, 6]), **{k: us(v[crit]) for k, v in seg.items()}}
        out["trips"] = {"mean": float(r[:, 6].mean()), "max": int(r[:, 6].max())}
        loop_per_trip = seg["loop"] / np.maximum(r[:, 6], 1)
        out["loop_us_per_trip"] = {"mean": us(loop_per_trip.mean()), "max": us(loop_per_trip.max())}
        if a.level >= 2 and a.L > 1:
            tr = r[:, 6].sum()
            per = r[:, 8:16].sum(0) / max(1.0, tr)
            out["cycles_per_trip"] = {k: round(float(v), 1) for k, v in zip(PHASES, per)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
