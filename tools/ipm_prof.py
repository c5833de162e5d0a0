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


def run(S, L, iters, defs, prof):
    os.environ["PHGPU_IPM_LANES"] = str(L)
    d = (defs + ";" if defs else "") + ("IPM_PROF=1" if prof else "")
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
    e.ipm_prof(reset=True)
    ph.options["PHIterLimit"] = iters
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ph.iterk_loop()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    p = e.ipm_prof(reset=True)
    e.close()
    return dt, p, info


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("S", type=int)
    ap.add_argument("L", type=int)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--defs", default="")
    ap.add_argument("--prof", type=int, default=1)
    a = ap.parse_args()
    dt, p, info = run(a.S, a.L, a.iters, a.defs, a.prof)
    L = a.L
    out = {"S": a.S, "L": a.L, "ms_per_step": 1e3 * dt, "lanes": info["lanes"], "kernel": info["kernel"],
           "scratch": info["scratch_bytes"], "defs": a.defs, "prof": bool(a.prof)}
    if a.prof and p[14]:
        w = max(1, p[14])
        us = lambda k: round(p[k] / w / 100.0, 2)  # noqa: E731  (100 MHz real-time ticks)
        out["wave_us_mean"] = {"entry_to_loop": us(11), "loop": us(9), "loop_end_to_stores": us(16),
                               "stats": us(17), "to_exit": us(18), "life": us(13)}
        out["waves"] = p[14]
        out["wave_us_max"] = {"life": p[20] / 100.0, "entry_to_loop_end": p[21] / 100.0}
    if a.prof and p[15] and L > 1:
        trips = p[15]
        per = [v / trips for v in p[:8]]
        out["trips_per_wave"] = trips / max(1, p[14])
        out["cycles_per_trip"] = {k: round(v, 1) for k, v in zip(PHASES, per)}
        out["cycles_per_trip_total"] = round(sum(per), 1)
        out["clock_GHz_est"] = (p[8] / max(1, p[9])) * 0.1
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
