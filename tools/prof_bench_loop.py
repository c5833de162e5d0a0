"""Host profile (cProfile) of bench.py's timed loop: config 3, instrumented as bench.py
instruments it, with and without the speculative solve.  Prints ms per step and the
functions with the most cumulative time."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy-1_amd"))
import torch  # noqa: E402
from mpisppy_amd.opt.ph import PH  # noqa: E402
from mpisppy_amd.examples import farmer  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
for spec in (True, False):
    opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": 5, "defaultPHrho": 1.0, "convthresh": -1.0,
            "verbose": False, "display_progress": False, "toc": False, "device": "cuda:0",
            "batch_creator": farmer.batch_creator, "speculative_solve": spec,
            "iterk_solver_options": {"eps_rel": 1e-9, **farmer.PDHG_ITERK_OPTIONS}}
    ph = PH(opts, farmer.scenario_names_creator(S), farmer.scenario_creator,
            scenario_creator_kwargs={"crops_multiplier": 1, "num_scens": S})
    ph.PH_Prep()
    ph.Iter0()
    ph.iterk_loop()
    for instrument in (False, True):
        if instrument:
            ph.engine.instrument(20)
        ph.options["PHIterLimit"] = 20
        torch.cuda.synchronize()
        pr = cProfile.Profile()
        t0 = time.perf_counter()
        pr.enable()
        ph.iterk_loop()
        torch.cuda.synchronize()
        pr.disable()
        dt = time.perf_counter() - t0
        print(f"=== speculative={spec} instrumented={instrument}: {1e3 * dt / 20:.3f} ms per step", flush=True)
        pstats.Stats(pr).sort_stats("cumulative").print_stats(18)
        ph.engine._ins = None
