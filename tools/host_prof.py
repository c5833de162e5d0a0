"""Host-side profile of PHBase.iterk_loop (TOOL ONLY): cProfile over K PH iterations of
farmer on S scenarios after a warm-up, the functions with the most own time.

    python tools/host_prof.py S [K]
"""
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

S = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
K = int(sys.argv[2]) if len(sys.argv) > 2 else 200
opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": 5, "defaultPHrho": 1.0, "convthresh": -1.0,
        "verbose": False, "display_progress": False, "toc": False, "device": "cuda:0",
        "batch_creator": farmer.batch_creator, "iterk_solver_options": dict(farmer.PDHG_ITERK_OPTIONS)}
ph = PH(opts, farmer.scenario_names_creator(S), farmer.scenario_creator,
        scenario_creator_kwargs={"crops_multiplier": 1, "num_scens": S})
ph.PH_Prep()
ph.Iter0()
ph.iterk_loop()
ph.options["PHIterLimit"] = K
torch.cuda.synchronize()
t0 = time.perf_counter()
ph.iterk_loop()
torch.cuda.synchronize()
plain = (time.perf_counter() - t0) / K
pr = cProfile.Profile()
torch.cuda.synchronize()
t0 = time.perf_counter()
pr.enable()
ph.iterk_loop()
pr.disable()
torch.cuda.synchronize()
prof = (time.perf_counter() - t0) / K
print(f"S={S} K={K}: {1e3 * plain:.4f} ms per PH iteration ({1e3 * prof:.4f} under cProfile)")
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
ph.engine.close()
