"""One cold solve of S UC scenarios on path 4 (profiling driver for rocprofv3)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy-1_amd"))
import torch  # noqa: E402
from mpisppy_amd import _lib  # noqa: E402
from mpisppy_amd.engine import PHEngine  # noqa: E402
from mpisppy_amd.examples import uc  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 256
max_iter = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
b = uc.batch_creator(uc.scenario_names_creator(S), num_scens=int(sys.argv[3]) if len(sys.argv) > 3 else 1000)
e = PHEngine(b, device="cuda:0")
torch.cuda.synchronize()
t = time.time()
e.solve(_lib.default_options(eps_rel=1e-6, max_iter=max_iter), warm=False)
torch.cuda.synchronize()
dt = time.time() - t
its = e.host("iters")
print(f"S={S} solve {dt:.3f}s scenario-iterations {int(its.sum())} max {its.max()} "
      f"-> {dt / its.max() * 1e3:.3f} ms per iteration, {8 * (5 * b.n + 4 * b.m) * its.sum() / dt / 1e9:.0f} GB/s alg",
      flush=True)
e.close()  # (before the interpreter's teardown: a profiler's exit otherwise finds the handle alive)
