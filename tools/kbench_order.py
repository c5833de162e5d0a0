"""Queue-order study for the register path (record mode): the same cold solve twice, so
the second launch is ordered by the exact iteration counts of the first (a perfect
longest-first predictor), next to warm PH solves ordered by the previous PH iteration's
counts, and the rank correlation of consecutive PH iterations' counts."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-sppy-1_amd"))
import numpy as np, torch
from mpisppy_amd.examples import farmer
from mpisppy_amd.engine import PHEngine
from mpisppy_amd import _lib

S = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
names = farmer.scenario_names_creator(S)
b = farmer.batch_creator(names, crops_multiplier=1, num_scens=S)
e = PHEngine(b, device="cuda:0")
o = _lib.default_options()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]


def timed(warm):
    ev[0].record(); e.solve(o, warm=warm); ev[1].record(); torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]), e.host("iters").copy()


def spearman(a, b):
    ra = np.argsort(np.argsort(a)); rb = np.argsort(np.argsort(b))
    return float(np.corrcoef(ra, rb)[0, 1])


t0, i0 = timed(False)
t1, i1 = timed(False)
print(f"Iter0 LP cold: first {t0:.3f} ms, repeat (exact order) {t1:.3f} ms; max it {i1.max()} mean {i1.mean():.0f}", flush=True)
e.set_rho(1.0); e.set_terms(1, 1)
prev = None
for k in range(6):
    e.compute_xbar(); e.update(True)
    t, it = timed(True)
    c = spearman(prev, it) if prev is not None else float('nan')
    print(f"PH {k}: warm {t:.3f} ms, max it {it.max()} mean {it.mean():.0f}, rank corr with previous {c:.3f}", flush=True)
    prev = it
# cold QP twice: the second is ordered by the first's exact counts
tq0, q0 = timed(False)
tq1, q1 = timed(False)
print(f"QP cold: first {tq0:.3f} ms, repeat (exact order) {tq1:.3f} ms; max it {q1.max()} mean {q1.mean():.0f}; "
      f"counts equal {np.array_equal(q0, q1)}", flush=True)
e.close()
