"""mpisppy_amd -- MI355X-native progressive-hedging hot path.

A drop-in engine for mpi-sppy's PH scenario-decomposition loop
(SPOpt.solve_loop + PHBase.Compute_Xbar / Update_W / convergence_diff): all local
scenarios are solved as one batched PDHG solve by hand-written HIP kernels
(csrc/phgpu.hip, C-ABI in include/phgpu.h), and the per-tree-node x̄ reduction is
one RCCL all-reduce per PH iteration.  See DESIGN.md.
"""
import time as _time

__version__ = "0.1.0"

_toc_start = _time.perf_counter()
_toc_last = _toc_start


def global_toc(msg, cond=True):
    """mpisppy/__init__.py:4-12 style tic-toc trace ("[elapsed] msg")."""
    global _toc_last
    now = _time.perf_counter()
    if cond:
        print(f"[{now - _toc_start:8.2f}] {msg}", flush=True)
    _toc_last = now
    return now - _toc_start
