import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-sppy-1_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
from test_gpu_parity import _random_lp_batch
from mpisppy_amd.engine import PHEngine
from mpisppy_amd import _lib
for S, wq, seed in [(5, False, 1), (97, True, 2), (300, False, 3)]:
    b = _random_lp_batch(S, 11, 7, 0.35, seed=seed, with_q=wq)
    print("S", S, "rowlens", np.diff(b.row_ptr).tolist(), "collens", np.bincount(b.col_idx, minlength=b.n).tolist())
    e = PHEngine(b, device="cuda:0")
    print(" info", e.kernel_info())
    e.solve(_lib.default_options(kernel=1), warm=False)
    o1 = e.host("obj").copy(); it1 = e.host("iters").copy(); x1 = e.host("x").copy()
    e.solve(_lib.default_options(kernel=2, max_iter=20000), warm=False)
    o2 = e.host("obj"); st2 = e.host("status"); it2 = e.host("iters"); x2 = e.host("x")
    bad = np.nonzero(st2 != 0)[0]
    print(" bad", bad[:10].tolist(), "it1", it1[bad[:5]].tolist(), "it2", it2[bad[:5]].tolist())
    print(" obj diff max", np.abs(o1 - o2).max(), "x diff", np.abs(x1 - x2).max())
    for k in bad[:2]:
        print("  ", k, o1[k], o2[k], x1[k], x2[k])
    e.close()
