"""GPU micro-benchmark of the solve kernels on farmer (Iter0 LP + 3 PH QP solves)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-sppy-1_amd"))
import numpy as np, torch
from mpisppy_amd.examples import farmer
from mpisppy_amd.engine import PHEngine
from mpisppy_amd import _lib
S = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
cm = int(sys.argv[2]) if len(sys.argv) > 2 else 1
lanes = [int(v) for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0]
extra = dict(kv.split('=') for kv in sys.argv[4].split(',')) if len(sys.argv) > 4 else {}
extra = {k: (float(v) if '.' in v or 'e' in v else int(v)) for k, v in extra.items()}
names = farmer.scenario_names_creator(S)
b = farmer.batch_creator(names, crops_multiplier=cm, num_scens=S)
ref = None
for L in lanes:
    for kern in ([1, 0] if (L == lanes[0] and not extra and os.environ.get('KB_GLOBAL')) else [0]):
        if L:
            os.environ["PHGPU_LANES"] = str(L)
        else:
            os.environ.pop("PHGPU_LANES", None)
        e = PHEngine(b, device="cuda:0")
        info = e.kernel_info()
        o = _lib.default_options(kernel=kern, **extra)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(); e.solve(o, warm=False); ev[1].record(); torch.cuda.synchronize()
        t0 = ev[0].elapsed_time(ev[1]); it0 = e.host("iters")
        # PH iterations
        e.set_rho(1.0); e.set_terms(1, 1)
        times = []
        for k in range(3):
            e.compute_xbar(); e.update(True)
            ev[0].record(); e.solve(o, warm=True); ev[1].record(); torch.cuda.synchronize()
            times.append(ev[0].elapsed_time(ev[1]))
        it = e.host("iters"); st = e.host("status")
        W = e.host("W")
        if ref is None: ref = W.copy()
        print(f"kernel={kern} path={info['path']} L={info['lanes']} inst=({info['KC']},{info['ZC']},{info['KR']},{info['ZR']}) wg=({info['wKC']},{info['wZC']},{info['wKR']},{info['wZR']},{info['wps']}) "
              f"iter0 {t0:.2f} ms (max it {it0.max()}) | PH solves ms {['%.2f' % t for t in times]} "
              f"max it {it.max()} mean {it.mean():.0f} | us/iter(max) {1e3 * times[-1] / max(1, it.max()):.2f} "
              f"| nonopt {(st != 0).sum()} | W dev vs first {np.abs(W - ref).max():.2e}", flush=True)
        e.close()
