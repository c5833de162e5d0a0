"""Path 6 without a GPU: the library's generator (phgpu_ipm_source) for the farmer and
aircond patterns.

  * the generated module compiles for gfx950 (hipcc, device only) and the farmer IPM
    kernel -- the headline's -- needs no scratch (its state fits VGPRs + AGPRs);
  * the same kernel text, compiled for the host (ipm_host.py), solves farmer's Iter0 LPs
    and PH prox QPs to the exact vectorised oracle (oracle/farmer_vec.py, pinned in
    test_oracle_scale.py) and aircond's LPs to HiGHS -- the arithmetic the GPU runs,
    checked on the CPU;
  * the symbolic factorisation is consistent (factor entries, flop counts).
Tolerances: objectives 1e-9 relative (the solves' own eps), x 1e-5 absolute (north_star).
"""
import os
import re
import subprocess

import numpy as np
import pytest

import ipm_host

HIPCC = "/opt/rocm/bin/hipcc"


def _farmer(S):
    from mpisppy_amd.examples import farmer
    return farmer.batch_creator(farmer.scenario_names_creator(S), crops_multiplier=1, num_scens=S)


def _aircond(bf=(4, 4, 4)):
    from mpisppy_amd.examples import aircond
    kw = {"Capacity": 200, "QuadShortCoeff": 0.3, "BeginInventory": 50, "mu_dev": 0, "sigma_dev": 40,
          "start_seed": 0}
    S = int(np.prod(bf))
    return aircond.batch_creator(aircond.scenario_names_creator(S), branching_factors=list(bf), **kw)


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_generated_module_compiles_for_gfx950_without_scratch(tmp_path):
    import mpisppy_amd._lib as L
    src, (rows, nf, fac, sol) = L.ipm_source(_farmer(64))
    assert rows == 7 and 7 <= nf <= 28 and fac > 0 and sol == 4 * (nf - rows) + rows
    p = tmp_path / "ipm_farmer.hip"
    p.write_text("#include <hip/hip_runtime.h>\n" + src)
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", "--cuda-device-only",
                        "-Rpass-analysis=kernel-resource-usage", "-o", str(tmp_path / "x.o"), str(p)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    # resource remarks of k_solve_ipm (the second kernel of the module)
    blocks = r.stderr.split("Function Name: ")
    ipm = [b for b in blocks if b.startswith("k_solve_ipm")]
    assert ipm, r.stderr[-2000:]
    scratch = int(re.search(r"ScratchSize \[bytes/lane\]: (\d+)", ipm[0]).group(1))
    assert scratch == 0, ipm[0][:1500]


def test_host_kernel_farmer_iter0_and_prox_vs_oracle():
    from mpisppy_amd.examples import farmer
    from oracle import farmer_vec as FV
    S = 1024
    names = farmer.scenario_names_creator(S)
    b = _farmer(S)
    ph = FV.FarmerVecPH(names, 1)
    ph.iter0()
    x, y, obj, bound, st, it = ipm_host.solve(b, eps_rel=1e-10)
    ok = st == 0
    assert ok.mean() >= 0.99, np.nonzero(~ok)[0]  # the rest go to the PDHG fallback on the GPU
    assert it[ok].max() <= 40
    rel = np.abs(obj[ok] - ph.iter0_obj[ok]) / np.abs(ph.iter0_obj[ok])
    assert rel.max() <= 1e-9, rel.max()
    assert np.all(bound[ok] <= obj[ok] + 1e-9 * np.abs(obj[ok]))
    assert np.abs(x[ok][:, b.nonant_col] - ph.iter0_x[ok]).max() <= 1e-5
    ph.iterk_loop(3)
    W, xb, rho = ph.W.copy(), ph.xbar.copy(), ph.rho.copy()
    xo, oo = FV.prox(ph.bp, ph.sl, ph.f0, W, xb, rho, ph.total)
    x2, y2, obj2, bd2, st2, it2 = ipm_host.solve(b, W=W, rho=rho, xbar=xb, eps_rel=1e-9)
    ok2 = st2 == 0
    assert ok2.all(), np.nonzero(~ok2)[0]
    assert np.abs(x2[:, b.nonant_col] - xo).max() <= 1e-5
    assert (np.abs(obj2 - oo) / np.abs(oo)).max() <= 1e-9


def test_host_kernel_aircond_lp_vs_highs():
    from oracle.lpqp import solve_lp_highs
    b = _aircond()
    x, y, obj, bound, st, it = ipm_host.solve(b, eps_rel=1e-9)
    assert (st == 0).all()
    q0 = b.q.copy()
    for s in range(0, b.S, 8):
        A = b.dense_A(s)
        if np.any(q0[s] != 0):
            continue  # aircond has a quadratic shortage term; checked by the GPU tests
        xr, ob, rc = solve_lp_highs(A, b.rl[s], b.ru[s], b.lb[s], b.ub[s], b.c[s])
        assert rc == 0 and abs(obj[s] - ob) <= 1e-7 * max(1.0, abs(ob))
    # feasibility of every answer
    for s in range(b.S):
        ax = b.dense_A(s) @ x[s]
        assert np.all(np.abs(ax - b.rl[s]) <= 1e-6 * (1 + np.abs(b.rl[s])))
        assert np.all(x[s] >= b.lb[s] - 1e-9) and np.all(x[s] <= b.ub[s] + 1e-9)


def test_host_kernel_warm_start_vs_oracle():
    """The warm start (a PH iteration's solve from the previous x / y, jit_ipm.hip.in
    IPM_WARM) reaches the same exact prox-QP solutions as the cold start, in fewer
    iterations."""
    from mpisppy_amd.examples import farmer
    from oracle import farmer_vec as FV
    S = 1024
    names = farmer.scenario_names_creator(S)
    b = _farmer(S)
    ph = FV.FarmerVecPH(names, 1)
    ph.iter0()
    ph.iterk_loop(2)
    W, xb, rho = ph.W.copy(), ph.xbar.copy(), ph.rho.copy()
    xp, yp, *_ = ipm_host.solve(b, W=W, rho=rho, xbar=xb, eps_rel=1e-9)    # the previous solve
    ph.iterk_loop(1)
    W, xb, rho = ph.W.copy(), ph.xbar.copy(), ph.rho.copy()
    xo, oo = FV.prox(ph.bp, ph.sl, ph.f0, W, xb, rho, ph.total)
    _, _, _, _, stc, itc = ipm_host.solve(b, W=W, rho=rho, xbar=xb, eps_rel=1e-9)
    x, y, obj, bd, st, it = ipm_host.solve(b, W=W, rho=rho, xbar=xb, eps_rel=1e-9, x_in=xp, y_in=yp)
    assert (st == 0).all() and (stc == 0).all()
    assert np.abs(x[:, b.nonant_col] - xo).max() <= 1e-5
    assert (np.abs(obj - oo) / np.abs(oo)).max() <= 1e-9
    assert np.all(bd <= obj + 1e-9 * np.abs(obj))
    assert it.mean() < 0.8 * itc.mean() and it.max() < itc.max(), (it.mean(), itc.mean(), it.max(), itc.max())
