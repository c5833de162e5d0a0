"""The workgroup interior point (jit_ipm_wave.hip.in) run on the CPU by tests/ipm_wave_host.py
(one std::thread per GPU thread, barriers for the workgroup syncs and sums): its generated
tables and arithmetic against HiGHS / the oracle's QP IPM / the exact farmer oracle, without
a GPU.  test_gpu_ipm_wave.py checks the real kernel."""
import numpy as np
import pytest

import ipm_wave_host
from test_gpu_ipm_wave import arrow_batch

OBJ_REL = 1e-5


@pytest.mark.parametrize("blocks,S,with_q,lanes", [(15, 3, False, 64), (30, 2, True, 64), (100, 1, False, 128)])
def test_host_wave_arrow_vs_oracle(blocks, S, with_q, lanes):
    from oracle.lpqp import solve_lp_highs, solve_qp_ipm
    b = arrow_batch(S, blocks, seed=blocks + S, with_q=with_q)
    x, y, obj, bound, st, it = ipm_wave_host.solve(b, lanes=lanes)
    assert (st == 0).all(), (st, it)
    for s in range(S):
        A = b.dense_A(s)
        if with_q:
            xr, ob, rc = solve_qp_ipm(A, b.rl[s], b.ru[s], b.lb[s], b.ub[s], b.c[s], b.q[s])
        else:
            xr, ob, rc = solve_lp_highs(A, b.rl[s], b.ru[s], b.lb[s], b.ub[s], b.c[s])
        assert rc == 0
        tol = OBJ_REL * max(1.0, abs(ob))
        assert abs(obj[s] - ob) <= tol and abs(bound[s] - ob) <= tol, (s, obj[s], bound[s], ob, it[s])


def test_host_wave_farmer_cm10_vs_oracle():
    from mpisppy_amd.examples import farmer
    from oracle import farmer_vec as fv
    names = ["scen0", "scen5", "scen17", "scen600"]
    b = farmer.batch_creator(names, crops_multiplier=10, num_scens=1024)
    x, y, obj, bound, st, it = ipm_wave_host.solve(b, lanes=64, eps_rel=1e-10)
    assert (st == 0).all(), (st, it)
    bp, sl, f0 = fv.pieces(fv.yields(names, 10), 10)
    x_ref, obj_ref = fv.iter0_lp(bp, sl, f0, 5000.0)
    assert np.abs(obj - obj_ref).max() <= OBJ_REL * np.abs(obj_ref).max(), (obj, obj_ref)
    err = np.abs(x[:, b.nonant_col] - x_ref).max()
    assert err <= 1e-5 * 5000, err


def test_host_wave_farmer_cm64_vs_oracle():
    """cm = 64 (n 768, m 385): four waves per scenario, 191 two-row subtrees over 256 threads."""
    from mpisppy_amd.examples import farmer
    from oracle import farmer_vec as fv
    names = ["scen7"]
    b = farmer.batch_creator(names, crops_multiplier=64, num_scens=2048)
    x, y, obj, bound, st, it = ipm_wave_host.solve(b, lanes=256, eps_rel=1e-10)
    assert (st == 0).all(), (st, it)
    bp, sl, f0 = fv.pieces(fv.yields(names, 64), 64)
    x_ref, obj_ref = fv.iter0_lp(bp, sl, f0, 500.0 * 64)
    assert abs(obj[0] - obj_ref[0]) <= OBJ_REL * abs(obj_ref[0]), (obj, obj_ref)
    assert np.abs(x[:, b.nonant_col] - x_ref).max() <= 1e-5 * 500 * 64
