"""The PH step's readbacks without copy launches (engine.update -> phgpu_ph_update_ex).

* x̄ partials: when no wave of local scenarios spans two nodes, k_xbar_partial clears
  node_buf itself (no memset); when one does (small multistage trees), the memset stays.
  Either way node_buf must equal the tree sums phbase.py:54-79 defines, computed here in
  numpy from the engine's own x, node ids and probability coefficients, and a node_buf
  full of garbage before the call must not leak into it.
* conv and the last solve's statistics are written by the update kernel into pinned host
  memory: conv must equal the device-buffer path (phgpu_ph_update) bit for bit and the
  statistics must equal phgpu_solve_stats.
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _expected_node_buf(e):
    b = e.batch_ref
    x = e.x.cpu().numpy()
    node_of = e.node_of.cpu().numpy().reshape(-1, e.S)
    pc = e.prob_coeff.cpu().numpy().reshape(-1, e.S)
    half = e.num_nodes * e.nlen_max
    out = np.zeros(2 * half)
    for k in range(e.nn):
        d, j, o = int(b.nonant_depth[k]), int(b.nonant_col[k]), int(b.nonant_off[k])
        v = x[j]
        np.add.at(out, node_of[d] * e.nlen_max + o, pc[d] * v)
        np.add.at(out, half + node_of[d] * e.nlen_max + o, pc[d] * v * v)
    return out


def _engine(model, S, bf=None):
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd.examples import aircond, farmer
    if model in ("farmer", "farmer10"):  # farmer10: crops_multiplier 10, 30 nonants (config 2)
        cm = 10 if model == "farmer10" else 1
        b = farmer.batch_creator(farmer.scenario_names_creator(S), crops_multiplier=cm, num_scens=S)
    else:
        kw = {"branching_factors": bf, "Capacity": 200, "QuadShortCoeff": 0.3, "BeginInventory": 50,
              "mu_dev": 0, "sigma_dev": 40, "start_seed": 0}
        b = aircond.batch_creator(aircond.scenario_names_creator(S), **kw)
    e = PHEngine(b, device="cuda:0")
    e.batch_ref = b
    return e


@pytest.mark.parametrize("model,S,bf", [("farmer", 1000, None),       # two-stage, ragged last wave
                                        ("aircond", 128, [2, 64]),    # nodes aligned to waves
                                        ("aircond", 24, [4, 3, 2])])  # waves span several nodes
def test_node_buf_cleared_and_summed(gpu, model, S, bf):
    from mpisppy_amd import _lib
    e = _engine(model, S, bf)
    e.solve(_lib.default_options(eps_rel=1e-9), warm=False)
    for _ in range(2):
        e.node_buf.fill_(1e30)                         # stale data must not survive
        e.compute_xbar()
        got = e.node_buf.cpu().numpy()
        ref = _expected_node_buf(e)
        np.testing.assert_allclose(got, ref, rtol=1e-13, atol=1e-12)
        e.update(True)
        e.solve(_lib.default_options(), warm=True)
    e.close()


@pytest.mark.parametrize("kernel", [0, 2])
def test_update_ex_host_conv_and_stats(gpu, kernel):
    from mpisppy_amd import _lib
    e = _engine("farmer", 3000)
    e.set_rho(1.0)
    e.set_terms(1, 1)
    e.solve(_lib.default_options(eps_rel=1e-9, kernel=kernel), warm=False)
    e.compute_xbar()
    W0 = e.W.clone()
    # device path: phgpu_ph_update into the device conv buffer
    _lib.check(e.lib.phgpu_ph_update(e.h, e.x.data_ptr(), e.node_buf.data_ptr(), e.xbar.data_ptr(),
                                     e.W.data_ptr(), e.rho.data_ptr(), 1, e.conv_buf.data_ptr(), e._stream()),
               "phgpu_ph_update")
    conv_dev = float(e.conv_buf.item())
    # the last-block reduction (a hardware ordering of relaxed atomics, phgpu.hip
    # conv_last_block) against an independent sum: a block partial read before its swap landed
    # would be off by a whole block's share (phbase.py:321-343: mean |x - x̄| over nonants)
    nc = torch.as_tensor(e.batch.nonant_col, dtype=torch.long, device=e.device)
    ref = (e.x.index_select(0, nc) - e.xbar[:e.nn]).abs().sum().item() / (e.S * e.nn)
    assert abs(conv_dev - ref) <= 1e-12 * abs(ref), (conv_dev, ref)
    ref_stats = torch.zeros(6, dtype=torch.int64).pin_memory()
    _lib.check(e.lib.phgpu_solve_stats(e.h, ref_stats.data_ptr(), e._stream()), "phgpu_solve_stats")
    torch.cuda.synchronize()
    # host-mapped path (what the PH loop uses with one rank)
    e.W.copy_(W0)
    conv_h = torch.full((1,), -1.0, dtype=torch.float64).pin_memory()
    st_h = torch.full((6,), -1, dtype=torch.int64).pin_memory()
    _lib.check(e.lib.phgpu_ph_update_ex(e.h, e.x.data_ptr(), e.node_buf.data_ptr(), e.xbar.data_ptr(),
                                        e.W.data_ptr(), e.rho.data_ptr(), 1, conv_h.data_ptr(),
                                        st_h.data_ptr(), e._stream()), "phgpu_ph_update_ex")
    torch.cuda.synchronize()
    assert float(conv_h[0]) == conv_dev
    assert st_h.tolist() == ref_stats.tolist()
    assert int(st_h[:4].sum()) == e.S and int(st_h[0]) == e.S     # all OPTIMAL, counts add up
    # the engine's own loop pieces: update -> convergence_diff / the gripe count
    e.W.copy_(W0)
    e.update(True)
    assert e.convergence_diff() == conv_dev
    e.count_not_optimal_async()
    e.solve(_lib.default_options(kernel=kernel), warm=True)
    e.count_not_optimal_async()
    e.compute_xbar()
    e.update(True)
    e.convergence_diff_async()
    e.convergence_wait()
    assert e.pending_not_optimal() == e.count_not_optimal() == 0
    e.close()


def test_update_ex_rejects_stats_before_solve(gpu):
    from mpisppy_amd import _lib
    e = _engine("farmer", 100)
    st_h = torch.zeros(6, dtype=torch.int64).pin_memory()
    rc = e.lib.phgpu_ph_update_ex(e.h, e.x.data_ptr(), e.node_buf.data_ptr(), e.xbar.data_ptr(),
                                  e.W.data_ptr(), e.rho.data_ptr(), 1, e.conv_buf.data_ptr(),
                                  ctypes.c_void_p(st_h.data_ptr()), e._stream())
    assert rc != 0
    e.close()



@pytest.mark.parametrize("model,S,bf", [("farmer", 1000, None), ("farmer", 20000, None),
                                        ("farmer10", 1024, None),   # 30 nonants: the 256-thread kernel
                                        ("aircond", 128, [2, 64])])
def test_step_local_matches_reduce_then_update(gpu, model, S, bf):
    """phgpu_ph_step_local (one rank: x̄ folded into the update launch for two-stage
    problems; the general route otherwise) gives the node sums, x̄, W, conv and statistics
    of phgpu_ph_reduce + phgpu_ph_update_ex, to the last bits of the summation order."""
    from mpisppy_amd import _lib
    e = _engine(model, S, bf)
    e.set_rho(1.0)
    e.set_terms(1, 1)
    e.solve(_lib.default_options(eps_rel=1e-9), warm=False)
    W0 = e.W.clone()
    conv_a = torch.zeros(1, dtype=torch.float64).pin_memory()
    st_a = torch.zeros(6, dtype=torch.int64).pin_memory()
    _lib.check(e.lib.phgpu_ph_reduce(e.h, e.x.data_ptr(), e.node_buf.data_ptr(), e._stream()), "phgpu_ph_reduce")
    _lib.check(e.lib.phgpu_ph_update_ex(e.h, e.x.data_ptr(), e.node_buf.data_ptr(), e.xbar.data_ptr(),
                                        e.W.data_ptr(), e.rho.data_ptr(), 1, conv_a.data_ptr(), st_a.data_ptr(),
                                        e._stream()), "phgpu_ph_update_ex")
    torch.cuda.synchronize()
    ref = {k: getattr(e, k).cpu().numpy().copy() for k in ("node_buf", "xbar", "W")}
    for _ in range(2):                              # the first call may take the general route
        e.W.copy_(W0)
        e.node_buf.fill_(1e30)
        conv_b = torch.zeros(1, dtype=torch.float64).pin_memory()
        st_b = torch.zeros(6, dtype=torch.int64).pin_memory()
        _lib.check(e.lib.phgpu_ph_step_local(e.h, e.x.data_ptr(), e.node_buf.data_ptr(), e.xbar.data_ptr(),
                                             e.W.data_ptr(), e.rho.data_ptr(), 1, conv_b.data_ptr(),
                                             st_b.data_ptr(), e._stream()), "phgpu_ph_step_local")
        torch.cuda.synchronize()
        for k, v in ref.items():
            np.testing.assert_allclose(getattr(e, k).cpu().numpy(), v, rtol=1e-13, atol=1e-13, err_msg=k)
        assert abs(float(conv_b[0]) - float(conv_a[0])) <= 1e-13 * abs(float(conv_a[0]))
        assert st_b.tolist() == st_a.tolist()
    # the PH loop's lazy path (engine.compute_xbar(lazy=True) + update) and a node_buf read
    e.W.copy_(W0)
    e.compute_xbar(lazy=True)
    nb = e.host("node_buf")                          # flushes the pending x̄
    np.testing.assert_allclose(nb, ref["node_buf"], rtol=1e-13, atol=1e-13)
    e.compute_xbar(lazy=True)
    e.update(True)
    assert abs(e.convergence_diff() - float(conv_a[0])) <= 1e-13 * abs(float(conv_a[0]))
    np.testing.assert_allclose(e.W.cpu().numpy(), ref["W"], rtol=1e-13, atol=1e-13)
    e.close()


@pytest.mark.parametrize("lanes", ["1", "8"])
@pytest.mark.parametrize("maxit", ["2", "12"])
def test_epilogue_partials_with_fallback_chunks(gpu, lanes, maxit):
    """Path 6 writes the x̄ partials in its epilogue (one chunk per wave, or per block of
    lane groups); a chunk with a scenario the PDHG fallback solved is recomputed from x by
    the consumer.  PHGPU_IPM_MAXIT sends every scenario (2) or some (12) to the fallback;
    node_buf (phgpu_ph_reduce), the folded one-rank step (phgpu_ph_step_local) and conv must
    equal the sums of phbase.py:54-79 / 330-339 over the engine's own x."""
    import os
    from mpisppy_amd import _lib
    keep = {k: os.environ.get(k) for k in ("PHGPU_IPM_MAXIT", "PHGPU_IPM_LANES")}
    os.environ["PHGPU_IPM_LANES"] = lanes
    try:
        e = _engine("farmer", 1000)
        e.solve(_lib.default_options(eps_rel=1e-9), warm=False)
        e.compute_xbar()                        # finds out the wave / node layout (once)
        e.set_rho(1.0)
        e.set_terms(1, 1)
        e.update(True)
        e.convergence_diff()
        os.environ["PHGPU_IPM_MAXIT"] = maxit
        e.solve(_lib.default_options(), warm=True)
        assert e.kernel_info()["path"] == 6 and int(e.ipm_info()["lanes"]) == int(lanes)
        it = e.host("iters")
        assert (e.host("status") == 0).all()
        fell = int((it > int(maxit)).sum())
        assert fell > 0 and (maxit != "2" or fell == e.S), fell
        e.node_buf.fill_(1e30)
        e.compute_xbar()
        ref = _expected_node_buf(e)
        np.testing.assert_allclose(e.node_buf.cpu().numpy(), ref, rtol=1e-13, atol=1e-12)
        # the folded step of one rank, from the same partials
        x = e.x.cpu().numpy()[e.batch_ref.nonant_col]
        half = e.num_nodes * e.nlen_max
        xb = ref[:half][:e.nn]
        conv_ref = np.abs(x - xb[:, None]).sum() / (e.S * e.nn)
        e.node_buf.fill_(1e30)
        e.compute_xbar(lazy=True)
        e.update(True)
        conv = e.convergence_diff()
        assert abs(conv - conv_ref) <= 1e-12 * max(1.0, conv_ref), (conv, conv_ref)
        np.testing.assert_allclose(e.host("node_buf"), ref, rtol=1e-13, atol=1e-12)
        e.close()
    finally:
        for k, v in keep.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
