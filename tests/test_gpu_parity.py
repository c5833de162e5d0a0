"""GPU parity tests: the HIP path (through the C-ABI) against the CPU oracle and the
reference's own fixtures.  Tolerances are those of BASELINE.json north_star:
objectives 1e-5 relative, x̄ / W 1e-5 absolute, PH iteration count +-1."""
import ctypes
import csv
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "golden.json")))

OBJ_REL = 1e-5
ABS = 1e-5


def _ph(names, creator, kwargs, rho=1.0, iters=5, thresh=1e-10, **extra):
    from mpisppy_amd.opt.ph import PH
    opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": iters, "defaultPHrho": rho,
            "convthresh": thresh, "verbose": False, "display_progress": False, "toc": False,
            "device": "cuda:0"}
    opts.update(extra)
    all_nodenames = opts.pop("all_nodenames", None)
    return PH(opts, names, creator, scenario_creator_kwargs=kwargs, all_nodenames=all_nodenames)


def test_farmer3_w_xbar_vs_reference_fixtures(gpu):
    """test_w_writer.py:85-117: farmer 3 scen, rho 1, 5 iterations."""
    from mpisppy_amd.examples import farmer
    names = farmer.scenario_names_creator(3)
    ph = _ph(names, farmer.scenario_creator, {"num_scens": 3})
    conv, eobj, tb = ph.ph_main()
    W = ph.W_array()
    xbar = ph.xbar_by_node()["ROOT"]
    g = GOLD["farmer3_rho1"]
    assert abs(tb - g["trivial_bound"]) <= OBJ_REL * abs(g["trivial_bound"])
    assert np.abs(W - np.array(g["traj"][4]["W"])).max() <= ABS
    assert np.abs(xbar[:3] - np.array(g["traj"][4]["xbar"])).max() <= ABS
    # the reference's fixture files (order: scen, DevotedAcreage[crop] in sorted order)
    ref_w = {}
    with open(os.path.join(HERE, "golden", "ref_w_file.csv")) as f:
        for row in csv.reader(f):
            ref_w[(row[0], row[1])] = float(row[2])
    for s, nm in enumerate(names):
        for k, vn in enumerate(ph.batch.nonant_names):
            assert abs(W[s, k] - ref_w[(nm, vn)]) <= ABS, (nm, vn, W[s, k], ref_w[(nm, vn)])
    ref_x = {}
    with open(os.path.join(HERE, "golden", "ref_xbar_file.csv")) as f:
        for row in csv.reader(f):
            ref_x[row[0]] = float(row[1])
    for k, vn in enumerate(ph.batch.nonant_names):
        assert abs(xbar[k] - ref_x[vn]) <= ABS


def test_farmer3_iterations_to_convergence(gpu):
    """Same PH iteration count as the exact solver, +-1 (convthresh 1e-3 and 1e-4)."""
    from mpisppy_amd.examples import farmer
    g = GOLD["farmer3_rho1"]
    names = farmer.scenario_names_creator(3)
    for thresh, key in ((1e-3, "conv_1e-3_iter"), (1e-4, "conv_1e-4_iter")):
        ph = _ph(names, farmer.scenario_creator, {"num_scens": 3}, iters=300, thresh=thresh)
        conv, eobj, tb = ph.ph_main()
        assert ph.converged
        assert abs(ph._PHIter - g[key]) <= 1, (thresh, ph._PHIter, g[key])
    # per-iteration conv metric along the way matches the oracle trajectory
    ph = _ph(names, farmer.scenario_creator, {"num_scens": 3}, iters=20)
    convs = []
    ph.PH_Prep()
    ph.Iter0()
    for it in range(20):
        ph.Compute_Xbar()
        ph.Update_W()
        convs.append(ph.convergence_diff())
        ph.solve_loop(solver_options=ph.iterk_solver_options)
    ref = [t["conv"] for t in g["traj"][:20]]
    assert np.abs(np.array(convs) - np.array(ref)).max() <= 1e-5


def test_farmer30_trivial_bound(gpu):
    """test_aph.py:230-253: Scenario1..30 trivial bound -137846 (3 significant digits);
    checked here to 1e-5 relative against the LP value."""
    from mpisppy_amd.examples import farmer
    names = [f"Scenario{i + 1}" for i in range(30)]
    ph = _ph(names, farmer.scenario_creator, {}, iters=1)
    ph.PH_Prep()
    tb = ph.Iter0()
    assert abs(tb - GOLD["farmer30_trivial_bound"]) <= OBJ_REL * abs(GOLD["farmer30_trivial_bound"])
    assert round(-tb, -3) == 138000.0  # round_pos_sig(137846, 3)


@pytest.mark.parametrize("kernel", [0, 2, 3])
def test_farmer_cm10_parity(gpu, kernel):
    """Config-2 problem size (cm = 10: n=120, m=61 after presolve) on 16 scenarios vs
    the exact oracle after 5 PH iterations; batch_creator path.  scen3..18: for
    scen0..2 the cm copies of a crop are identical, so their Iter0 LP has a whole
    optimal face and only the objective (trivial bound) is solver-independent.
    kernel 0 (auto) takes path 6's subtree interior point (k_solve_ipm_blk, one wave per
    scenario, jit_ipm_blk.hip.in: the block-angular pattern's automatic choice); kernel 3 the
    workgroup PDHG (one wave per scenario, the 30-entry acreage row as a long row); kernel 2
    the wide-row register instance."""
    from mpisppy_amd.examples import farmer
    g = GOLD["farmer16_cm10_rho1"]
    names = g["names"]
    so = {"kernel": kernel}
    ph = _ph(names, farmer.scenario_creator, {"crops_multiplier": 10, "num_scens": 16},
             batch_creator=farmer.batch_creator, iter0_solver_options=so, iterk_solver_options=so)
    conv, eobj, tb = ph.ph_main()
    info = ph.engine.kernel_info()
    if kernel == 0:
        ii = ph.engine.ipm_info()
        assert info["path"] == 6 and ii["lanes"] == 64 and ii["scratch_bytes"] == 0, (info, ii)
        assert ii["kernel"] == 4, ii    # the subtree kernel, not the workgroup one (3)
    else:
        assert info["wps"] == 1 and (info["wZC"], info["wZR"]) == (3, 4), info
        assert info["instance"] >= 0 and info["lanes"] == 64 and info["ZR"] >= 30, info
    assert abs(tb - g["trivial_bound"]) <= OBJ_REL * abs(g["trivial_bound"])
    assert (ph.engine.host("status") == 0).all()
    assert np.abs(ph.W_array() - np.array(g["W5"])).max() <= ABS
    assert np.abs(ph.xbar_by_node()["ROOT"][:30] - np.array(g["xbar5"])).max() <= ABS
    assert abs(eobj - g["Eobj5"]) <= OBJ_REL * abs(g["Eobj5"])


def test_aircond_multistage_parity(gpu):
    """Config 4 at parity size: bf 4 3 2 (24 scen, 17 non-leaf nodes), QuadShortCoeff
    0.3 (QP even in Iter0), per-node x̄ and W vs the oracle; iterations to 1e-4."""
    from mpisppy_amd.examples import aircond
    from mpisppy_amd.sputils import create_nodenames_from_branching_factors
    g = GOLD["aircond432_rho1"]
    kw = dict(g["kwargs"])
    kw["branching_factors"] = g["branching_factors"]
    names = g["names"]
    nodes = create_nodenames_from_branching_factors(g["branching_factors"])
    ph = _ph(names, aircond.scenario_creator, kw, iters=5, all_nodenames=nodes)
    conv, eobj, tb = ph.ph_main()
    assert abs(tb - g["trivial_bound"]) <= OBJ_REL * abs(g["trivial_bound"])
    assert np.abs(ph.W_array() - np.array(g["traj5"][4]["W"])).max() <= ABS
    ph2 = _ph(names, aircond.scenario_creator, kw, iters=300, thresh=1e-4, all_nodenames=nodes,
              batch_creator=aircond.batch_creator)
    ph2.ph_main()
    assert ph2.converged and abs(ph2._PHIter - g["conv_1e-4_iter"]) <= 1
    nx = ph2.xbar_by_node()
    for nd, v in g["node_xbar_final"].items():
        assert np.abs(nx[nd][:2] - np.array(v)).max() <= 1e-4, nd


def _random_lp_batch(S, n, m, density, seed, with_q=False):
    """Feasible, bounded random LPs/QPs sharing one pattern (for direct C-ABI tests)."""
    from mpisppy_amd.batch import ScenarioBatch
    rng = np.random.default_rng(seed)
    mask = rng.random((m, n)) < density
    for i in range(m):
        if not mask[i].any():
            mask[i, rng.integers(n)] = True
    rows, cols = np.nonzero(mask)
    row_ptr = np.concatenate([[0], np.cumsum(mask.sum(1))]).astype(np.int32)
    nnz = rows.size
    A = rng.normal(size=(S, nnz))
    x_feas = rng.uniform(0.0, 5.0, size=(S, n))
    Ax = np.zeros((S, m))
    for k in range(nnz):
        Ax[:, rows[k]] += A[:, k] * x_feas[:, cols[k]]
    kind = rng.integers(0, 3, size=m)
    rl = np.where(kind == 1, np.inf, Ax - rng.uniform(0.1, 2.0, size=(S, m)))
    ru = np.where(kind == 0, np.inf, Ax + rng.uniform(0.1, 2.0, size=(S, m)))
    rl = np.where(kind == 1, -np.inf, rl)
    eqr = kind == 2
    rl[:, eqr] = Ax[:, eqr]
    ru[:, eqr] = Ax[:, eqr]
    lb = np.zeros((S, n))
    ub = np.full((S, n), 10.0)
    ub[:, ::3] = np.inf
    c = rng.normal(size=(S, n))
    c[:, ::3] = np.abs(c[:, ::3]) + 0.1  # unbounded-above columns get positive cost
    q = rng.uniform(0.0, 1.0, size=(S, n)) if with_q else np.zeros((S, n))
    nn = 2
    return ScenarioBatch([f"s{i}" for i in range(S)], row_ptr, cols.astype(np.int32), A, c, lb, ub, rl, ru,
                         q, np.zeros(S), np.arange(nn, dtype=np.int32), np.zeros(nn, np.int32),
                         np.arange(nn, dtype=np.int32), np.zeros((S, 1), np.int32), ["ROOT"],
                         np.full(S, 1.0 / S), np.full((S, 1), 1.0 / S))


@pytest.mark.parametrize("S,with_q", [(1, False), (67, False), (130, True)])
def test_random_batches_vs_highs_and_ipm(gpu, S, with_q):
    """Direct engine calls on random LP/QP batches with ranged, equality and one-sided
    rows and infinite bounds; S not a multiple of the 64-lane wave."""
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd import _lib
    from oracle.lpqp import solve_lp_highs, solve_qp_ipm
    b = _random_lp_batch(S, 9, 6, 0.5, seed=S, with_q=with_q)
    e = PHEngine(b, device="cuda:0")
    e.solve(_lib.default_options(), warm=False)
    st = e.host("status")
    obj = e.host("obj")
    bnd = e.host("bound")
    x = e.host("x")
    assert (st == _lib.OPTIMAL).all()
    for s in range(S):
        A = b.dense_A(s)
        if with_q:
            xr, ob, rc = solve_qp_ipm(A, b.rl[s], b.ru[s], b.lb[s], b.ub[s], b.c[s], b.q[s])
        else:
            xr, ob, rc = solve_lp_highs(A, b.rl[s], b.ru[s], b.lb[s], b.ub[s], b.c[s])
        assert rc == 0
        tol = OBJ_REL * max(1.0, abs(ob))
        assert abs(obj[s] - ob) <= tol, (s, obj[s], ob)
        assert abs(bnd[s] - ob) <= tol, (s, bnd[s], ob)
        # primal feasibility of the returned x
        ax = A @ x[s]
        assert np.all(ax >= b.rl[s] - 1e-6 * (1 + np.abs(b.rl[s])))
        assert np.all(ax <= b.ru[s] + 1e-6 * (1 + np.abs(b.ru[s])))
        assert np.all(x[s] >= b.lb[s] - 1e-9) and np.all(x[s] <= b.ub[s] + 1e-9)
    # warm start reproduces the same answer quickly
    it_cold = e.host("iters").copy()
    e.solve(_lib.default_options(), warm=True)
    assert np.abs(e.host("obj") - obj).max() <= 1e-6 * max(1.0, np.abs(obj).max())
    assert e.host("iters").max() <= it_cold.max()
    e.close()


def test_maximize_sense(gpu):
    """A maximise model (max -f, PH term subtracted, phbase.py:696-699): same x and W
    trajectory as min f; bounds / objectives come back with the model's sign
    (spopt.py:201-206 swaps Lower/Upper bound for max)."""
    from mpisppy_amd.examples import farmer
    names = farmer.scenario_names_creator(3)
    ph_min = _ph(names, farmer.scenario_creator, {"num_scens": 3}, iters=3)
    _, e1, tb1 = ph_min.ph_main()
    ph_max = _ph(names, farmer.scenario_creator, {"num_scens": 3, "sense": -1}, iters=3)
    _, e2, tb2 = ph_max.ph_main()
    assert abs(tb1 + tb2) <= 1e-6 * abs(tb1)
    assert abs(e1 + e2) <= 1e-5 * abs(e1)
    assert np.abs(ph_min.W_array() - ph_max.W_array()).max() <= ABS


def test_capi_errors_are_loud(gpu):
    from mpisppy_amd import _lib
    lib = _lib.load()
    h = ctypes.c_void_p()
    rp = np.array([0, 5], dtype=np.int32)  # row_ptr end != nnz
    ci = np.zeros(2, dtype=np.int32)
    P = lambda a: a.ctypes.data_as(_lib.P_i32)  # noqa: E731
    rc = lib.phgpu_create(ctypes.byref(h), 0, 4, 2, 1, 2, P(rp), P(ci), 0, None, None, None, 1, 1, 1)
    assert rc != 0 and "row_ptr" in _lib.last_error()
    with pytest.raises(_lib.PhgpuError):
        _lib.check(rc, "phgpu_create")


@pytest.mark.parametrize("kernel", [1, 2])
def test_both_solve_kernels_match_oracle(gpu, kernel):
    """The global-memory kernel (1) and the register-resident kernel (2) both reproduce
    the farmer 3-scenario trajectory and agree on random LP batches."""
    from mpisppy_amd.examples import farmer
    names = farmer.scenario_names_creator(3)
    opt = {"kernel": kernel}
    ph = _ph(names, farmer.scenario_creator, {"num_scens": 3}, iter0_solver_options=opt,
             iterk_solver_options=opt)
    conv, eobj, tb = ph.ph_main()
    g = GOLD["farmer3_rho1"]
    assert abs(tb - g["trivial_bound"]) <= OBJ_REL * abs(g["trivial_bound"])
    assert np.abs(ph.W_array() - np.array(g["traj"][4]["W"])).max() <= ABS


def test_register_kernel_on_random_batches(gpu):
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd import _lib
    for S, wq, seed in [(5, False, 1), (97, True, 2), (300, False, 3)]:
        b = _random_lp_batch(S, 11, 7, 0.35, seed=seed, with_q=wq)
        e = PHEngine(b, device="cuda:0")
        info = e.kernel_info()
        assert info["instance"] >= 0, info
        e.solve(_lib.default_options(kernel=1), warm=False)
        o1 = e.host("obj").copy()
        b1 = e.host("bound").copy()
        e.solve(_lib.default_options(kernel=2), warm=False)
        o2 = e.host("obj")
        assert (e.host("status") == 0).all()
        tol = OBJ_REL * np.maximum(1.0, np.abs(o1))
        assert np.all(np.abs(o1 - o2) <= tol), (o1, o2)
        assert np.all(np.abs(e.host("bound") - b1) <= tol)
        e.close()


def test_gamma_not_one_uses_global_kernel(gpu):
    """The register-resident kernel is specialised for the reflected step (gamma = 1):
    auto selection runs another gamma on the global-memory kernel, and forcing the
    register kernel with it is a loud error."""
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd import _lib
    b = _random_lp_batch(37, 11, 7, 0.35, seed=5, with_q=False)
    e = PHEngine(b, device="cuda:0")
    assert e.kernel_info()["instance"] >= 0
    e.solve(_lib.default_options(kernel=2), warm=False)
    o_ref = e.host("obj").copy()
    e.solve(_lib.default_options(kernel=0, gamma=0.5), warm=False)
    assert (e.host("status") == 0).all()
    tol = OBJ_REL * np.maximum(1.0, np.abs(o_ref))
    assert np.all(np.abs(e.host("obj") - o_ref) <= tol)
    with pytest.raises(_lib.PhgpuError):
        e.solve(_lib.default_options(kernel=2, gamma=0.5), warm=False)
    e.close()


def test_multinode_xbar_reduction_large_tree(gpu):
    """Compute_Xbar (phbase.py:27-87) on a 3-level aircond tree large enough that node
    runs span several waves and several merge chunks (bf 8 x 32 x 128: 32,768 scenarios,
    512 waves, 264 non-leaf nodes): per-node x̄ equals the host sum of prob_coeff * x,
    and two launches agree bit for bit."""
    from mpisppy_amd.examples import aircond
    from mpisppy_amd.sputils import create_nodenames_from_branching_factors
    bf = [8, 32, 128]
    kw = dict(GOLD["aircond432_rho1"]["kwargs"])
    kw["branching_factors"] = bf
    names = aircond.scenario_names_creator(int(np.prod(bf)))
    ph = _ph(names, aircond.scenario_creator, kw, iters=1, batch_creator=aircond.batch_creator,
             all_nodenames=create_nodenames_from_branching_factors(bf))
    ph.PH_Prep()
    ph.Iter0()
    ph.Compute_Xbar()
    got = ph.xbar_by_node()
    ph.Compute_Xbar()
    again = ph.xbar_by_node()
    b = ph.batch
    X = ph.nonants_array()
    exp = np.zeros((len(b.node_names), b.nlen_max))
    for k in range(b.nn):
        d, off = b.nonant_depth[k], b.nonant_off[k]
        np.add.at(exp[:, off], b.node_of[:, d], b.prob_coeff[:, d] * X[:, k])
    for g, nd in enumerate(b.node_names):
        assert np.array_equal(got[nd], again[nd]), nd
        assert np.allclose(got[nd], exp[g], rtol=1e-12, atol=1e-9), (nd, got[nd], exp[g])
