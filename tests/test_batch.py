"""Host-side data formats either side of the hot path: model builders, the shared
CSR batch, presolve, rank slicing, tree bookkeeping."""
import warnings

import numpy as np
import pytest

from mpisppy_amd.examples import farmer, aircond
from mpisppy_amd.batch import batch_from_models, fold_singleton_rows
from mpisppy_amd.sputils import rank_slices, create_nodenames_from_branching_factors, node_idx
from mpisppy_amd.spbase import nonleaf_nodenames

warnings.simplefilter("ignore")
AIR = dict(branching_factors=[4, 3, 2], Capacity=200, QuadShortCoeff=0.3, BeginInventory=50,
           mu_dev=0, sigma_dev=40, start_seed=0)


@pytest.mark.parametrize("cm", [1, 2, 11])
def test_farmer_batch_creator_equals_per_scenario(cm):
    names = farmer.scenario_names_creator(8, start=2)
    b1 = farmer.batch_creator(names, crops_multiplier=cm)
    b2 = batch_from_models(names, [farmer.scenario_creator(n, crops_multiplier=cm) for n in names])
    for f in ["A_val", "c", "lb", "ub", "rl", "ru", "q", "row_ptr", "col_idx", "nonant_col", "prob"]:
        assert np.array_equal(getattr(b1, f), getattr(b2, f)), f
    assert b1.n == 12 * cm and b1.m == 1 + 6 * cm and b1.nnz == 3 * cm + 7 * 3 * cm
    if cm == 11:  # lexicographic nonant order (scenario_tree.py:39)
        assert b1.nonant_names[:3] == ["DevotedAcreage[CORN0]", "DevotedAcreage[CORN1]", "DevotedAcreage[CORN10]"]


def test_farmer_matches_oracle_model():
    from oracle.models import farmer_scenario
    from oracle.lpqp import solve_lp_highs
    b = farmer.batch_creator(["scen0", "scen5"], crops_multiplier=2)
    for s, nm in enumerate(["scen0", "scen5"]):
        o = farmer_scenario(nm, 2)
        A, rl, ru, lb, ub, c, q = o.arrays()
        _, o1, _ = solve_lp_highs(A, rl, ru, lb, ub, c)          # oracle: quota rows kept
        _, o2, _ = solve_lp_highs(b.dense_A(s), b.rl[s], b.ru[s], b.lb[s], b.ub[s], b.c[s])  # folded
        assert abs(o1 - o2) <= 1e-9 * abs(o1)
        assert [o.var_names[j] for j in o.nonant_indices()] == b.nonant_names


def test_aircond_batch_and_tree():
    names = aircond.scenario_names_creator(24)
    nodes = create_nodenames_from_branching_factors([4, 3, 2])
    b1 = aircond.batch_creator(names, **AIR)
    b2 = batch_from_models(names, [aircond.scenario_creator(n, **AIR) for n in names],
                           all_nodenames=nodes, node_names=nonleaf_nodenames(nodes))
    for f in ["A_val", "c", "lb", "ub", "rl", "ru", "q", "node_of", "prob_coeff", "nonant_col"]:
        assert np.array_equal(getattr(b1, f), getattr(b2, f)), f
    assert b1.node_names == nonleaf_nodenames(nodes)
    assert len(b1.node_names) == 1 + 4 + 12
    # prob_coeff = pi_s / pi_node (spbase.py:390)
    assert np.allclose(b1.prob_coeff[0], [1 / 24, 1 / 6, 1 / 2])
    from oracle.models import aircond_scenario
    o = aircond_scenario("scen13", [4, 3, 2], **{k: v for k, v in AIR.items() if k != "branching_factors"})
    assert np.allclose(b1.rl[13][-4:], np.array(o.demands) - np.array([50, 0, 0, 0]))


def test_fold_singleton_rows():
    rp = np.array([0, 1, 3, 4], dtype=np.int32)
    ci = np.array([0, 0, 1, 1], dtype=np.int32)
    A = np.array([[2.0, 1.0, 1.0, -4.0]])
    lb = np.zeros((1, 2))
    ub = np.full((1, 2), 10.0)
    rl = np.array([[-np.inf, 1.0, -8.0]])
    ru = np.array([[6.0, 5.0, 4.0]])
    rp2, ci2, A2, lb2, ub2, rl2, ru2, keep = fold_singleton_rows(rp, ci, A, lb, ub, rl, ru)
    assert keep.tolist() == [False, True, False]
    assert ub2[0, 0] == 3.0 and lb2[0, 1] == 0.0 and ub2[0, 1] == 2.0
    assert rp2.tolist() == [0, 2] and A2.tolist() == [[1.0, 1.0]]


def test_rank_slices_and_node_idx():
    for S, P in [(65536, 8), (1000, 3), (24, 4), (5, 5)]:
        sl = rank_slices(S, P)
        assert sum(len(x) for x in sl) == S and sl[0][0] == 0 and sl[-1][-1] == S - 1
        avg = S / P
        assert all(x[0] == int(i * avg) for i, x in enumerate(sl))
    assert node_idx([], [4, 3, 2]) == 0 and node_idx([1], [4, 3, 2]) == 2 and node_idx([1, 2], [4, 3, 2]) == 10


def test_drop_duplicate_rows_checks_every_scenario():
    """A row is dropped only if an earlier row equals it in EVERY scenario (the UC
    production-cost rows, ReferenceModel_OK.py:1466-1470); rows equal in scenario 0 only
    are kept."""
    from mpisppy_amd.batch import drop_duplicate_rows
    row_ptr = np.array([0, 2, 4, 6, 8], dtype=np.int32)
    col_idx = np.array([0, 1, 0, 1, 0, 1, 1, 2], dtype=np.int32)
    A = np.array([[1.0, 2.0, 1.0, 2.0, 1.0, 2.0, 3.0, 4.0],
                  [1.0, 2.0, 1.0, 2.0, 1.0, 5.0, 3.0, 4.0]])      # row 2 differs in scenario 1
    rl = np.array([[0.0, 0.0, 0.0, -np.inf], [0.0, 0.0, 0.0, -np.inf]])
    ru = np.array([[1.0, 1.0, 1.0, 2.0], [1.0, 1.0, 1.0, 2.0]])
    rp, ci, Av, l, u, keep = drop_duplicate_rows(row_ptr, col_idx, A, rl, ru)
    assert keep.tolist() == [True, False, True, True]
    assert rp.tolist() == [0, 2, 4, 6] and ci.tolist() == [0, 1, 0, 1, 1, 2]
    assert Av.shape == (2, 6) and l.shape == (2, 3) and u.shape == (2, 3)
