"""Batched scenario container: one shared CSR pattern + per-scenario arrays.

This is the data format either side of the hot path.  All local scenarios of a
rank must share one sparsity pattern; they differ only in
coefficient, bound / right-hand-side and objective arrays.

Layout (host, numpy, scenario-major ``[S, k]``; the engine transposes to the device's
scenario-fastest ``[k, S]`` layout):

  row_ptr[m+1], col_idx[nnz]         int32  shared CSR pattern (rows sorted by col)
  A_val[S, nnz]                      f64    per-scenario values in CSR order
  c, lb, ub, q[S, n]                 f64    objective, column bounds, diag quadratic
  rl, ru[S, m]                       f64    row ranges (+-inf allowed)
  obj_const[S]                       f64
  nonant_col[nn]                     int32  column of flat nonant k (node-list order,
                                            then sorted index: spbase.py:293-302,
                                            scenario_tree.py:39)
  nonant_depth[nn], nonant_off[nn]   int32  tree depth of its node / offset in node
  node_of[S, D]                      int32  global node id of the scenario's depth-d node
  prob[S], prob_coeff[S, D]          f64    pi_s and pi_s / pi_node (spbase.py:378-391)

Everything is stored for a *minimisation*; a maximise model is negated on entry
(the PH term is then added, matching phbase.py:696-699's subtraction) and ``sense``
records -1 so objective values / bounds are negated back.
"""
import numpy as np

from .model import LinearModel, INF


class ScenarioBatch:
    def __init__(self, names, row_ptr, col_idx, A_val, c, lb, ub, rl, ru, q, obj_const,
                 nonant_col, nonant_depth, nonant_off, node_of, node_names, prob, prob_coeff,
                 sense=1, var_names=None, nonant_names=None):
        self.names = list(names)
        self.row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int32)
        self.col_idx = np.ascontiguousarray(col_idx, dtype=np.int32)
        self.A_val = np.ascontiguousarray(A_val, dtype=np.float64)
        self.c = np.ascontiguousarray(c, dtype=np.float64)
        self.lb = np.ascontiguousarray(lb, dtype=np.float64)
        self.ub = np.ascontiguousarray(ub, dtype=np.float64)
        self.rl = np.ascontiguousarray(rl, dtype=np.float64)
        self.ru = np.ascontiguousarray(ru, dtype=np.float64)
        self.q = np.ascontiguousarray(q, dtype=np.float64)
        self.obj_const = np.ascontiguousarray(obj_const, dtype=np.float64)
        self.nonant_col = np.ascontiguousarray(nonant_col, dtype=np.int32)
        self.nonant_depth = np.ascontiguousarray(nonant_depth, dtype=np.int32)
        self.nonant_off = np.ascontiguousarray(nonant_off, dtype=np.int32)
        self.node_of = np.ascontiguousarray(node_of, dtype=np.int32)
        self.node_names = list(node_names)
        self.prob = np.ascontiguousarray(prob, dtype=np.float64)
        self.prob_coeff = np.ascontiguousarray(prob_coeff, dtype=np.float64)
        self.sense = int(sense)
        self.var_names = var_names
        self.nonant_names = nonant_names
        self.validate()

    # -- sizes
    @property
    def S(self):
        return self.A_val.shape[0]

    @property
    def n(self):
        return self.c.shape[1]

    @property
    def m(self):
        return self.rl.shape[1]

    @property
    def nnz(self):
        return self.col_idx.shape[0]

    @property
    def nn(self):
        return self.nonant_col.shape[0]

    @property
    def depth(self):
        return self.node_of.shape[1]

    @property
    def nlen_max(self):
        return int(self.nonant_off.max()) + 1 if self.nn else 0

    def nlens(self):
        """nonants per depth (all nodes of one depth carry the same count)."""
        return np.bincount(self.nonant_depth, minlength=self.depth)

    def validate(self):
        S, n, m, nnz = self.S, self.n, self.m, self.nnz
        assert self.row_ptr.shape == (m + 1,) and self.row_ptr[0] == 0 and self.row_ptr[-1] == nnz
        assert np.all(np.diff(self.row_ptr) >= 0)
        assert nnz == 0 or (self.col_idx.min() >= 0 and self.col_idx.max() < n)
        for a in (self.c, self.lb, self.ub, self.q):
            assert a.shape == (S, n)
        for a in (self.rl, self.ru):
            assert a.shape == (S, m)
        assert self.A_val.shape == (S, nnz)
        assert self.obj_const.shape == (S,)
        nn = self.nn
        assert self.nonant_depth.shape == (nn,) and self.nonant_off.shape == (nn,)
        assert nn == 0 or (self.nonant_col.min() >= 0 and self.nonant_col.max() < n)
        assert len(set(self.nonant_col.tolist())) == nn, "a column is nonant twice"
        assert self.node_of.shape[0] == S and self.prob.shape == (S,)
        assert self.prob_coeff.shape == self.node_of.shape
        assert np.all(self.lb <= self.ub), "empty column bound interval"
        assert np.all(self.rl <= self.ru), "empty row range"

    # -- helpers
    def transposed_pattern(self):
        """CSC of the shared pattern: (col_ptr[n+1], row_idx[nnz], perm[nnz]) with
        perm[k_csc] = k_csr, so per-scenario values in CSC order are A_val[:, perm]."""
        m, n = self.m, self.n
        rows = np.repeat(np.arange(m, dtype=np.int64), np.diff(self.row_ptr))
        order = np.lexsort((rows, self.col_idx))
        col_ptr = np.zeros(n + 1, dtype=np.int32)
        np.add.at(col_ptr, self.col_idx.astype(np.int64) + 1, 1)
        col_ptr = np.cumsum(col_ptr).astype(np.int32)
        return col_ptr, rows[order].astype(np.int32), order.astype(np.int32)

    def dense_A(self, s):
        A = np.zeros((self.m, self.n))
        for r in range(self.m):
            for k in range(self.row_ptr[r], self.row_ptr[r + 1]):
                A[r, self.col_idx[k]] += self.A_val[s, k]
        return A

    def subset(self, idx):
        """Batch of the scenarios ``idx`` (same pattern)."""
        idx = np.asarray(idx, dtype=np.int64)
        return ScenarioBatch([self.names[i] for i in idx], self.row_ptr, self.col_idx,
                             self.A_val[idx], self.c[idx], self.lb[idx], self.ub[idx],
                             self.rl[idx], self.ru[idx], self.q[idx], self.obj_const[idx],
                             self.nonant_col, self.nonant_depth, self.nonant_off,
                             self.node_of[idx], self.node_names, self.prob[idx],
                             self.prob_coeff[idx], self.sense, self.var_names, self.nonant_names)


# ---------------------------------------------------------------- presolve
def fold_singleton_rows(row_ptr, col_idx, A_val, lb, ub, rl, ru):
    """Fold rows that hold a single pattern entry into the column bounds.

    ``rl <= a x_j <= ru`` becomes ``x_j in [rl/a, ru/a]`` (swapped for a < 0),
    intersected with the existing bounds.  The optimum set is unchanged (the
    reference's EnforceQuotas rows, farmer.py:199-202, and aircond's MaximumCapacity,
    aircond.py:137-139, are such rows).  Rows whose coefficient is zero in some
    scenario are kept.  Returns the reduced arrays and the kept-row mask.
    """
    m = rl.shape[1]
    counts = np.diff(row_ptr)
    keep = np.ones(m, dtype=bool)
    lb = lb.copy()
    ub = ub.copy()
    for r in np.nonzero(counts == 1)[0]:
        k = row_ptr[r]
        j = col_idx[k]
        a = A_val[:, k]
        if np.any(a == 0.0):
            continue
        lo = np.where(a > 0, rl[:, r] / a, ru[:, r] / a)
        hi = np.where(a > 0, ru[:, r] / a, rl[:, r] / a)
        lb[:, j] = np.maximum(lb[:, j], lo)
        ub[:, j] = np.minimum(ub[:, j], hi)
        keep[r] = False
    if keep.all():
        return row_ptr, col_idx, A_val, lb, ub, rl, ru, keep
    ent_keep = np.repeat(keep, counts)
    new_ptr = np.concatenate([[0], np.cumsum(counts[keep])]).astype(np.int32)
    return (new_ptr, col_idx[ent_keep], A_val[:, ent_keep], lb, ub, rl[:, keep], ru[:, keep], keep)


def drop_duplicate_rows(row_ptr, col_idx, A_val, rl, ru):
    """Drop rows that repeat an earlier row exactly (same columns, same coefficients
    and same range in every scenario).  The feasible set is unchanged.  The UC model
    declares its production-cost row once per piecewise segment
    (ReferenceModel_OK.py:1466-1470: indexed by (g, t, i), the body does not use i),
    which would otherwise add ~15k redundant rows and ~40% of the nonzeros.  Returns
    the reduced arrays and the kept-row mask.

    Candidates are found on the first scenario only (a dict keyed by its row bytes, so
    no copy of the S-scenario arrays is held), and a candidate is dropped only after its
    coefficients and range compare equal to the earlier row's in every scenario."""
    m = rl.shape[1]
    keep = np.ones(m, dtype=bool)
    seen = {}
    for r in range(m):
        a, b = row_ptr[r], row_ptr[r + 1]
        if b == a:
            continue
        key = (col_idx[a:b].tobytes(), A_val[0, a:b].tobytes(), rl[0, r].tobytes(), ru[0, r].tobytes())
        first = seen.setdefault(key, [])
        for r0 in first:
            a0 = row_ptr[r0]
            if (np.array_equal(A_val[:, a:b], A_val[:, a0:a0 + (b - a)]) and np.array_equal(rl[:, r], rl[:, r0])
                    and np.array_equal(ru[:, r], ru[:, r0])):
                keep[r] = False
                break
        else:
            first.append(r)
    if keep.all():
        return row_ptr, col_idx, A_val, rl, ru, keep
    counts = np.diff(row_ptr)
    ent_keep = np.repeat(keep, counts)
    new_ptr = np.concatenate([[0], np.cumsum(counts[keep])]).astype(np.int32)
    return new_ptr, col_idx[ent_keep], A_val[:, ent_keep], rl[:, keep], ru[:, keep], keep


# ---------------------------------------------------------------- from models
def _nonleaf_node_ids(models, all_nodenames):
    """Global node ids (index into the nonleaf node list) in all_nodenames order."""
    if all_nodenames is None:
        all_nodenames = ["ROOT"]
    used = set()
    for mdl in models:
        for nd in mdl._mpisppy_node_list:
            used.add(nd.name)
    names = [nd for nd in all_nodenames if nd in used]
    extra = sorted(used - set(names))
    return names + extra


def batch_from_models(names, models, all_nodenames=None, num_all_scens=None, presolve=True,
                      node_names=None):
    """Build a ScenarioBatch from per-scenario LinearModels (the SPBase path:
    spbase.py:255-320 -- creation, probabilities, nlens, nonant indices)."""
    S = len(models)
    assert S > 0
    m0 = models[0]
    n = m0.n
    # pattern: per row the sorted union of columns over all scenarios
    pattern = []
    for r in range(m0.m):
        cols = set()
        for mdl in models:
            cols.update(j for (j, _) in mdl.rows[r][0])
        pattern.append(sorted(cols))
    row_ptr = np.zeros(m0.m + 1, dtype=np.int32)
    row_ptr[1:] = np.cumsum([len(p) for p in pattern])
    col_idx = np.array([j for p in pattern for j in p], dtype=np.int32)
    nnz = col_idx.size
    A_val = np.zeros((S, nnz))
    rl = np.empty((S, m0.m))
    ru = np.empty((S, m0.m))
    c = np.empty((S, n))
    q = np.empty((S, n))
    lb = np.empty((S, n))
    ub = np.empty((S, n))
    oc = np.empty(S)
    sense = 1 if m0.sense_min else -1
    for s, mdl in enumerate(models):
        if mdl.n != n or mdl.m != m0.m:
            raise RuntimeError(f"scenario {names[s]} does not share the pattern of {names[0]}")
        if (1 if mdl.sense_min else -1) != sense:
            raise RuntimeError("All scenario models must have the same sense (spbase.py:122-139)")
        for r, (terms, lo, hi, _) in enumerate(mdl.rows):
            base = row_ptr[r]
            pos = {j: base + i for i, j in enumerate(pattern[r])}
            for (j, a) in terms:
                A_val[s, pos[j]] += a
            rl[s, r] = lo
            ru[s, r] = hi
        c[s] = mdl.cost
        q[s] = mdl.quad
        lb[s] = mdl.lb
        ub[s] = mdl.ub
        oc[s] = mdl.obj_const
    if sense < 0:
        c, q, oc = -c, -q, -oc
    if presolve:
        row_ptr, col_idx, A_val, lb, ub, rl, ru, _ = fold_singleton_rows(row_ptr, col_idx, A_val,
                                                                        lb, ub, rl, ru)
        row_ptr, col_idx, A_val, rl, ru, _ = drop_duplicate_rows(row_ptr, col_idx, A_val, rl, ru)
    # nonants / tree (spbase.py:293-320, 378-391)
    if node_names is None:
        node_names = _nonleaf_node_ids(models, all_nodenames)
    node_id = {nd: i for i, nd in enumerate(node_names)}
    nl0 = m0._mpisppy_node_list
    D = len(nl0)
    nonant_col, nonant_depth, nonant_off = [], [], []
    for d, nd in enumerate(nl0):
        for o, v in enumerate(nd.nonant_vardata_list):
            nonant_col.append(v.index)
            nonant_depth.append(d)
            nonant_off.append(o)
    node_of = np.empty((S, D), dtype=np.int32)
    prob = np.empty(S)
    prob_coeff = np.empty((S, D))
    num_all = num_all_scens if num_all_scens is not None else S
    for s, mdl in enumerate(models):
        nl = mdl._mpisppy_node_list
        if len(nl) != D:
            raise RuntimeError("all scenarios must have the same number of tree nodes")
        p = mdl._mpisppy_probability
        if p is None or p == "uniform":
            p = 1.0 / num_all                         # spbase.py:515-520
        prob[s] = p
        uncond = 1.0
        for d, nd in enumerate(nl):
            if d > 0:
                uncond *= nd.cond_prob
            node_of[s, d] = node_id[nd.name]
            prob_coeff[s, d] = p / uncond             # spbase.py:390
            if [v.index for v in nd.nonant_vardata_list] != \
                    [nonant_col[k] for k in range(len(nonant_col)) if nonant_depth[k] == d]:
                raise RuntimeError("nonant columns differ between scenarios")
    var_names = [v.name for v in m0.vars]
    nonant_names = [var_names[j] for j in nonant_col]
    return ScenarioBatch(names, row_ptr, col_idx, A_val, c, lb, ub, rl, ru, q, oc,
                         nonant_col, nonant_depth, nonant_off, node_of, node_names, prob,
                         prob_coeff, sense, var_names, nonant_names)
