"""Vectorised exact farmer oracle for headline-scale parity (TEST INFRASTRUCTURE ONLY).

The farmer scenario (examples/farmer/farmer.py:85-224) is separable per crop once the
recourse variables are eliminated: crop k's first + second stage cost is a convex
piecewise-linear function g_k(x_k) of its acreage, coupled only by the acreage row
sum_k x_k <= 500 cm (farmer.py:181-184).  Per crop (farmer.py:186-222, data :127-150):

  * WHEAT / CORN: buy the feed shortfall (req - Y x)+ at PurchasePrice, sell the surplus
    at SubQuotaSellingPrice up to the 1e5 quota, then at SuperQuotaSellingPrice (0):
    slopes  plant - buy Y | plant - sub Y | plant - super Y
    kinks   req / Y       | (req + 1e5) / Y
  * SUGAR_BEETS: sell up to the 6000 quota at 36, then at 10:
    slopes  260 - 36 Y    | 260 - 10 Y
    kinks   6000 / Y

(The quota kink of WHEAT / CORN only matters once 500 cm acres of one crop can exceed
it -- cm >= ~28, e.g. the cm = 64 variant of config 3.)

Solvers, all vectorised over scenarios with numpy:

  * ``iter0_lp``: the Iter0 LP (W_on = prox_on = 0, phbase.py:594-597): a fractional
    knapsack -- the segments with negative slope are filled in slope order until the
    acreage is used up (exact; unique x when no two slopes tie).
  * ``prox``: the PH subproblem  min sum_k g_k(x_k) + W_k x_k + rho/2 (x_k - xbar_k)^2
    s.t. sum x_k <= 500 cm (phbase.py:617-699): for a multiplier lam of the acreage row
    each crop's minimiser is  b0 + sum_i clamp(xbar - (s_i + W + lam)/rho - b_{i-1}, 0,
    b_i - b_{i-1}); lam >= 0 by bisection (the same closed form as lpqp.farmer_prox_exact,
    which tests/test_oracle_golden.py pins against the reference's w_test_data).

``FarmerVecPH`` restates PHBase.Iter0 / iterk_loop (phbase.py:758-979) for a
single-rank run on these solvers.  It is checked against HiGHS (LP) and
lpqp.farmer_prox_exact on samples in tests/test_oracle_scale.py.
"""
import math

import numpy as np

from .models import extract_num

_PLANT = {"WHEAT": 150.0, "CORN": 230.0, "SUGAR_BEETS": 260.0}
_REQ = {"WHEAT": 200.0, "CORN": 240.0}
_BUY = {"WHEAT": 238.0, "CORN": 210.0}
_SUB = {"WHEAT": 170.0, "CORN": 150.0, "SUGAR_BEETS": 36.0}
_SUPER = {"WHEAT": 0.0, "CORN": 0.0, "SUGAR_BEETS": 10.0}
_QUOTA = {"WHEAT": 100000.0, "CORN": 100000.0, "SUGAR_BEETS": 6000.0}
_BASE_Y = [
    {"WHEAT": 2.0, "CORN": 2.4, "SUGAR_BEETS": 16.0},   # BelowAverageScenario
    {"WHEAT": 2.5, "CORN": 3.0, "SUGAR_BEETS": 20.0},   # AverageScenario
    {"WHEAT": 3.0, "CORN": 3.6, "SUGAR_BEETS": 24.0},   # AboveAverageScenario
]
_BASES = ["WHEAT", "CORN", "SUGAR_BEETS"]


def crops_insertion(cm):
    """CROPS order (farmer.py:99-105)."""
    return [b + str(i) for i in range(cm) for b in _BASES]


def crops_sorted(cm):
    """Nonant order: DevotedAcreage expanded in sorted key order (scenario_tree.py:39)."""
    return sorted(crops_insertion(cm))


def yields(names, cm, seedoffset=0):
    """[S, 3cm] yields in CROPS order (farmer.py:52-60, 151-157)."""
    out = np.empty((len(names), 3 * cm))
    for s, nm in enumerate(names):
        num = extract_num(nm)
        base = _BASE_Y[num % 3]
        y = np.array([base[b] for b in _BASES] * cm)
        if num // 3 != 0:
            st = np.random.RandomState()
            st.seed(num + seedoffset)
            y = y + st.rand(3 * cm)
        out[s] = y
    return out


def pieces(Y, cm):
    """Breakpoints [S, K, 4] and slopes [S, K, 3] of g_k on [0, 500 cm] plus g_k(0)
    [S, K], in the SORTED nonant order (K = 3 cm)."""
    total = 500.0 * cm
    ins = crops_insertion(cm)
    order = [ins.index(c) for c in crops_sorted(cm)]
    Y = Y[:, order]
    S, K = Y.shape
    bases = [c.rstrip("0123456789") for c in crops_sorted(cm)]
    bp = np.zeros((S, K, 4))
    sl = np.zeros((S, K, 3))
    f0 = np.zeros((S, K))
    for k, b in enumerate(bases):
        y = Y[:, k]
        if b in ("WHEAT", "CORN"):
            k1 = _REQ[b] / y
            k2 = (_REQ[b] + _QUOTA[b]) / y
            sl[:, k] = np.stack([_PLANT[b] - _BUY[b] * y, _PLANT[b] - _SUB[b] * y,
                                 _PLANT[b] - _SUPER[b] * y], axis=1)
            f0[:, k] = _BUY[b] * _REQ[b]
        else:
            k1 = _QUOTA[b] / y
            k2 = np.full_like(y, np.inf)
            sl[:, k] = np.stack([_PLANT[b] - _SUB[b] * y, _PLANT[b] - _SUPER[b] * y,
                                 _PLANT[b] - _SUPER[b] * y], axis=1)
        bp[:, k, 1] = np.minimum(k1, total)
        bp[:, k, 2] = np.minimum(k2, total)
        bp[:, k, 3] = total
    return bp, sl, f0


def crop_cost(bp, sl, f0, x):
    """g_k(x_k), [S, K]."""
    seg = np.clip(x[..., None] - bp[..., :-1], 0.0, np.diff(bp, axis=-1))
    return f0 + (sl * seg).sum(-1)


def iter0_lp(bp, sl, f0, total, ties="symmetric"):
    """Exact Iter0 LP: fractional knapsack over the negative-slope segments.

    ``ties``: the point taken on an optimal face (exact slope ties, below): "symmetric"
    (the analytic-centre point an interior-point solve converges to, the fixtures' choice)
    or "vertex" (the stable slope order fills the first tied segment first -- a basic
    solution, what a simplex solver such as the reference's would return).  The objective
    and every tied group's total acreage are the same either way."""
    S, K, J = sl.shape
    length = np.diff(bp, axis=-1).reshape(S, K * J)
    slope = sl.reshape(S, K * J)
    order = np.argsort(slope, axis=1, kind="stable")
    sl_o = np.take_along_axis(slope, order, 1)
    len_o = np.where(sl_o < 0.0, np.take_along_axis(length, order, 1), 0.0)
    before = np.cumsum(len_o, axis=1) - len_o
    fill_o = np.clip(total - before, 0.0, len_o)
    # Exact slope ties (scen0..2 with cm > 1: their crop copies have identical yields, so
    # the optimum is a face, not a vertex): the acreage a tied group receives is split over
    # its segments in proportion to their lengths -- for identical copies the symmetric
    # point of the face, the solution an interior-point solve (the analytic centre) or a
    # PDHG solve from a symmetric start converges to.  The objective is unchanged.  The
    # reference's own point there depends on its solver (a simplex basis: ties="vertex"),
    # and so does every later PH iterate of a batch holding these scenarios.
    tied = (np.diff(sl_o, axis=1) == 0.0) & (len_o[:, 1:] > 0.0) & (len_o[:, :-1] > 0.0)
    for s in (np.nonzero(tied.any(1))[0] if ties == "symmetric" else []):
        k = 0
        while k < K * J:
            e = k + 1
            while e < K * J and sl_o[s, e] == sl_o[s, k] and len_o[s, e] > 0.0:
                e += 1
            if e - k > 1 and len_o[s, k] > 0.0:
                tot_fill, tot_len = fill_o[s, k:e].sum(), len_o[s, k:e].sum()
                fill_o[s, k:e] = tot_fill * len_o[s, k:e] / tot_len
            k = e
    fill = np.empty_like(fill_o)
    np.put_along_axis(fill, order, fill_o, 1)
    x = fill.reshape(S, K, J).sum(-1)
    obj = f0.sum(1) + (slope * fill).sum(1)
    return x, obj


def lp_margin(bp, sl, total):
    """Conditioning of the Iter0 LP: the slope gap between the marginal segment (the one
    the acreage row cuts) and its nearest neighbour in slope order ([S]; inf when the
    acreage row is slack).  A tiny margin is a near-tie: the optimum is unique but a
    first-order method needs ~1/margin iterations to pick the right crop."""
    S, K, J = sl.shape
    length = np.diff(bp, axis=-1).reshape(S, K * J)
    slope = sl.reshape(S, K * J)
    order = np.argsort(slope, axis=1, kind="stable")
    s_o = np.take_along_axis(slope, order, 1)
    l_o = np.where(s_o < 0.0, np.take_along_axis(length, order, 1), 0.0)
    cum = np.cumsum(l_o, axis=1)
    out = np.full(S, np.inf)
    for s in range(S):
        k = int(np.searchsorted(cum[s], total))
        if k >= K * J or s_o[s, k] >= 0.0:
            continue
        nb = [abs(s_o[s, k] - s_o[s, kk]) for kk in (k - 1, k + 1)
              if 0 <= kk < K * J and l_o[s, kk] > 0 and kk != k]
        out[s] = min(nb) if nb else np.inf
    return out


def _x_of_lam(bp, sl, lin, rho, xbar, lam):
    a = xbar[..., None] - (sl + (lin + lam[:, None])[..., None]) / rho[..., None]
    return bp[..., 0] + np.clip(a - bp[..., :-1], 0.0, np.diff(bp, axis=-1)).sum(-1)


def prox(bp, sl, f0, W, xbar, rho, total, iters=200, method="auto"):
    """Exact PH subproblem for all scenarios: (x [S, K], augmented objective [S]).

    ``method="breakpoints"`` finds the acreage multiplier exactly: sum_k x_k(lam)
    is piecewise linear and nonincreasing in lam, with kinks where a segment term of
    ``_x_of_lam`` enters or leaves its clip range (lam = rho (xbar - b) - s - W for every
    segment end b); it is evaluated at every kink >= 0 and interpolated linearly on the
    piece that crosses the acreage ``total``.  ``method="bisect"`` bisects lam (``iters``
    halvings); the two agree to rounding (tests/test_oracle_scale.py).  ``"auto"`` takes
    the kinks for few crops (cm = 1: 6x faster) and bisection for many (the kink table
    grows as K^2 per scenario)."""
    if method == "auto":
        method = "breakpoints" if sl.shape[1] <= 6 else "bisect"
    if method == "breakpoints":
        return _prox_breakpoints(bp, sl, f0, W, xbar, rho, total)
    S = bp.shape[0]
    lam = np.zeros(S)
    x = _x_of_lam(bp, sl, W, rho, xbar, lam)
    over = x.sum(1) > total
    if over.any():
        lo = np.zeros(S)
        hi = np.ones(S)
        while True:
            bad = over & (_x_of_lam(bp, sl, W, rho, xbar, hi).sum(1) > total)
            if not bad.any():
                break
            hi[bad] *= 2.0
        for _ in range(iters):
            mid = 0.5 * (lo + hi)
            gt = _x_of_lam(bp, sl, W, rho, xbar, mid).sum(1) > total
            lo = np.where(gt, mid, lo)
            hi = np.where(gt, hi, mid)
        xh = _x_of_lam(bp, sl, W, rho, xbar, hi)
        x = np.where(over[:, None], xh, x)
    obj = crop_cost(bp, sl, f0, x).sum(1) + (W * x).sum(1) + 0.5 * (rho * (x - xbar) ** 2).sum(1)
    return x, obj


def _prox_breakpoints(bp, sl, f0, W, xbar, rho, total, chunk_elems=1 << 24):
    S, K, J = sl.shape
    xbar = np.broadcast_to(xbar, W.shape)
    rho = np.broadcast_to(rho, W.shape)
    x = _x_of_lam(bp, sl, W, rho, xbar, np.zeros(S))
    over = np.nonzero(x.sum(1) > total)[0]
    P = 2 * K * J + 1
    step = max(1, chunk_elems // (P * K * J))
    for a in range(0, len(over), step):
        ix = over[a:a + step]
        b, s_, w, r, xb = bp[ix], sl[ix], W[ix], rho[ix], xbar[ix]
        # kinks: lam where xbar - (s_i + W + lam) / rho equals b_{i-1} or b_i
        base = (r * xb - w)[..., None] - s_                              # [n, K, J]
        kinks = np.concatenate([base - r[..., None] * b[..., :-1], base - r[..., None] * b[..., 1:]], axis=2)
        kinks = np.where(np.isfinite(kinks), kinks, 0.0).reshape(len(ix), -1)
        lam = np.sort(np.concatenate([np.zeros((len(ix), 1)), np.maximum(kinks, 0.0)], axis=1), axis=1)
        av = xb[:, None, :, None] - (s_[:, None] + (w[:, None, :] + lam[:, :, None])[..., None]) / r[:, None, :, None]
        seg = np.clip(av - b[:, None, :, :-1], 0.0, np.diff(b, axis=-1)[:, None])
        tot = (b[:, None, :, 0] + seg.sum(-1)).sum(-1)                    # [n, P], nonincreasing
        j = np.argmax(tot <= total, axis=1)                               # first kink at or below
        rows = np.arange(len(ix))
        l1, l2 = lam[rows, j - 1], lam[rows, j]
        t1, t2 = tot[rows, j - 1], tot[rows, j]
        lam_star = l1 + (t1 - total) * (l2 - l1) / (t1 - t2)
        x[ix] = _x_of_lam(b, s_, w, r, xb, lam_star)
    obj = crop_cost(bp, sl, f0, x).sum(1) + (W * x).sum(1) + 0.5 * (rho * (x - xbar) ** 2).sum(1)
    return x, obj


class FarmerVecPH:
    """Single-rank PH on the vectorised farmer solvers (phbase.py:758-979)."""

    def __init__(self, names, cm, rho=1.0, num_scens=None, seedoffset=0, ties="symmetric"):
        self.names = list(names)
        self.cm = cm
        self.total = 500.0 * cm
        self.S = len(self.names)
        self.K = 3 * cm
        self.prob = np.full(self.S, 1.0 / (num_scens or self.S))   # spbase.py:515-520
        self.bp, self.sl, self.f0 = pieces(yields(self.names, cm, seedoffset), cm)
        self.rho = np.full((self.S, self.K), float(rho))
        self.W = np.zeros((self.S, self.K))
        self.xbar = np.zeros((self.S, self.K))
        self.history = []
        self.ties = ties

    def iter0(self):
        self.x, self.obj = iter0_lp(self.bp, self.sl, self.f0, self.total, ties=self.ties)
        self.iter0_x = self.x.copy()
        self.iter0_obj = self.obj.copy()
        self.trivial_bound = math.fsum(self.prob * self.obj)        # spopt.py:346-391
        return self.trivial_bound

    def compute_xbar(self):                                          # phbase.py:27-107
        xb = (self.prob[:, None] * self.x).sum(0)              # prob_coeff = pi_s / pi_ROOT
        self.xbar[:] = xb
        return xb

    def iterk_loop(self, max_iterations, convthresh=-1.0):
        for it in range(1, max_iterations + 1):
            xb = self.compute_xbar()
            self.W += self.rho * (self.x - self.xbar)                # phbase.py:293-318
            conv = np.abs(self.x - self.xbar).sum() / (self.S * self.K)   # :321-343
            self.history.append({"iter": it, "conv": conv, "xbar": xb.copy()})
            if conv < convthresh:
                return it
            self.x, self.obj = prox(self.bp, self.sl, self.f0, self.W, self.xbar, self.rho, self.total)
        return max_iterations

    def Eobjective(self):
        return math.fsum(self.prob * self.obj)
