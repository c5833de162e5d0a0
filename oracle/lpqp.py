"""Exact per-scenario LP/QP solvers for the oracle (TEST INFRASTRUCTURE ONLY).

They stand in for the external solver that SPOpt.solve_one reaches through Pyomo's
SolverFactory (spopt.py:85-223): given one scenario's augmented objective
(phbase.py:617-699) they return the optimal x, the objective and an outer bound.

* ``solve_lp_highs``   -- scipy-bundled HiGHS (simplex; exact vertex) for the pure
                          LPs of Iter0 (W_on = prox_on = 0, phbase.py:594-597).
* ``solve_qp_ipm``     -- dense Mehrotra predictor-corrector interior point for
                          diagonal-Q QPs, followed by an active-set polish (one
                          equality-constrained KKT solve), giving ~1e-12 accuracy on
                          the small scenario QPs used in parity tests.
* ``farmer_prox_exact``-- closed form for the farmer prox QP:
                          per crop the second stage is a convex piecewise-linear
                          function of the acreage, so the QP is separable except for
                          the acreage row, solved by bisection on its multiplier.
"""
import numpy as np
from scipy.optimize import linprog

INF = float("inf")


# ------------------------------------------------------------------ HiGHS LP
def solve_lp_highs(A, rl, ru, lb, ub, c):
    """min c'x s.t. rl <= Ax <= ru, lb <= x <= ub via scipy HiGHS (dual simplex)."""
    m = A.shape[0]
    eq = np.isfinite(rl) & np.isfinite(ru) & (rl == ru)
    A_eq = A[eq]
    b_eq = rl[eq]
    ub_rows = (~eq) & np.isfinite(ru)
    lb_rows = (~eq) & np.isfinite(rl)
    A_ub = np.vstack([A[ub_rows], -A[lb_rows]]) if m else np.zeros((0, A.shape[1]))
    b_ub = np.concatenate([ru[ub_rows], -rl[lb_rows]])
    bounds = [(None if not np.isfinite(l) else l, None if not np.isfinite(u) else u)
              for l, u in zip(lb, ub)]
    res = linprog(c, A_ub=A_ub if len(b_ub) else None, b_ub=b_ub if len(b_ub) else None,
                  A_eq=A_eq if eq.any() else None, b_eq=b_eq if eq.any() else None,
                  bounds=bounds, method="highs-ds",
                  options={"primal_feasibility_tolerance": 1e-10,
                           "dual_feasibility_tolerance": 1e-10})
    if res.status != 0:
        return None, None, res.status
    return res.x, float(res.fun), 0


# ------------------------------------------------------------------ HiGHS QP (stock solver)
def solve_qp_highs(A, rl, ru, lb, ub, c, q):
    """min c'x + 1/2 sum q x^2 s.t. rl <= Ax <= ru, lb <= x <= ub with the HiGHS QP solver
    bundled in scipy (scipy.optimize._highspy, HiGHS 1.8.0; its active-set QP), default
    options: the "stock solver" timing of BASELINE.md section 4.  Its x is only accurate to
    ~4e-3 on the farmer prox QPs, so it is a timing reference, not a parity
    oracle.  Returns (x, obj, status) with status 0 = optimal."""
    from scipy.optimize._highspy import _core as hc
    A = np.asarray(A, dtype=np.float64)
    m, n = A.shape
    csc_start, csc_index, csc_value = [0], [], []
    for j in range(n):
        nzr = np.nonzero(A[:, j])[0]
        csc_index.extend(nzr.tolist())
        csc_value.extend(A[nzr, j].tolist())
        csc_start.append(len(csc_index))
    inf = hc.kHighsInf
    fin = lambda v, d: float(v) if np.isfinite(v) else d  # noqa: E731
    lp = hc.HighsLp()
    lp.num_col_, lp.num_row_ = n, m
    lp.col_cost_ = np.asarray(c, dtype=np.float64)
    lp.col_lower_ = np.array([fin(v, -inf) for v in lb])
    lp.col_upper_ = np.array([fin(v, inf) for v in ub])
    lp.row_lower_ = np.array([fin(v, -inf) for v in rl])
    lp.row_upper_ = np.array([fin(v, inf) for v in ru])
    lp.a_matrix_.format_ = hc.MatrixFormat.kColwise if hasattr(hc, "MatrixFormat") else lp.a_matrix_.format_
    lp.a_matrix_.start_ = np.array(csc_start, dtype=np.int32)
    lp.a_matrix_.index_ = np.array(csc_index, dtype=np.int32)
    lp.a_matrix_.value_ = np.array(csc_value, dtype=np.float64)
    lp.a_matrix_.num_col_, lp.a_matrix_.num_row_ = n, m
    model = hc.HighsModel()
    model.lp_ = lp
    qd = np.asarray(q, dtype=np.float64)
    nzq = np.nonzero(qd)[0]
    if len(nzq):
        hs = hc.HighsHessian()
        hs.dim_ = n
        hs.format_ = hc.HessianFormat.kTriangular
        start = np.zeros(n + 1, dtype=np.int32)
        for j in nzq:
            start[j + 1:] += 1
        hs.start_ = start
        hs.index_ = nzq.astype(np.int32)
        hs.value_ = qd[nzq]
        model.hessian_ = hs
    h = hc._Highs()
    h.setOptionValue("output_flag", False)
    h.passModel(model)
    h.run()
    st = h.getModelStatus()
    if st != hc.HighsModelStatus.kOptimal:
        return None, None, 1
    x = np.array(h.getSolution().col_value)
    return x, float(h.getInfo().objective_function_value), 0


# ------------------------------------------------------------------ dense IPM
def solve_qp_ipm(A, rl, ru, lb, ub, c, q, tol=1e-11, max_iter=200, polish=True):
    """min c'x + 1/2 sum q x^2 s.t. rl <= Ax <= ru, lb <= x <= ub (q >= 0).

    Returns (x, obj, status) with status 0 = optimal.
    """
    A = np.asarray(A, float)
    m, n = A.shape
    eq = np.isfinite(rl) & np.isfinite(ru) & (np.abs(ru - rl) <= 0.0)
    ineq = ~eq
    AE, bE = A[eq], rl[eq]
    AI = A[ineq]
    mI = AI.shape[0]
    # w = [x; s], s = A_I x.
    N = n + mI
    M = np.zeros((AE.shape[0] + mI, N))
    M[:AE.shape[0], :n] = AE
    M[AE.shape[0]:, :n] = AI
    M[AE.shape[0]:, n:] = -np.eye(mI)
    r = np.concatenate([bE, np.zeros(mI)])
    lw = np.concatenate([lb, rl[ineq]])
    uw = np.concatenate([ub, ru[ineq]])
    g = np.concatenate([c, np.zeros(mI)])
    h = np.concatenate([q, np.zeros(mI)])
    fl = np.isfinite(lw)
    fu = np.isfinite(uw)
    # starting point strictly inside the box
    w = np.zeros(N)
    both = fl & fu
    w[both] = 0.5 * (lw[both] + uw[both])
    lo = fl & ~fu
    w[lo] = lw[lo] + np.maximum(1.0, 0.1 * np.abs(lw[lo]))
    up = fu & ~fl
    w[up] = uw[up] - np.maximum(1.0, 0.1 * np.abs(uw[up]))
    # duals chosen so the initial dual residual is O(1) (costs reach 1e5 in farmer)
    scale = 1.0 + np.abs(g)
    zl = np.where(fl, np.where(fu, scale, 1.0 + np.maximum(g, 0.0)), 0.0)
    zu = np.where(fu, np.where(fl, scale - g, 1.0 + np.maximum(-g, 0.0)), 0.0)
    lam = np.zeros(M.shape[0])
    ncomp = max(1, int(fl.sum() + fu.sum()))
    gnorm = 1.0 + np.abs(g).max(initial=0.0)
    rnorm = 1.0 + np.abs(r).max(initial=0.0)
    status = 1
    mu_hist = []
    for it in range(max_iter):
        dl = np.where(fl, w - lw, 1.0)
        du = np.where(fu, uw - w, 1.0)
        rd = h * w + g - M.T @ lam - zl + zu
        rp = M @ w - r
        mu = (np.sum((dl * zl)[fl]) + np.sum((du * zu)[fu])) / ncomp
        obj = g @ w + 0.5 * np.sum(h * w * w)
        if (np.abs(rd).max(initial=0) <= tol * gnorm and np.abs(rp).max(initial=0) <= tol * rnorm
                and mu * ncomp <= tol * (1.0 + abs(obj))):
            status = 0
            break
        Dl = np.where(fl, zl / dl, 0.0)
        Du = np.where(fu, zu / du, 0.0)
        K = np.diag(h + Dl + Du + 1e-14)
        KKT = np.block([[K, -M.T], [M, -1e-14 * np.eye(M.shape[0])]])

        def newton(tl, tu):
            rhs1 = -rd + np.where(fl, (tl - dl * zl) / dl, 0.0) - np.where(fu, (tu - du * zu) / du, 0.0)
            sol = np.linalg.lstsq(KKT, np.concatenate([rhs1, -rp]), rcond=None)[0] \
                if not np.all(np.isfinite(rhs1)) else np.linalg.solve(KKT, np.concatenate([rhs1, -rp]))
            dw = sol[:N]
            dlam = sol[N:]
            dzl = np.where(fl, (tl - dl * zl - zl * dw) / dl, 0.0)
            dzu = np.where(fu, (tu - du * zu + zu * dw) / du, 0.0)
            return dw, dlam, dzl, dzu

        def max_step(dw, dzl, dzu):
            ap = 1.0
            ad = 1.0
            neg = fl & (dw < 0)
            if neg.any():
                ap = min(ap, np.min(-dl[neg] / dw[neg]))
            pos = fu & (dw > 0)
            if pos.any():
                ap = min(ap, np.min(du[pos] / dw[pos]))
            nz = fl & (dzl < 0)
            if nz.any():
                ad = min(ad, np.min(-zl[nz] / dzl[nz]))
            nz = fu & (dzu < 0)
            if nz.any():
                ad = min(ad, np.min(-zu[nz] / dzu[nz]))
            return ap, ad

        zeros = np.zeros(N)
        dw, dlam, dzl, dzu = newton(zeros, zeros)
        ap, ad = max_step(dw, dzl, dzu)
        mu_aff = (np.sum(((dl + ap * dw) * (zl + ad * dzl))[fl]) +
                  np.sum(((du - ap * dw) * (zu + ad * dzu))[fu])) / ncomp
        sigma = (mu_aff / max(mu, 1e-300)) ** 3
        # safeguard: Mehrotra's corrector can cycle without reducing mu (seen on a few
        # PH-augmented aircond QPs: a period-4 orbit at mu ~ 0.13); after 5 iterations
        # without halving mu, take a well-centred step instead
        mu_hist.append(mu)
        if len(mu_hist) > 5 and mu > 0.5 * mu_hist[-6]:
            sigma = max(sigma, 0.5)
        tl = np.where(fl, sigma * mu - dw * dzl, 0.0)
        tu = np.where(fu, sigma * mu + dw * dzu, 0.0)
        dw, dlam, dzl, dzu = newton(tl, tu)
        ap, ad = max_step(dw, dzl, dzu)
        ap = min(1.0, 0.995 * ap)
        ad = min(1.0, 0.995 * ad)
        w = w + ap * dw
        lam = lam + ad * dlam
        zl = zl + ad * dzl
        zu = zu + ad * dzu
    x = w[:n]
    if polish:
        xp = _polish(A, rl, ru, lb, ub, c, q, w, zl, zu, lw, uw, fl, fu, M, r, h, g, n)
        if xp is not None:
            x = xp
    obj = float(c @ x + 0.5 * np.sum(q * x * x))
    return x, obj, status


def _polish(A, rl, ru, lb, ub, c, q, w, zl, zu, lw, uw, fl, fu, M, r, h, g, n):
    """One equality-constrained KKT solve on the IPM's active set (accept if feasible
    and not worse)."""
    N = w.size
    dl = np.where(fl, w - lw, INF)
    du = np.where(fu, uw - w, INF)
    act_l = fl & (zl > dl)
    act_u = fu & (zu > du) & ~act_l
    fixed = act_l | act_u
    val = np.where(act_l, lw, np.where(act_u, uw, 0.0))
    free = ~fixed
    nf = int(free.sum())
    Mf = M[:, free]
    rr = r - M[:, fixed] @ val[fixed]
    KKT = np.block([[np.diag(h[free]), -Mf.T], [Mf, np.zeros((M.shape[0], M.shape[0]))]])
    rhs = np.concatenate([-g[free], rr])
    sol = np.linalg.lstsq(KKT, rhs, rcond=None)[0]
    wp = val.copy()
    wp[free] = sol[:nf]
    tol = 1e-9 * (1.0 + np.abs(w).max())
    if np.any(wp[fl] < lw[fl] - tol) or np.any(wp[fu] > uw[fu] + tol):
        return None
    if np.abs(M @ wp - r).max(initial=0) > tol:
        return None
    obj_p = g @ wp + 0.5 * np.sum(h * wp * wp)
    obj_w = g @ w + 0.5 * np.sum(h * w * w)
    if obj_p > obj_w + 1e-9 * (1.0 + abs(obj_w)):
        return None
    x = np.clip(wp[:n], lb, ub)
    return x


# ------------------------------------------------------- farmer closed form
def kkt_certify(A, rl, ru, lb, ub, c, q, x, act_tol=1e-7):
    """Certify that x solves  min c'x + 1/2 sum q x^2  s.t. rl <= Ax <= ru, lb <= x <= ub
    (q >= 0, a convex QP) by its KKT conditions: x feasible, and multipliers with the
    right signs on the active bounds / rows (y_i >= 0 on a row at rl, <= 0 at ru, free on
    an equality; reduced costs >= 0 at lb, <= 0 at ub) that make q x + c - A'y - r = 0.
    The multipliers come from a bounded least-squares fit (scipy lsq_linear); returns
    (primal violation, stationarity residual), both relative to 1 + max|c|.  For the
    oracle's IPM runs that stop short of its own tolerance: their polished x is accepted
    when both are tiny (make_golden_aircond.py)."""
    from scipy.optimize import lsq_linear
    A = np.asarray(A, float)
    m, n = A.shape
    scale = 1.0 + np.abs(c).max(initial=0.0)
    ax = A @ x
    pviol = max(np.maximum(rl - ax, 0).max(initial=0), np.maximum(ax - ru, 0).max(initial=0),
                np.maximum(lb - x, 0).max(initial=0), np.maximum(x - ub, 0).max(initial=0))
    tol_r = act_tol * (1.0 + np.abs(ax))
    tol_x = act_tol * (1.0 + np.abs(x))
    at_rl = np.isfinite(rl) & (ax - rl <= tol_r)
    at_ru = np.isfinite(ru) & (ru - ax <= tol_r)
    at_lb = np.isfinite(lb) & (x - lb <= tol_x)
    at_ub = np.isfinite(ub) & (ub - x <= tol_x)
    cols, lo, hi = [], [], []
    for i in range(m):                       # y_i: row multipliers
        if at_rl[i] or at_ru[i]:
            cols.append(A[i])
            lo.append(0.0 if not at_ru[i] else -INF)
            hi.append(0.0 if not at_rl[i] else INF)
    for j in range(n):                       # reduced costs of active column bounds
        if at_lb[j] or at_ub[j]:
            e = np.zeros(n)
            e[j] = 1.0
            cols.append(e)
            lo.append(0.0 if not at_ub[j] else -INF)
            hi.append(0.0 if not at_lb[j] else INF)
    grad = q * x + c
    if not cols:
        return pviol / scale, np.abs(grad).max() / scale
    M = np.array(cols).T
    sol = lsq_linear(M, grad, bounds=(np.array(lo), np.array(hi)), method="bvls", tol=1e-14)
    return pviol / scale, np.abs(M @ sol.x - grad).max() / scale


def _farmer_crop_pieces(base, Y, cm):
    """Convex piecewise-linear first+second stage cost of one crop as a function of its
    acreage x in [0, 500*cm]: returns (breakpoints, slopes, value at 0).

    Restates the recourse of farmer.py:181-222 for one crop: wheat/corn buy the feed
    shortfall at PurchasePrice, sell the surplus at SubQuotaSellingPrice up to the 1e5
    quota and the rest at SuperQuotaSellingPrice (0; the quota kink lies inside
    [0, 500 cm] only for cm >= ~28); beets sell up to the 6000 quota at 36 and the rest
    at 10.
    """
    total = 500.0 * cm
    plant = {"WHEAT": 150.0, "CORN": 230.0, "SUGAR_BEETS": 260.0}[base]
    if base in ("WHEAT", "CORN"):
        req = {"WHEAT": 200.0, "CORN": 240.0}[base]
        buy = {"WHEAT": 238.0, "CORN": 210.0}[base]
        sub = {"WHEAT": 170.0, "CORN": 150.0}[base]
        kink = req / Y
        kq = (req + 100000.0) / Y
        f0 = buy * req
        return ([0.0, min(kink, total), min(kq, total), total],
                [plant - buy * Y, plant - sub * Y, plant], f0)
    kink = 6000.0 / Y
    return [0.0, min(kink, total), total], [plant - 36.0 * Y, plant - 10.0 * Y], 0.0


def _crop_argmin(bp, slopes, f0, lin, rho, xbar):
    """argmin over [bp0, bp_end] of g(x) + lin*x + rho/2 (x - xbar)^2, g convex PL."""
    best_x, best_v = None, INF
    val_at = f0
    for k in range(len(slopes)):
        lo, hi = bp[k], bp[k + 1]
        if hi < lo:
            continue
        s = slopes[k] + lin
        xc = min(max(xbar - s / rho, lo), hi)
        v = val_at + slopes[k] * (xc - lo) + lin * xc + 0.5 * rho * (xc - xbar) ** 2
        if v < best_v:
            best_x, best_v = xc, v
        val_at += slopes[k] * (hi - lo)
    return best_x


def _crop_cost(bp, slopes, f0, x):
    v = f0
    for k in range(len(slopes)):
        lo, hi = bp[k], bp[k + 1]
        seg = min(max(x, lo), hi) - lo
        v += slopes[k] * max(seg, 0.0)
    return v


def farmer_prox_exact(crops_sorted, Y, W, xbar, rho, cm):
    """Exact farmer prox QP in the nonant variables (sorted crop order).

    min sum_k g_k(x_k) + W_k x_k + rho_k/2 (x_k - xbar_k)^2  s.t. sum x_k <= 500 cm.
    Returns (x_nonant, augmented objective).
    """
    pieces = [_farmer_crop_pieces(cn.rstrip("0123456789"), Y[cn], cm) for cn in crops_sorted]
    total = 500.0 * cm

    def xs(lam):
        return np.array([_crop_argmin(bp, sl, f0, W[k] + lam, rho[k], xbar[k])
                         for k, (bp, sl, f0) in enumerate(pieces)])

    x = xs(0.0)
    if x.sum() > total:
        lo, hi = 0.0, 1.0
        while xs(hi).sum() > total:
            hi *= 2.0
        for _ in range(200):
            mid = 0.5 * (lo + hi)
            if xs(mid).sum() > total:
                lo = mid
            else:
                hi = mid
            if hi - lo <= 1e-15 * max(1.0, hi):
                break
        x = xs(hi)  # x(lam) is 1/rho-Lipschitz: error <= (hi-lo)/rho
    obj = sum(_crop_cost(bp, sl, f0, x[k]) for k, (bp, sl, f0) in enumerate(pieces))
    obj += float(np.dot(W, x) + 0.5 * np.sum(rho * (x - xbar) ** 2))
    return x, obj
