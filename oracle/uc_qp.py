"""Sparse interior-point QP oracle for the UC PH subproblems (TEST INFRASTRUCTURE ONLY --
tests/ and the fixture generators may use it; the product path never does).

Config 5's PH subproblem (spopt.py:85-223 with the PH terms of phbase.py:617-699) is the UC
LP relaxation (mpisppy_amd/examples/uc.py) plus W and a proximal term on the 4,080 UnitOn
nonants:

    min c'x + W'x_N + rho/2 ||x_N - xbar||^2   s.t.  rl <= A x <= ru,  lb <= x <= ub.

The reference hands it to an external QP solver through Pyomo; scipy's HiGHS QP (the only QP
solver in the image) stops with a solve error on it, so this is a restatement of the standard
primal-dual interior point with Mehrotra's predictor-corrector (Nocedal & Wright ch. 16.6,
Wright "Primal-Dual Interior-Point Methods" ch. 10) on the sparse normal equations, factored by
SuperLU in symmetric mode (minimum degree on A D A'): ~1 s per factorisation for UC.  It is an
independent algorithm from the engine's path 4 (a first-order PDHG), run to a relative KKT
error of 1e-10 so its nonants -- unique, the objective being strongly convex in them -- serve
as the fixture the GPU's PH trajectory is compared with (tests/golden/make_golden_uc_ph.py).

Parity note: UC has no fixture in the reference (egret is absent), so these fixtures pin the
GPU against this restatement of our own LP (examples/uc.py), not against the reference.
"""
import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

INF = np.inf


def solve_qp(A, rl, ru, lb, ub, c, q, tol=1e-10, max_iter=200, verbose=False):
    """min c'x + 1/2 sum q_j x_j^2  s.t.  rl <= A x <= ru, lb <= x <= ub   (q >= 0, A sparse).

    Returns dict(x, y, obj, status, iters, kkt) -- status 0 = converged to ``tol`` (relative
    primal residual, dual residual and complementarity), 1 = iteration limit."""
    A = sp.csr_matrix(A, dtype=np.float64)
    m, n = A.shape
    c = np.asarray(c, float)
    q = np.asarray(q, float)
    lb, ub, rl, ru = (np.asarray(v, float) for v in (lb, ub, rl, ru))
    # objective scaling (UC costs reach 1e6)
    cs = max(1.0, np.abs(c).max(initial=0.0), np.abs(q).max(initial=0.0))
    c, q = c / cs, q / cs
    # fixed columns out
    fixc = np.isfinite(lb) & np.isfinite(ub) & (ub <= lb)
    xfix = np.where(fixc, lb, 0.0)
    keep = ~fixc
    Af = A[:, keep].tocsr()
    shift = A[:, fixc] @ xfix[fixc] if fixc.any() else np.zeros(m)
    rl_s, ru_s = rl - shift, ru - shift
    # rows: equality (w fixed), bounded (slack w), free (dropped)
    eq = np.isfinite(rl_s) & np.isfinite(ru_s) & (ru_s <= rl_s)
    free = ~np.isfinite(rl_s) & ~np.isfinite(ru_s)
    rows = ~free
    Ar = Af[rows].tocsr()
    rl_r, ru_r, eq_r = rl_s[rows], ru_s[rows], eq[rows]
    mr = Ar.shape[0]
    cf, qf, lbf, ubf = c[keep], q[keep], lb[keep], ub[keep]
    nf = cf.size
    # Ruiz equilibration (10 passes): A_s = R A C, x = C x_s, rows scaled by R
    R, C = np.ones(mr), np.ones(nf)
    As = Ar.copy()
    for _ in range(10):
        rmax = abs(As).max(axis=1).toarray().ravel()
        cmax = abs(As).max(axis=0).toarray().ravel()
        rmax = np.sqrt(np.where(rmax > 0, rmax, 1.0))        # empty rows / columns keep scale 1
        cmax = np.sqrt(np.where(cmax > 0, cmax, 1.0))
        As = (sp.diags(1.0 / rmax) @ As @ sp.diags(1.0 / cmax)).tocsr()
        R, C = R / rmax, C / cmax
    Ar = As
    rl_r, ru_r = rl_r * R, ru_r * R
    cf, qf = cf * C, qf * C * C
    lbf, ubf = lbf / C, ubf / C
    hl, hu = np.isfinite(lbf), np.isfinite(ubf)
    hlw, huw = np.isfinite(rl_r) & ~eq_r, np.isfinite(ru_r) & ~eq_r
    # starting point: x inside its box, w = clamp(A x)
    x = np.zeros(nf)
    both = hl & hu
    x[both] = 0.5 * (lbf[both] + ubf[both])
    x[hl & ~hu] = lbf[hl & ~hu] + 1.0
    x[hu & ~hl] = ubf[hu & ~hl] - 1.0
    ax = Ar @ x
    w = ax.copy()
    wb = hlw & huw
    w[wb] = np.clip(ax[wb], rl_r[wb] + 0.1 * (ru_r[wb] - rl_r[wb]), ru_r[wb] - 0.1 * (ru_r[wb] - rl_r[wb]))
    w[hlw & ~huw] = np.maximum(ax[hlw & ~huw], rl_r[hlw & ~huw] + 1.0)
    w[huw & ~hlw] = np.minimum(ax[huw & ~hlw], ru_r[huw & ~hlw] - 1.0)
    w[eq_r] = rl_r[eq_r]
    y = np.zeros(mr)
    zl, zu = np.where(hl, 1.0, 0.0), np.where(hu, 1.0, 0.0)
    zlw, zuw = np.where(hlw, 1.0, 0.0), np.where(huw, 1.0, 0.0)
    ncomp = max(1, int(hl.sum() + hu.sum() + hlw.sum() + huw.sum()))
    bnorm = 1.0 + max(np.abs(np.where(np.isfinite(rl_r), rl_r, 0)).max(initial=0),
                      np.abs(np.where(np.isfinite(ru_r), ru_r, 0)).max(initial=0))
    cnorm = 1.0 + np.abs(cf).max(initial=0)
    reg_p, reg_d = 1e-9, 1e-10
    status, it = 1, 0
    kkt = (INF, INF, INF)
    AT = Ar.T.tocsr()
    for it in range(max_iter):
        sl = np.where(hl, x - lbf, 1.0)
        su = np.where(hu, ubf - x, 1.0)
        slw = np.where(hlw, w - rl_r, 1.0)
        suw = np.where(huw, ru_r - w, 1.0)
        # residuals: r_d (x stationarity), r_w (w stationarity), r_p (A x - w)
        r_d = cf + qf * x - AT @ y - zl + zu
        r_w = np.where(eq_r, 0.0, y - zlw + zuw)
        r_p = Ar @ x - w
        mu = (np.sum((sl * zl)[hl]) + np.sum((su * zu)[hu]) + np.sum((slw * zlw)[hlw]) +
              np.sum((suw * zuw)[huw])) / ncomp
        pobj = cf @ x + 0.5 * np.sum(qf * x * x)
        kkt = (np.abs(r_p).max(initial=0) / bnorm, max(np.abs(r_d).max(initial=0), np.abs(r_w).max(initial=0)) / cnorm,
               mu * ncomp / (1.0 + abs(pobj)))
        if verbose:
            print(f"it {it:3d} pobj {pobj * cs:.10e} pres {kkt[0]:.2e} dres {kkt[1]:.2e} comp {kkt[2]:.2e}", flush=True)
        if max(kkt) <= tol:
            status = 0
            break
        Sx = np.where(hl, zl / sl, 0.0) + np.where(hu, zu / su, 0.0)
        Sw = np.where(hlw, zlw / slw, 0.0) + np.where(huw, zuw / suw, 0.0)
        Dx = 1.0 / (qf + Sx + reg_p)
        # w rows: equality rows carry dual regularisation only; bounded rows 1 / Sw
        Ew = np.where(eq_r, 0.0, 1.0 / np.maximum(Sw, 1e-300))
        N = (Ar @ sp.diags(Dx) @ AT).tocsc() + sp.diags(Ew, format="csc")
        # the factor carries a dual regularisation relative to each row's scale (equality rows
        # may be linearly dependent: the Schur complement would cancel to an exact zero pivot);
        # iterative refinement then solves the unregularised system
        lu = None
        for rd, thr in ((reg_d, 0.0), (1e3 * reg_d, 0.0), (1e3 * reg_d, 0.1), (1e6 * reg_d, 1.0)):
            Nr = N + sp.diags(rd * (1.0 + N.diagonal()), format="csc")
            try:
                lu = spla.splu(Nr, permc_spec="MMD_AT_PLUS_A", diag_pivot_thresh=thr,
                               options=dict(SymmetricMode=True))
                break
            except RuntimeError:                    # an exact zero pivot: more regularisation
                continue
        if lu is None:
            break                                    # numerical end: keep the last iterate

        def solve_N(b):
            v = lu.solve(b)
            for _ in range(3):                       # iterative refinement against N
                v = v + lu.solve(b - N @ v)
            return v

        def direction(tl, tu, tlw, tuw):
            # complementarity targets t: zl sl = tl etc.; eliminate dz, dw, dx
            gx = -r_d + np.where(hl, (tl - sl * zl) / sl, 0.0) - np.where(hu, (tu - su * zu) / su, 0.0)
            gw = -r_w + np.where(hlw, (tlw - slw * zlw) / slw, 0.0) - np.where(huw, (tuw - suw * zuw) / suw, 0.0)
            # (Q + Sx) dx - A' dy = gx ;  Sw dw + dy = gw ;  A dx - dw = -r_p
            rhs = -r_p - Ar @ (Dx * gx) + np.where(eq_r, 0.0, Ew * gw)
            dy = solve_N(rhs)
            dx = Dx * (gx + AT @ dy)
            dw = np.where(eq_r, 0.0, Ew * (gw - dy))
            dzl = np.where(hl, (tl - sl * zl - zl * dx) / sl, 0.0)
            dzu = np.where(hu, (tu - su * zu + zu * dx) / su, 0.0)
            dzlw = np.where(hlw, (tlw - slw * zlw - zlw * dw) / slw, 0.0)
            dzuw = np.where(huw, (tuw - suw * zuw + zuw * dw) / suw, 0.0)
            return dx, dw, dy, dzl, dzu, dzlw, dzuw

        def steps(dx, dw, dzl, dzu, dzlw, dzuw):
            def ratio(v, dv, mask):
                neg = mask & (dv < 0)
                return min(1.0, float(np.min(-v[neg] / dv[neg]))) if neg.any() else 1.0
            ap = min(ratio(sl, dx, hl), ratio(su, -dx, hu), ratio(slw, dw, hlw), ratio(suw, -dw, huw))
            ad = min(ratio(zl, dzl, hl), ratio(zu, dzu, hu), ratio(zlw, dzlw, hlw), ratio(zuw, dzuw, huw))
            return ap, ad

        zeros_n, zeros_m = np.zeros(nf), np.zeros(mr)
        d_aff = direction(zeros_n, zeros_n, zeros_m, zeros_m)
        ap, ad = steps(d_aff[0], d_aff[1], *d_aff[3:])
        dx, dw, _, dzl, dzu, dzlw, dzuw = d_aff
        mu_aff = (np.sum(((sl + ap * dx) * (zl + ad * dzl))[hl]) + np.sum(((su - ap * dx) * (zu + ad * dzu))[hu]) +
                  np.sum(((slw + ap * dw) * (zlw + ad * dzlw))[hlw]) +
                  np.sum(((suw - ap * dw) * (zuw + ad * dzuw))[huw])) / ncomp
        sigma = min(1.0, (mu_aff / max(mu, 1e-300)) ** 3)
        sm = sigma * mu
        tl = np.where(hl, sm - dx * dzl, 0.0)
        tu = np.where(hu, sm + dx * dzu, 0.0)
        tlw = np.where(hlw, sm - dw * dzlw, 0.0)
        tuw = np.where(huw, sm + dw * dzuw, 0.0)
        dx, dw, dy, dzl, dzu, dzlw, dzuw = direction(tl, tu, tlw, tuw)
        ap, ad = steps(dx, dw, dzl, dzu, dzlw, dzuw)
        if np.any(qf > 0):                           # a common step for QPs
            ap = ad = min(ap, ad)
        ap, ad = min(1.0, 0.995 * ap), min(1.0, 0.995 * ad)
        if not (np.isfinite(ap) and np.isfinite(ad) and np.all(np.isfinite(dx)) and np.all(np.isfinite(dy))):
            break                                    # numerical end: keep the last iterate
        x, w = x + ap * dx, w + ap * dw
        y = y + ad * dy
        zl, zu, zlw, zuw = zl + ad * dzl, zu + ad * dzu, zlw + ad * dzlw, zuw + ad * dzuw
    xo = xfix.copy()
    xo[keep] = x * C
    yo = np.zeros(m)
    yo[np.nonzero(rows)[0]] = y * R * cs
    obj = float((c * cs) @ xo + 0.5 * np.sum(q * cs * xo * xo))
    return {"x": xo, "y": yo, "obj": obj, "status": status, "iters": it, "kkt": kkt}
