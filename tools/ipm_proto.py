"""Design prototype (numpy, vectorised over scenarios) of the batched Mehrotra
predictor-corrector IPM that path 6 runs per lane.  Not product code and
not the oracle: it exists to count IPM iterations and check the formulation before the
kernel is written.  Usage: python tools/ipm_proto.py [S] [cm]

Problem:  min c'x + 1/2 sum q_j x_j^2  s.t.  rl <= A x <= ru,  lb <= x <= ub.
Row activities w = A x are variables for rows with rl < ru (equality rows pin w = rl);
x and w are kept strictly inside their boxes, so only A x - w = 0 carries an
infeasibility residual.
"""
import sys
import time

import numpy as np

sys.path.insert(0, "mpi-sppy-1_amd")


def ruiz(A, iters=10):
    S, m, n = A.shape
    Dr = np.ones((S, m))
    Dc = np.ones((S, n))
    As = A.copy()
    for _ in range(iters):
        r = np.sqrt(np.abs(As).max(2))
        r[r == 0] = 1
        c = np.sqrt(np.abs(As).max(1))
        c[c == 0] = 1
        As = As / r[:, :, None] / c[:, None, :]
        Dr /= r
        Dc /= c
    return As, Dr, Dc


def ldl_factor(M, piv_rel=1e-30):
    """In-place batched LDL^T without pivoting (the kernel's order); a pivot below
    piv_rel x the row's original diagonal is replaced by 1e128 (that row's step -> 0)."""
    S, m, _ = M.shape
    L = M.copy()
    d = np.zeros((S, m))
    dg = np.einsum("smm->sm", M).copy()
    for k in range(m):
        dk = L[:, k, k] - (L[:, k, :k] ** 2 * d[:, :k]).sum(1)
        dk = np.where(dk > piv_rel * np.maximum(dg[:, k], 1e-300), dk, 1e128)
        d[:, k] = dk
        for i in range(k + 1, m):
            L[:, i, k] = (L[:, i, k] - (L[:, i, :k] * L[:, k, :k] * d[:, :k]).sum(1)) / dk
    return L, d


def ldl_solve(L, d, r):
    S, m = r.shape
    z = r.copy()
    for k in range(m):
        z[:, k] -= (L[:, k, :k] * z[:, :k]).sum(1)
    z /= d
    for k in range(m - 1, -1, -1):
        z[:, k] -= (L[:, k + 1:, k] * z[:, k + 1:]).sum(1)
    return z


def ipm(A, c, q, lb, ub, rl, ru, eps=1e-9, max_it=100, x0=None, verbose=False, common_step=True, regp=1e-12, regd=1e-12, single=None):
    """Vectorised over the leading scenario axis.  Returns x, y, obj, iters, converged."""
    S, m, n = A.shape
    gam = np.maximum(1.0, np.abs(c).max(1))[:, None]
    c = c / gam
    q = q / gam
    hl, hu = np.isfinite(lb), np.isfinite(ub)
    eq = rl == ru
    hlw, huw = np.isfinite(rl) & ~eq, np.isfinite(ru) & ~eq
    L = np.where(hl, lb, 0.0)
    U = np.where(hu, ub, 0.0)
    RL = np.where(np.isfinite(rl), rl, 0.0)
    RU = np.where(np.isfinite(ru), ru, 0.0)

    def interior(v, lo, hi, hlo, hhi):
        both = hlo & hhi
        mid = 0.5 * (lo + hi)
        half = 0.5 * (hi - lo)
        out = v.copy()
        k = np.maximum(1.0, 0.1 * np.abs(v))
        out = np.where(hlo & ~hhi, np.maximum(v, lo + k), out)
        out = np.where(hhi & ~hlo, np.minimum(v, hi - k), out)
        out = np.where(both, np.clip(v, lo + 0.1 * half, hi - 0.1 * half), out)
        out = np.where(both & (half <= 0), mid, out)
        return out

    x = interior(np.zeros((S, n)) if x0 is None else x0, L, U, hl, hu)
    w = interior(np.einsum("smn,sn->sm", A, x), RL, RU, hlw, huw)
    w = np.where(eq, RL, w)
    r0 = c + q * x
    kap = 1.0
    zl = np.where(hl, np.where(hu, np.maximum(r0, 0), np.abs(r0)) + kap, 0.0)
    zu = np.where(hu, np.where(hl, np.maximum(-r0, 0), np.abs(r0)) + kap, 0.0)
    zlw = np.where(hlw, 1.0, 0.0)
    zuw = np.where(huw, 1.0, 0.0)
    y = np.zeros((S, m))
    ncomp = hl.sum(1) + hu.sum(1) + hlw.sum(1) + huw.sum(1)
    done = np.zeros(S, bool)
    iters = np.zeros(S, int)
    bnorm = np.sqrt(np.where(np.isfinite(rl), rl, 0) ** 2 + np.where(np.isfinite(ru) & ~eq, ru, 0) ** 2).sum(1)
    cnorm = np.sqrt((c * c).sum(1))
    for it in range(max_it):
        sl = np.where(hl, x - L, 1.0)
        su = np.where(hu, U - x, 1.0)
        slw = np.where(hlw, w - RL, 1.0)
        suw = np.where(huw, RU - w, 1.0)
        Ax = np.einsum("smn,sn->sm", A, x)
        Aty = np.einsum("smn,sm->sn", A, y)
        # convergence: relative KKT on (x, y) as the PDHG paths test it
        pres = Ax - np.clip(Ax, np.where(np.isfinite(rl), rl, -np.inf), np.where(np.isfinite(ru), ru, np.inf))
        rc = c + q * x - Aty
        lam = np.where(hl & hu, rc, np.where(hl, np.maximum(rc, 0), np.where(hu, np.minimum(rc, 0), 0)))
        dres = rc - lam
        pobj = (c * x + 0.5 * q * x * x).sum(1)
        rr = c - Aty
        with np.errstate(divide="ignore", invalid="ignore"):
            xm = np.clip(np.where(q > 0, -rr / np.where(q > 0, q, 1), 0), np.where(hl, lb, -np.inf), np.where(hu, ub, np.inf))
        cd = np.where(q > 0, rr * xm + 0.5 * q * xm * xm,
                      np.where(rr > 0, np.where(hl, rr * L, 0.0), np.where(rr < 0, np.where(hu, rr * U, 0.0), 0)))
        rd = np.where(y > 0, np.where(np.isfinite(rl), RL * y, 0.0), np.where(y < 0, np.where(np.isfinite(ru), RU * y, 0.0), 0))
        dobj = cd.sum(1) + rd.sum(1)
        tp = eps * (1 + bnorm)
        td = eps * (1 + cnorm)
        conv = ((pres ** 2).sum(1) <= tp ** 2) & ((dres ** 2).sum(1) <= td ** 2) & \
               (np.abs(pobj - dobj) <= eps * (1 + np.abs(pobj) + np.abs(dobj)))
        newly = conv & ~done
        iters[newly] = it
        done |= conv
        if verbose:
            print(it, 'pres', np.sqrt((pres**2).sum(1)).max(), 'dres', np.sqrt((dres**2).sum(1)).max(), 'gap', np.abs(pobj-dobj).max(), 'pobj', pobj[0], dobj[0])
        if done.all():
            break
        mu = ((sl * zl)[hl.nonzero()].sum() if False else (np.where(hl, sl * zl, 0).sum(1) + np.where(hu, su * zu, 0).sum(1)
              + np.where(hlw, slw * zlw, 0).sum(1) + np.where(huw, suw * zuw, 0).sum(1))) / np.maximum(ncomp, 1)
        rd_ = c + q * x - Aty - zl + zu
        rw = np.where(eq, 0.0, y - zlw + zuw)
        rp = np.where(eq, Ax - RL, Ax - w)
        Sx = np.where(hl, zl / sl, 0) + np.where(hu, zu / su, 0)
        Sw = np.where(hlw, zlw / slw, 0) + np.where(huw, zuw / suw, 0)
        Dx = 1.0 / (q + Sx + regp)
        Einv = np.where(eq, regd, 1.0 / np.where(eq, 1.0, Sw) + regd)
        M = np.einsum("smn,sn,skn->smk", A, Dx, A) + Einv[:, :, None] * np.eye(m)[None]
        bad = ~np.isfinite(M).all((1, 2))
        M = np.where((done | bad)[:, None, None], np.eye(m)[None], M)
        LF, DF = ldl_factor(M)

        def solve(tl, tu, tlw, tuw):
            hx = -rd_ + np.where(hl, tl / sl - zl, 0) - np.where(hu, tu / su - zu, 0)
            hw = -rw + np.where(hlw, tlw / slw - zlw, 0) - np.where(huw, tuw / suw - zuw, 0)
            rhs = -rp - np.einsum("smn,sn->sm", A, Dx * hx) + np.where(eq, 0.0, hw / np.where(eq, 1.0, Sw))
            dy = ldl_solve(LF, DF, rhs)
            dx = Dx * (hx + np.einsum("smn,sm->sn", A, dy))
            dw = np.where(eq, 0.0, np.einsum("smn,sn->sm", A, dx) + rp)   # the primal row equation exactly
            dzl = np.where(hl, (tl - sl * zl - zl * dx) / sl, 0)
            dzu = np.where(hu, (tu - su * zu + zu * dx) / su, 0)
            dzlw = np.where(hlw, (tlw - slw * zlw - zlw * dw) / slw, 0)
            dzuw = np.where(huw, (tuw - suw * zuw + zuw * dw) / suw, 0)
            return dx, dw, dy, dzl, dzu, dzlw, dzuw

        def maxstep(v, dv, has):
            with np.errstate(divide="ignore", invalid="ignore"):
                r = np.where(has & (dv < 0), -v / dv, np.inf)
            return np.minimum(1.0, r.min(1))

        z = np.zeros_like
        if single is not None:
            if it == 0:
                aprev = np.zeros(S)
            sig = single(aprev, mu)
            sm = (sig * mu)[:, None]
            dx, dw, dy, dzl, dzu, dzlw, dzuw = solve(sm + z(sl), sm + z(su), sm + z(slw), sm + z(suw))
        else:
          dx, dw, dy, dzl, dzu, dzlw, dzuw = solve(z(sl), z(su), z(slw), z(suw))
          ap = np.minimum.reduce([maxstep(sl, dx, hl), maxstep(su, -dx, hu), maxstep(slw, dw, hlw), maxstep(suw, -dw, huw)])
          ad = np.minimum.reduce([maxstep(zl, dzl, hl), maxstep(zu, dzu, hu), maxstep(zlw, dzlw, hlw), maxstep(zuw, dzuw, huw)])
          if common_step:
            ap = ad = np.minimum(ap, ad)
          mua = (np.where(hl, (sl + ap[:, None] * dx) * (zl + ad[:, None] * dzl), 0).sum(1)
               + np.where(hu, (su - ap[:, None] * dx) * (zu + ad[:, None] * dzu), 0).sum(1)
               + np.where(hlw, (slw + ap[:, None] * dw) * (zlw + ad[:, None] * dzlw), 0).sum(1)
               + np.where(huw, (suw - ap[:, None] * dw) * (zuw + ad[:, None] * dzuw), 0).sum(1)) / np.maximum(ncomp, 1)
          sig = np.where(mu > 0, (mua / np.where(mu > 0, mu, 1)) ** 3, 0.0)
          sm = (sig * mu)[:, None]
          tl = sm - dx * dzl
          tu = sm + dx * dzu
          tlw = sm - dw * dzlw
          tuw = sm + dw * dzuw
          dx, dw, dy, dzl, dzu, dzlw, dzuw = solve(tl, tu, tlw, tuw)
        ap = np.minimum.reduce([maxstep(sl, dx, hl), maxstep(su, -dx, hu), maxstep(slw, dw, hlw), maxstep(suw, -dw, huw)])
        ad = np.minimum.reduce([maxstep(zl, dzl, hl), maxstep(zu, dzu, hu), maxstep(zlw, dzlw, hlw), maxstep(zuw, dzuw, huw)])
        if common_step:
            ap = ad = np.minimum(ap, ad)
        if verbose:
            print('   mu', mu[0], 'sig', sig[0], 'ap', ap[0], 'ad', ad[0])
        aprev = np.minimum(ap, ad)
        ap = np.minimum(1.0, 0.995 * ap)[:, None]
        ad = np.minimum(1.0, 0.995 * ad)[:, None]
        act = ~done[:, None]
        x = np.where(act, x + ap * dx, x)
        w = np.where(act, w + ap * dw, w)
        y = np.where(act, y + ad * dy, y)
        zl = np.where(act, zl + ad * dzl, zl)
        zu = np.where(act, zu + ad * dzu, zu)
        zlw = np.where(act, zlw + ad * dzlw, zlw)
        zuw = np.where(act, zuw + ad * dzuw, zuw)
    iters[~done] = max_it
    return x, y * gam, pobj * gam[:, 0], iters, done


def main():
    from mpisppy_amd.examples import farmer
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    cm = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    names = farmer.scenario_names_creator(S)
    b = farmer.batch_creator(names, crops_multiplier=cm)
    Ad = np.stack([b.dense_A(s) for s in range(S)])
    As, Dr, Dc = ruiz(Ad)
    c = b.c * Dc
    q = b.q * Dc * Dc
    lb, ub = b.lb / Dc, b.ub / Dc
    rl, ru = b.rl * Dr, b.ru * Dr
    print(f"S={S} cm={cm} n={b.n} m={b.m} nnz={b.nnz}")
    for cs in (True, False):
        t = time.time()
        x, y, obj, it, ok = ipm(As, c, q, lb, ub, rl, ru, common_step=cs)
        print(f"Iter0 LP common_step={cs}: iters max {it.max()} mean {it.mean():.1f}  conv {ok.mean():.3f}  "
              f"E[obj] {np.mean(obj):.6f}  ({time.time() - t:.1f}s)")
    # a PH-like prox QP: W = 0.5 * (x - mean), rho = 1 on the nonants
    xo = x * Dc
    nc = b.nonant_col
    xb = xo[:, nc].mean(0)
    W = 1.0 * (xo[:, nc] - xb)
    c2 = b.c.copy()
    q2 = b.q.copy()
    c2[:, nc] += W - 1.0 * xb
    q2[:, nc] += 1.0
    for cs in (True, False):
        x2, y2, obj2, it2, ok2 = ipm(As, c2 * Dc, q2 * Dc * Dc, lb, ub, rl, ru, common_step=cs)
        print(f"prox QP common_step={cs}: iters max {it2.max()} mean {it2.mean():.1f} conv {ok2.mean():.3f}")
    x3, y3, obj3, it3, ok3 = ipm(As, c2 * Dc, q2 * Dc * Dc, lb, ub, rl, ru, x0=x)
    print(f"prox QP warm x0: iters max {it3.max()} mean {it3.mean():.1f} conv {ok3.mean():.3f}")
    try:
        from scipy.optimize import linprog
        bad = 0
        for s in range(min(S, 64)):
            A = Ad[s]
            fin_u = np.isfinite(b.ru[s])
            fin_l = np.isfinite(b.rl[s])
            r = linprog(b.c[s], A_ub=np.vstack([A[fin_u], -A[fin_l]]), b_ub=np.concatenate([b.ru[s][fin_u], -b.rl[s][fin_l]]),
                        bounds=list(zip(b.lb[s], b.ub[s])), method="highs")
            ob = (b.c[s] * xo[s]).sum()
            if abs(ob - r.fun) > 1e-7 * (1 + abs(r.fun)):
                bad += 1
                print("mismatch", s, ob, r.fun)
        print("HiGHS check on", min(S, 64), "scenarios: mismatches", bad)
    except ImportError:
        pass


if __name__ == "__main__":
    main()
