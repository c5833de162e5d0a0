"""Development prototype of the batched PDHG (numpy) -- NOT product, NOT oracle.

Used only to tune the algorithm the HIP kernel implements (csrc/phgpu.hip): scaling,
restarted reflected-Halpern PDHG, termination and bound computation, batched over
scenarios with a shared CSR pattern.  Shapes: [S, k].
"""
import numpy as np


def spmv(rp, ci, Av, x):
    """y[s, r] = sum_k Av[s,k] x[s, ci[k]] over row r."""
    prod = Av * x[:, ci]
    cs = np.concatenate([np.zeros((x.shape[0], 1)), np.cumsum(prod, axis=1)], axis=1)
    return cs[:, rp[1:]] - cs[:, rp[:-1]]


def spmvT(rp, ci, Av, y, n):
    rows = np.repeat(np.arange(len(rp) - 1), np.diff(rp))
    prod = Av * y[:, rows]
    out = np.zeros((y.shape[0], n))
    for k in range(len(ci)):
        out[:, ci[k]] += prod[:, k]
    return out


class Proto:
    def __init__(self, b, ruiz_iters=10, pc_alpha=1.0):
        self.b = b
        S, n, m = b.S, b.n, b.m
        rp, ci = b.row_ptr, b.col_idx
        rows = np.repeat(np.arange(m), np.diff(rp))
        A = b.A_val.copy()
        Dr = np.ones((S, m))
        Dc = np.ones((S, n))
        for _ in range(ruiz_iters):
            ra = np.zeros((S, m))
            ca = np.zeros((S, n))
            aa = np.abs(A)
            for k in range(len(ci)):
                ra[:, rows[k]] = np.maximum(ra[:, rows[k]], aa[:, k])
                ca[:, ci[k]] = np.maximum(ca[:, ci[k]], aa[:, k])
            rs = np.where(ra > 0, 1 / np.sqrt(ra), 1.0)
            cs = np.where(ca > 0, 1 / np.sqrt(ca), 1.0)
            A = A * rs[:, rows] * cs[:, ci]
            Dr *= rs
            Dc *= cs
        if pc_alpha is not None:
            ra = np.zeros((S, m))
            ca = np.zeros((S, n))
            aa = np.abs(A)
            for k in range(len(ci)):
                ra[:, rows[k]] += aa[:, k] ** (2 - pc_alpha)
                ca[:, ci[k]] += aa[:, k] ** pc_alpha
            rs = np.where(ra > 0, 1 / np.sqrt(ra), 1.0)
            cs = np.where(ca > 0, 1 / np.sqrt(ca), 1.0)
            A = A * rs[:, rows] * cs[:, ci]
            Dr *= rs
            Dc *= cs
        self.Ah, self.Dr, self.Dc, self.rows = A, Dr, Dc, rows
        # power iteration for ||Ah||_2
        v = (1 + 0.5 * np.sin(1.7 * np.arange(n)))[None, :].repeat(S, 0)
        for _ in range(200):
            w = spmvT(rp, ci, A, spmv(rp, ci, A, v), n)
            nv = np.linalg.norm(w, axis=1, keepdims=True)
            v = w / np.maximum(nv, 1e-300)
        self.normA = 1.01 * np.sqrt(np.maximum(nv[:, 0], 1e-300))
        self.x = np.zeros((S, n))
        self.y = np.zeros((S, m))

    def solve(self, c, q, eps=1e-9, max_iter=100000, gamma=1.0, check=64, warm=True,
              eta_frac=0.998, verbose=False, omega0=None, restart_every=None, theta=0.5, art=None, kernel_mode=False, km_hk0=True, km_rlast_inf=True, trace=None, wclamp=None):
        b = self.b
        S, n, m = b.S, b.n, b.m
        rp, ci, A, Dr, Dc = b.row_ptr, b.col_idx, self.Ah, self.Dr, self.Dc
        ch = c * Dc
        qh = q * Dc * Dc
        lbh = b.lb / Dc
        ubh = b.ub / Dc
        rlh = b.rl * Dr
        ruh = b.ru * Dr
        eta = eta_frac / self.normA[:, None]
        bnorm = np.sqrt(np.sum(np.where(np.isfinite(rlh), rlh, 0) ** 2 + np.where(np.isfinite(ruh), ruh, 0) ** 2, axis=1))
        cnorm = np.linalg.norm(ch, axis=1)
        if omega0 is None:
            omega = np.where((bnorm > 1e-10) & (cnorm > 1e-10), cnorm / np.maximum(bnorm, 1e-300), 1.0)
        else:
            omega = np.full(S, omega0)
        omega = omega[:, None]
        x = self.x / Dc if warm else np.zeros((S, n))
        y = self.y / Dr if warm else np.zeros((S, m))
        x = np.clip(x, lbh, ubh)
        aty = spmvT(rp, ci, A, y, n)

        def T(x, y, aty):
            tau = eta / omega
            sig = eta * omega
            xn = np.clip((x - tau * (ch - aty)) / (1 + tau * qh), lbh, ubh)
            ax = spmv(rp, ci, A, 2 * xn - x)
            v = y - sig * ax
            a = v + sig * rlh
            bb = v + sig * ruh
            yn = np.where(a > 0, a, np.where(bb < 0, bb, 0.0))
            atyn = spmvT(rp, ci, A, yn, n)
            return xn, yn, atyn

        def wnorm(dx, dy):
            return np.sqrt(omega[:, 0] * np.sum(dx * dx, 1) + np.sum(dy * dy, 1) / omega[:, 0])

        done = np.zeros(S, bool)
        iters = np.zeros(S, int)
        x0, y0, aty0 = x.copy(), y.copy(), aty.copy()
        k = np.zeros(S)
        r0 = None
        rlast = None
        total = 0
        restarts = np.zeros(S, int)
        while total < max_iter:
            xt, yt, atyt = T(x, y, aty)
            re_ = restart_every or check
            if total % re_ == 0 and total % check != 0:
                r = wnorm(x - xt, y - yt)
                if r0 is None:
                    r0 = r.copy(); rlast = r.copy()
                rs = (r <= 0.2 * r0) | ((r <= 0.8 * r0) & (r > rlast))
                if art is not None:
                    rs |= k >= art * np.maximum(total, 1)
                rs &= ~done
                if rs.any():
                    dx = np.linalg.norm(xt - x0, axis=1)
                    dy = np.linalg.norm(yt - y0, axis=1)
                    upd = rs & (dx > 1e-10) & (dy > 1e-10)
                    lw = np.log(omega[:, 0])
                    lw[upd] = theta * np.log(dy[upd] / dx[upd]) + (1 - theta) * lw[upd]
                    if wclamp is not None:
                        lw = np.clip(lw, -np.log(wclamp), np.log(wclamp))
                    omega = np.exp(lw)[:, None]
                    x0[rs], y0[rs], aty0[rs] = xt[rs], yt[rs], atyt[rs]
                    x[rs], y[rs], aty[rs] = xt[rs], yt[rs], atyt[rs]
                    k[rs] = 0
                    r0[rs] = wnorm(x - T(x, y, aty)[0], y - T(x, y, aty)[1])[rs]
                    restarts[rs] += 1
                    rlast = r
                    if kernel_mode and km_rlast_inf:
                        rlast = np.where(rs, np.inf, r)
                    if kernel_mode and not km_hk0:
                        k[rs] = 1
                    total += 1
                    continue
                rlast = r
            if total % check == 0:
                r = wnorm(x - xt, y - yt)
                if r0 is None:
                    r0 = r.copy()
                    rlast = r.copy()
                # termination in original space using T(z)
                xo = xt * Dc
                yo = yt * Dr
                conv = self._kkt(xo, yo, c, q, eps)
                if trace is not None:
                    t_ = trace['idx']
                    trace.setdefault('rows', []).append((total, float(omega[t_, 0]), float(r[t_]), float(r0[t_]), int(k[t_]), float(self.last_pobj[t_]), float(self.last_dobj[t_]), int(restarts[t_])))
                newly = conv & ~done
                iters[newly] = total
                done |= conv
                if done.all():
                    x, y = xt, yt
                    break
                # restarts
                rs = (r <= 0.2 * r0) | ((r <= 0.8 * r0) & (r > rlast))
                if art is not None:
                    rs |= k >= art * np.maximum(total, 1)
                rs &= ~done
                if rs.any():
                    dx = np.linalg.norm(xt - x0, axis=1)
                    dy = np.linalg.norm(yt - y0, axis=1)
                    upd = rs & (dx > 1e-10) & (dy > 1e-10)
                    lw = np.log(omega[:, 0])
                    lw[upd] = theta * np.log(dy[upd] / dx[upd]) + (1 - theta) * lw[upd]
                    if wclamp is not None:
                        lw = np.clip(lw, -np.log(wclamp), np.log(wclamp))
                    omega = np.exp(lw)[:, None]
                    x0[rs], y0[rs], aty0[rs] = xt[rs], yt[rs], atyt[rs]
                    x[rs], y[rs], aty[rs] = xt[rs], yt[rs], atyt[rs]
                    k[rs] = 0
                    r0[rs] = wnorm(x - T(x, y, aty)[0], y - T(x, y, aty)[1])[rs]
                    restarts[rs] += 1
                rlast = r
                if kernel_mode and rs.any():
                    if km_rlast_inf:
                        rlast[rs] = np.inf
                    if km_hk0:
                        total += 1
                        continue
            # Halpern step for active scenarios
            kk = k[:, None]
            a1 = (kk + 1) / (kk + 2)
            a0 = 1 / (kk + 2)
            xn = a1 * ((1 + gamma) * xt - gamma * x) + a0 * x0
            yn = a1 * ((1 + gamma) * yt - gamma * y) + a0 * y0
            atyn = a1 * ((1 + gamma) * atyt - gamma * aty) + a0 * aty0
            act = ~done
            x[act], y[act], aty[act] = xn[act], yn[act], atyn[act]
            k[act] += 1
            total += 1
        iters[~done] = total
        self.x = x * Dc
        self.y = y * Dr
        return self.x, self.y, iters, done, restarts

    def _kkt(self, x, y, c, q, eps):
        b = self.b
        n = b.n
        ax = spmv(b.row_ptr, b.col_idx, b.A_val, x)
        pres = ax - np.clip(ax, b.rl, b.ru)
        aty = spmvT(b.row_ptr, b.col_idx, b.A_val, y, n)
        rc = c + q * x - aty
        fl = np.isfinite(b.lb)
        fu = np.isfinite(b.ub)
        lam = np.where(fl & fu, rc, np.where(fl, np.maximum(rc, 0), np.where(fu, np.minimum(rc, 0), 0.0)))
        dres = rc - lam
        pobj = np.sum(c * x + 0.5 * q * x * x, 1)
        yterm = np.where(y > 0, np.where(np.isfinite(b.rl), b.rl, 0) * y,
                         np.where(np.isfinite(b.ru), b.ru, 0) * y)
        lterm = np.where(lam > 0, np.where(fl, b.lb, 0) * lam, np.where(fu, b.ub, 0) * lam)
        dobj = -np.sum(0.5 * q * x * x, 1) + np.sum(yterm, 1) + np.sum(lterm, 1)
        bn = np.sqrt(np.sum(np.where(np.isfinite(b.rl), b.rl, 0) ** 2 + np.where(np.isfinite(b.ru), b.ru, 0) ** 2, 1))
        cn = np.linalg.norm(c, axis=1)
        ok = (np.linalg.norm(pres, axis=1) <= eps * (1 + bn)) & \
             (np.linalg.norm(dres, axis=1) <= eps * (1 + cn)) & \
             (np.abs(pobj - dobj) <= eps * (1 + np.abs(pobj) + np.abs(dobj)))
        self.last_pobj, self.last_dobj = pobj, dobj
        return ok
