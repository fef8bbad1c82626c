"""Diagnostic (CPU): numpy model of osc_ipm_kernel's interior-point method on the reduced QP, for
tuning the iteration strategy before touching the kernel.  Not a test and not product code.

Reduced QP (as osc_setup_kernel builds it): y = (dv_a, z), dv_b and u affine in y,
    min 1/2 y'Hr y + g'y   s.t.  G y + s = h, s >= 0
rows: torque upper/lower interleaved (2q, 2q+1), then per contact k: 4 pyramid rows,
-fz <= 0, fz <= 1e4 (masked contacts: no rows, z pinned to 0).

Usage: python tools/ipm_model.py [robot] [nenv] [variant ...]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np  # noqa: E402
import scipy.linalg as sla  # noqa: E402
from osc_amd.synth import SEED_BASE, generate  # noqa: E402
from osc_qp import BIG_NUMBER, build_qp, contact_jacobian, load_model  # noqa: E402


def reduce_qp(model, M, C, J, b, T, mask):
    qp = build_qp(model, M, C, J, b, T, mask)
    nv, nu, nc = model.nv, model.nu, model.nc
    nz, NB = 3 * nc, nv - nu
    NY = nu + nz
    n = model.n
    Jc = contact_jacobian(model, J)
    pinned = np.repeat(np.asarray(mask) == 0, 3)
    Jcm = Jc * (~pinned)[None, :]
    Mbb_inv = np.linalg.inv(M[:NB, :NB])
    # dv_b = Xy y + x0
    Xy = np.hstack([-Mbb_inv @ M[:NB, NB:], Mbb_inv @ Jcm[:NB]])
    x0 = -Mbb_inv @ C[:NB]
    # u = M[NB:, :NB] dv_b + M[NB:, NB:] dv_a + C_a - Jc_a z
    Uy = M[NB:, :NB] @ Xy + np.hstack([M[NB:, NB:], -Jcm[NB:]])
    u0 = M[NB:, :NB] @ x0 + C[NB:]
    P = np.zeros((n, NY))
    p0 = np.zeros(n)
    P[:NB] = Xy
    p0[:NB] = x0
    P[NB:nv, :nu] = np.eye(nu)
    P[nv:nv + nu] = Uy
    p0[nv:nv + nu] = u0
    P[nv + nu:, nu:] = np.eye(nz)
    Hr = P.T @ qp.H @ P
    g = P.T @ (qp.H @ p0 + qp.f)
    rows, hs = [], []
    for q in range(nu):
        rows.append(Uy[q]); hs.append(model.u_ub[q] - u0[q])
        rows.append(-Uy[q]); hs.append(u0[q] - model.u_lb[q])
    for k in range(nc):
        if mask[k] == 0:
            continue
        zc = nu + 3 * k
        for sx, sy in ((1, 1), (-1, 1), (1, -1), (-1, -1)):
            r = np.zeros(NY); r[zc] = sx; r[zc + 1] = sy; r[zc + 2] = -model.mu
            rows.append(r); hs.append(0.0)
        r = np.zeros(NY); r[zc + 2] = -1.0; rows.append(r); hs.append(0.0)
        r = np.zeros(NY); r[zc + 2] = 1.0; rows.append(r); hs.append(BIG_NUMBER * mask[k])
    return Hr, g, np.array(rows), np.array(hs), P, p0


def reduce_qp_tau(model, M, C, J, b, T, mask):
    """Alternative reduction y = (u, z): dv = M^-1 (B u + Jc z - C) from all nv dynamics rows,
    so the torque bounds are plain bounds on y (no dense U rows)."""
    qp = build_qp(model, M, C, J, b, T, mask)
    nv, nu, nc = model.nv, model.nu, model.nc
    nz, NB = 3 * nc, nv - nu
    NY = nu + nz
    n = model.n
    Jc = contact_jacobian(model, J)
    pinned = np.repeat(np.asarray(mask) == 0, 3)
    Jcm = Jc * (~pinned)[None, :]
    Minv = np.linalg.inv(M)
    Bm = np.zeros((nv, nu)); Bm[NB:] = np.eye(nu)
    P = np.zeros((n, NY))
    p0 = np.zeros(n)
    P[:nv] = Minv @ np.hstack([Bm, Jcm])
    p0[:nv] = -Minv @ C
    P[nv:nv + nu, :nu] = np.eye(nu)
    P[nv + nu:, nu:] = np.eye(nz)
    Hr = P.T @ qp.H @ P
    g = P.T @ (qp.H @ p0 + qp.f)
    rows, hs = [], []
    for q in range(nu):
        r = np.zeros(NY); r[q] = 1.0; rows.append(r); hs.append(model.u_ub[q])
        r = np.zeros(NY); r[q] = -1.0; rows.append(r); hs.append(-model.u_lb[q])
    for k in range(nc):
        if mask[k] == 0:
            continue
        zc = nu + 3 * k
        for sx, sy in ((1, 1), (-1, 1), (1, -1), (-1, -1)):
            r = np.zeros(NY); r[zc] = sx; r[zc + 1] = sy; r[zc + 2] = -model.mu
            rows.append(r); hs.append(0.0)
        r = np.zeros(NY); r[zc + 2] = -1.0; rows.append(r); hs.append(0.0)
        r = np.zeros(NY); r[zc + 2] = 1.0; rows.append(r); hs.append(BIG_NUMBER * mask[k])
    return Hr, g, np.array(rows), np.array(hs), P, p0


def ldl_factor(K):
    """The kernel's LDL^T: right-looking, Cholesky-infinity guard (pivot <= 1e-13 * original
    diagonal -> 1e128), as ldl_rows in osc_batch.hip."""
    A = K.copy()
    n = len(A)
    dg = np.diag(K).copy()
    L = np.eye(n)
    d = np.zeros(n)
    for k in range(n):
        dk = A[k, k]
        if not dk > 1e-13 * dg[k]:
            dk = 1e128
        d[k] = dk
        col = A[k + 1:, k] / dk
        L[k + 1:, k] = col
        A[k + 1:, k + 1:] -= np.outer(col, A[k, k + 1:])
    return L, d


def ldl_solve(F, r):
    L, d = F
    z = sla.solve_triangular(L, r, lower=True, unit_diagonal=True)
    return sla.solve_triangular(L.T, z / d, lower=False, unit_diagonal=True)


FINAL = {}     # (s, lam) of the last returned iterate, for refinement studies
RD_EXACT = None   # optional y -> Hr y + g evaluated in factored form (X'(Hdv (X y + x0) + gdv) ..)
RD_EXACT_MU = 1e-6
NU_STOP = 12   # torque entries of y in torque coordinates (Go2) for the "ustop" variant
TRACE = None   # set to a list to record (it, mu, a_aff, a, alpha, sigma) per iteration


def ipm(Hr, g, G, h, eps_mu=1e-12, max_iter=40, variant=(), init=None):
    """init: (y, s, lam) -- a warm start (tools/warm_model.py) instead of the cold start."""
    m = len(h)
    small = np.abs(h) < 1e3
    if init is not None:
        y, s, lam = (np.array(v, dtype=np.float64) for v in init)
    elif "y0_nofz" in variant:                   # least-squares start without the fz <= big rows
        keep = ~np.isclose(h, BIG_NUMBER)
        Gs, hs = G[keep], h[keep]
        y = np.linalg.solve(Hr + Gs.T @ Gs, -g + Gs.T @ hs)
    elif "y0_small" in variant:                # least-squares start over the |h| < 1e3 rows only
        Gs, hs = G[small], h[small]
        y = np.linalg.solve(Hr + Gs.T @ Gs, -g + Gs.T @ hs)
    elif "y0_unc" in variant:                  # unconstrained minimiser
        y = np.linalg.solve(Hr, -g)
    else:
        K0 = Hr + G.T @ G
        y = np.linalg.solve(K0, -g + G.T @ h)
    zr = G @ y - h
    if init is not None:
        pass
    elif "mehrotra_init" in variant:
        s, lam = -zr.copy(), zr.copy()
        ds_ = max(-1.5 * s.min(), 0.0); dl_ = max(-1.5 * lam.min(), 0.0)
        s += ds_; lam += dl_
        sl = s @ lam
        s += 0.5 * sl / lam.sum(); lam += 0.5 * sl / s.sum()
    elif any(v.startswith("lsR") for v in variant):
        # scaled least-squares start: rows weighted by R_r = c x (Hr diagonal under row r), so
        # the start sees the bounds at the objective's own scale; lambda0 = R (G y0 - h) is the
        # penalty estimate of the multipliers.  Shifts as the kernel's, lambda's in R units.
        v = [v for v in variant if v.startswith("lsR")][0]
        c = float(v[3:])
        keep = ~np.isclose(h, BIG_NUMBER)
        dgh = np.abs(np.diag(Hr))
        R = c * (np.abs(G) @ dgh) / np.maximum(np.abs(G).sum(axis=1), 1e-300)
        Gs, hs, Rs = G[keep], h[keep], R[keep]
        y = np.linalg.solve(Hr + Gs.T @ (Rs[:, None] * Gs), -g + Gs.T @ (Rs * hs))
        zr = G @ y - h
        ap = max(zr.max(), 0.0)
        s = -zr + (1.0 + ap if zr.max() >= 0 else 0.0)
        zl = zr * (R if "lsRlam" not in variant else 1.0)
        rowc = [float(v[4:]) for v in variant if v.startswith("rowc") and len(v) > 4]
        if rowc:                                   # per-row floors, products >= c0 x mean
            s = np.maximum(-zr, 1.0)
            mu0 = rowc[0] * np.abs(zl).mean()
            lam = np.maximum(zl, mu0 / s)
            s = np.maximum(s, mu0 / lam)
        elif "lsRdual1" in variant:                  # lambda shift in units of R
            ad = max((-zr).max(), 0.0)
            lam = R * (zr + 1.0 + ad)
        else:
            ad = (-zl).max()
            lam = zl + (1.0 + ad if ad >= 0 else 0.0)
        eta = 0.99
    elif "init_row1" in variant:               # per-row: slack and multiplier each >= 1
        s, lam = np.maximum(-zr, 1.0), np.maximum(zr, 1.0)
    elif "init_rowc" in variant:               # per-row slack; lambda centred on mu0
        s = np.maximum(-zr, 1.0)
        lam = np.maximum(zr, 1.0 / s)
    elif "init_rowc10" in variant:
        s = np.maximum(-zr, 1.0)
        lam = np.maximum(zr, 10.0 / s)
    elif any(v.startswith("init_rowm") for v in variant):   # shift over |h| < 1e3 rows only
        v = [v for v in variant if v.startswith("init_rowm")][0]
        c = float(v[9:]) if len(v) > 9 else 1.0
        small = np.abs(h) < 1e3
        ap = max(-(-zr[small]).min(), 0.0); ad = max(-zr[small].min(), 0.0)
        s = np.maximum(-zr + ap + c, c)
        lam = np.maximum(zr + ad + c, c * c / s)
        if "mcorr" in variant:                 # Mehrotra's second shift (centering)
            sl = s[small] @ lam[small]
            s[small] += 0.5 * sl / lam[small].sum()
            lam[small] += 0.5 * sl / s[small].sum()
    elif any(v.startswith("shift") for v in variant):
        c = [float(v[5:]) for v in variant if v.startswith("shift")][0]
        ap, ad = -(-zr).min(), -zr.min()
        s = -zr + (c + ap if ap >= 0 else 0.0)
        lam = zr + (c + ad if ad >= 0 else 0.0)
    else:
        ap, ad = (-zr).min(), zr.min()          # kernel: shift by 1 + max(-s), 1 + max(-lambda)
        ap, ad = -ap, -ad
        s = -zr + (1.0 + ap if ap >= 0 else 0.0)
        lam = zr + (1.0 + ad if ad >= 0 else 0.0)
    eta = 0.99
    rp_c = None
    last_du = None
    for it in range(max_iter + 1):
        for v in variant:
            if v.startswith("recenter") and it == int(v[8:]) and s @ lam / m > 1e-6:
                s = np.maximum(h - G @ y, 0.0) + 1.0   # re-centre a stalled iterate in place
                lam = np.ones(m)
                rp_c = None
        rp = G @ y + s - h
        thr = [float(v[7:]) for v in variant if v.startswith("rpcarry") and len(v) > 7]
        mu_now = s @ lam / m
        if "rpcarry" in variant or thr:
            if rp_c is None or (thr and mu_now <= thr[0]):
                rp_c = rp
            rp = rp_c
        rd = Hr @ y + g + G.T @ lam
        if RD_EXACT is not None and s @ lam / m <= RD_EXACT_MU:
            rd = RD_EXACT(y) + G.T @ lam     # factored gradient (never through Hr)
        mu = s @ lam / m
        if mu <= eps_mu:
            FINAL.update(s=s.copy(), lam=lam.copy())
            return y, it, True
        asstop = [v for v in variant if v.startswith("asstop")]
        if asstop:
            # active-set stop ("asstop<mu>,<k>"): mu <= <mu> and the rows with lambda > s the same
            # for <k> consecutive iterations -- the refinement takes it from there
            mth, kk = asstop[0][6:].split(",")
            act = tuple(np.nonzero(lam > s)[0])
            hist = FINAL.setdefault("_acts", [])
            if it == 0:
                hist.clear()
            hist.append(act)
            if mu <= float(mth) and len(hist) > int(kk) and all(a == act for a in hist[-int(kk) - 1:]):
                FINAL.update(s=s.copy(), lam=lam.copy())
                return y, it, True
        ustop = [v for v in variant if v.startswith("ustop")]
        if ustop and last_du is not None:
            # torque-coordinate stop: the last step moved the torques y[:NU] by less than
            # tol * max(|u|, 1) while mu is already small ("ustop<tol>,<mu>")
            tol, mth = (float(a) for a in ustop[0][5:].split(","))
            if mu <= mth and last_du <= tol * max(np.abs(y[:NU_STOP]).max(), 1.0):
                return y, it, True
        if it >= max_iter:
            FINAL.update(s=s.copy(), lam=lam.copy())
            return y, it, False
        pol = [float(v[6:]) for v in variant if v.startswith("polish")]
        if pol and mu <= pol[0]:
            # active-set polish: rows with s < lambda treated as equalities, exact KKT solve
            A = s < lam
            GA = G[A]
            nA = int(A.sum())
            try:
                if "penalty" in variant:   # kernel form: (Hr + rho GA'GA), refined 2x
                    rho = 1e8
                    Kp = Hr + rho * GA.T @ GA
                    Fp = ldl_factor(Kp)
                    yp = ldl_solve(Fp, -g + rho * GA.T @ h[A])
                    lp = rho * (GA @ yp - h[A])
                    for _ in range(2):
                        r1 = -g - Hr @ yp - GA.T @ lp       # stationarity residual
                        r2 = h[A] - GA @ yp                  # active-row residual
                        # regularised KKT [Hr GA'; GA -1/rho] correction via the Schur form
                        dy = ldl_solve(Fp, r1 + rho * GA.T @ r2)
                        dl_ = rho * (GA @ dy - r2)
                        yp, lp = yp + dy, lp + dl_
                else:
                    KKT = np.block([[Hr, GA.T], [GA, np.zeros((nA, nA))]])
                    sol = np.linalg.solve(KKT, np.concatenate([-g, h[A]]))
                    yp, lp = sol[:len(g)], sol[len(g):]
                ptol = [float(v[4:]) for v in variant if v.startswith("ptol")]
                ptol = ptol[0] if ptol else 1e-9
                feas = np.all(G @ yp <= h + ptol * (1 + np.abs(h)))
                dual = nA == 0 or np.all(lp >= -ptol * (1 + np.abs(lp).max()))
                if feas and dual:
                    return yp, it + 1, True
            except np.linalg.LinAlgError:
                pass
        D = lam / s
        K = Hr + G.T @ (D[:, None] * G)
        Kf = ldl_factor(K)

        def direction(rc):
            w = (rc - lam * rp) / s
            dy = ldl_solve(Kf, -rd + G.T @ w)
            ds = -rp - G @ dy
            dl = -(rc + lam * ds) / s
            return dy, ds, dl

        def max_step(ds, dl):
            a = 1.0
            neg = ds < 0
            if neg.any():
                a = min(a, (-s[neg] / ds[neg]).min())
            neg = dl < 0
            if neg.any():
                a = min(a, (-lam[neg] / dl[neg]).min())
            return a

        dy, ds, dl = direction(s * lam)
        a_aff = max_step(ds, dl)
        skip = [float(v[8:]) for v in variant if v.startswith("skipcorr")]
        if skip and a_aff >= skip[0]:           # near the end: affine (Newton) step only
            eta = min(1.0 - 1e-5, max(0.99, 1.0 - mu, 1.0 - 0.1 * (1.0 - a_aff)))
            alpha = min(1.0, eta * a_aff)
            y, s, lam = y + alpha * dy, s + alpha * ds, lam + alpha * dl
            continue
        mu_aff = (s + a_aff * ds) @ (lam + a_aff * dl) / m
        sig = (mu_aff / mu) ** (2 if "sig2" in variant else 3)
        so = 1.0
        for v in variant:
            if v.startswith("soguard"):       # drop the second-order term after a short affine step
                if a_aff < float(v[7:]):
                    so = 0.0
            if v.startswith("sigfloor"):      # sigma >= c after a short affine step
                if a_aff < 0.1:
                    sig = max(sig, float(v[8:]))
        if "sigcap" in variant:
            sig = min(sig, 0.5)
        rc = s * lam + so * ds * dl - sig * mu
        dy, ds, dl = direction(rc)
        a = max_step(ds, dl)
        if "gondzio" in variant or ("gshort" in variant and a < 0.5):
            # one centrality corrector (Gondzio 1996): push complementarity products into a box
            at = min(1.0, 1.5 * a + 0.1)
            st, lt = s + at * ds, lam + at * dl
            v = st * lt
            tgt = sig * mu
            lo, hi = 0.1 * tgt, 10.0 * tgt
            corr = np.where(v < lo, lo - v, np.where(v > hi, np.maximum(hi - v, -hi), 0.0))
            dy2, ds2, dl2 = direction(rc - corr)
            a2 = max_step(ds2, dl2)
            if a2 >= 1.01 * a:
                dy, ds, dl, a = dy2, ds2, dl2, a2
        if "eta" in variant:
            eta = max(0.99, 1.0 - mu)
        for v in variant:
            if v.startswith("etafix"):
                eta = float(v[6:])
            if v.startswith("etak"):        # eta = max(0.99, 1 - k mu)
                eta = max(0.99, 1.0 - float(v[4:]) * mu)
            if v.startswith("etaa"):        # eta = max(0.99, 1 - a_aff-based)  (PCx-like)
                eta = max(0.99, 1.0 - (1.0 - a_aff) * float(v[4:]))
            if v.startswith("etam"):        # eta = max(0.99, 1 - mu, 1 - c (1 - a_aff))
                eta = max(0.99, 1.0 - mu, 1.0 - (1.0 - a_aff) * float(v[4:]))
            if v.startswith("cap"):         # eta <= 1 - c
                eta = min(eta, 1.0 - float(v[3:]))
            if v.startswith("etalate"):     # from iteration k on: eta = max(0.99, 1 - mu), capped
                if it >= int(v[7:]):
                    eta = min(max(0.99, 1.0 - mu), 1.0 - 1e-5)
        alpha = min(1.0, eta * a)
        if TRACE is not None:
            TRACE.append((it, mu, a_aff, a, alpha, sig, float(np.abs(rp).max()),
                          float(np.abs(rd).max())))
        last_du = float(np.abs(alpha * dy[:NU_STOP]).max())
        y, s, lam = y + alpha * dy, s + alpha * ds, lam + alpha * dl
        if rp_c is not None:
            rp_c = (1.0 - alpha) * rp_c
    return y, max_iter, False


def main():
    robot = sys.argv[1] if len(sys.argv) > 1 else "unitree_go2"
    nenv = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    vs = [a for a in sys.argv[3:] if not a.startswith("--")]
    variants = [tuple(v.split("+")) if v != "base" else () for v in (vs or ["base"])]
    model = load_model(robot)
    d = generate(robot, nenv, SEED_BASE + 2, "standing", "ones")
    probs = [reduce_qp(model, *(d[k][e] for k in ("M", "C", "J", "b", "T", "mask")))
             for e in range(nenv)]
    ref = [ipm(*p[:4], eps_mu=1e-12, max_iter=80)[0] for p in probs]
    for v in variants:
        its, errs = [], []
        for p, yr in zip(probs, ref):
            y, it, ok = ipm(*p[:4], variant=v)
            its.append(it)
            errs.append(np.abs(y - yr).max() / max(np.abs(yr).max(), 1.0))
        its = np.array(its)
        if "--hist" in sys.argv:
            print("   hist", np.bincount(its).tolist())
        print(f"{'+'.join(v) or 'base':24s} fail {int((its >= 40).sum())} mean_it {its.mean():6.2f}  wave4_max "
              f"{its.reshape(-1, 4).max(1).mean():6.2f}  max_it {its.max():3d}  "
              f"max_err {max(errs):.2e}")


if __name__ == "__main__":
    main()
