"""CPU oracle, part 2: exact solution of the OSC QP + KKT certificate (numpy, fp64).

TEST INFRASTRUCTURE ONLY (see oracle/osc_qp.py header; parity unpinned vs reference outputs).

The reference solves the QP with OSQP 0.6.3 (operational_space_controller.h:346, 507-535) to
eps_abs = eps_rel = 1e-3 with time-based adaptive rho, so its own torques are only ~1e-3
accurate and run-to-run non-deterministic.  The QP is strictly convex
(H >= 2 w_reg I > 0) and always feasible (x = (-M^-1 C, 0, 0)), so its optimum is UNIQUE: that
optimum is what the product's torques are checked against.

Algorithm here: a textbook primal active-set method (Nocedal & Wright, Alg. 16.3) on the FULL
reference QP in OSQP form  min 1/2 x'Hx + f'x  s.t.  l <= A x <= u  (equality rows l == u are
always in the working set), started from a strictly feasible point, finished by an exact KKT
solve on the final active set.  It shares no code and no algorithm with the product's batched
interior-point kernel, so agreement between the two is an independent check.
"""
from __future__ import annotations

import dataclasses

import numpy as np

from osc_qp import OSCModel, QPData, b_matrix, contact_jacobian

INF_THRESH = 1e20   # |bound| >= this is "infinite" (the reference uses OSQP_INFTY = 1e30)


@dataclasses.dataclass
class ExactSolution:
    x: np.ndarray          # primal (n)
    y: np.ndarray          # OSQP-convention duals (m): H x + f + A' y = 0
    active: np.ndarray     # bool (m): row at a bound
    iterations: int
    cert: dict


def _constraints(qp: QPData):
    """Split l <= Ax <= u into equality rows and one-sided rows (row, sign): sign*a_i x <= sign*bound."""
    eq, ineq = [], []
    m, n = qp.A.shape
    # variables pinned by an identity box row with l == u (masked-off contact forces)
    pinned = np.zeros(n, bool)
    for i in range(m - n, m):
        if qp.l[i] == qp.u[i]:
            pinned[i - (m - n)] = True
    for i in range(m):
        lo, hi = qp.l[i], qp.u[i]
        if lo == hi:
            if i < m - n and not qp.A[i].any():
                # a trivial row 0 = 0 (the no-slip rows of a wheel off the ground): implied
                assert lo == 0.0, "inconsistent zero row"
                continue
            eq.append(i)
            continue
        support = np.nonzero(qp.A[i])[0]
        if i < m - n and pinned[support].all():
            # row only touches pinned variables (pyramid of a masked contact): it is a
            # constant 0 <= 0, implied by the pins; keeping it would make the working set
            # linearly dependent.
            continue
        if hi < INF_THRESH:
            ineq.append((i, +1.0, hi))
        if lo > -INF_THRESH:
            ineq.append((i, -1.0, -lo))
    return _independent(qp.A, eq), ineq


def _independent(A, eq):
    """A maximal linearly independent subset of the equality rows (QR with column pivoting of the
    unit-scaled A_eq').  The wheel no-slip rows of seven or eight grounded wheels are 14-16 rows on
    nv = 14 accelerations, so some are implied by the others (consistent by construction); kept,
    they make every working-set KKT matrix singular.  The rows kept are the original ones (an
    orthonormalised basis instead moves the constraint set by its rounding, amplified by the
    rows' near-dependence)."""
    if len(eq) == 0:
        return eq
    import scipy.linalg
    rows = A[eq] / np.linalg.norm(A[eq], axis=1, keepdims=True)
    _, R, piv = scipy.linalg.qr(rows.T, mode="economic", pivoting=True)
    d = np.abs(np.diag(R))
    rank = int((d > 1e-10 * d[0]).sum())
    return sorted(eq[p] for p in piv[:rank])


def _feasible_start(model: OSCModel, qp: QPData, M, C, J):
    """Strictly interior point for every one-sided row (u mid-box, z = (0, 0, fz0))."""
    nv, nu, nz = model.nv, model.nu, model.nz
    off_u = qp.A.shape[0] - model.n + nv
    off_z = off_u + nu
    lu, uu = qp.l[off_u:off_u + nu], qp.u[off_u:off_u + nu]
    u0 = np.where((lu < 0) & (uu > 0), 0.0, 0.5 * (lu + uu))
    z0 = np.zeros(nz)
    for k in range(model.nc):
        lo, hi = qp.l[off_z + 3 * k + 2], qp.u[off_z + 3 * k + 2]
        if lo != hi:
            z0[3 * k + 2] = min(1.0, 0.5 * (lo + hi))
    rhs = b_matrix(model) @ u0 + contact_jacobian(model, J) @ z0 - np.asarray(C).reshape(-1)
    dv0 = np.linalg.solve(np.asarray(M).reshape(nv, nv), rhs)
    return np.concatenate([dv0, u0, z0])


def _phase1_start(qp: QPData, eq, ineq):
    """A point that satisfies every equality row and is as deep inside the one-sided rows as the
    LP  max t  s.t.  A_eq x = b_eq,  s_i a_i x + t <= bound_i,  t <= 1  can make it (HiGHS).  Used
    when equality rows beyond the dynamics (wheel no-slip rows) constrain dv, so the dynamics-only
    start of _feasible_start no longer applies."""
    from scipy.optimize import linprog
    n = qp.A.shape[1]
    c = np.zeros(n + 1)
    c[-1] = -1.0
    A_ub = np.array([np.append(sg * qp.A[i], 1.0) for (i, sg, _) in ineq])
    b_ub = np.array([bd for (_, _, bd) in ineq])
    A_eq = np.hstack([qp.A[eq], np.zeros((len(eq), 1))])
    res = linprog(c, A_ub=A_ub, b_ub=b_ub, A_eq=A_eq, b_eq=qp.u[eq],
                  bounds=[(None, None)] * n + [(None, 1.0)], method="highs")
    if res.status != 0 or res.x[-1] <= 0.0:
        raise RuntimeError(f"QP has no strictly feasible point (phase-1 status {res.status})")
    return res.x[:n]


def kkt_certificate(qp: QPData, x: np.ndarray, y: np.ndarray) -> dict:
    """Residuals of the OSQP-form KKT conditions, each scaled to be dimensionless."""
    Ax = qp.A @ x
    grad = qp.H @ x + qp.f
    stat = grad + qp.A.T @ y
    scale_d = 1.0 + max(np.abs(grad).max(), np.abs(qp.A.T @ y).max())
    lo_fin = qp.l > -INF_THRESH
    hi_fin = qp.u < INF_THRESH
    viol = np.zeros_like(Ax)
    viol[hi_fin] = np.maximum(viol[hi_fin], Ax[hi_fin] - qp.u[hi_fin])
    viol[lo_fin] = np.maximum(viol[lo_fin], qp.l[lo_fin] - Ax[lo_fin])
    bnd = np.where(hi_fin, np.abs(qp.u), 0.0) + np.where(lo_fin, np.abs(qp.l), 0.0)
    scale_p = 1.0 + max(np.abs(Ax).max(), bnd.max())
    yp, ym = np.maximum(y, 0.0), np.maximum(-y, 0.0)
    # dual feasibility: positive y only on finite upper bounds, negative only on finite lower --
    # measured against the one-sided rows' own multipliers (a gradient scale set by the equality
    # rows' multipliers would hide a wrong-signed contact multiplier, qp_exact.solve_exact)
    dual_inf = max(np.where(hi_fin, 0.0, yp).max(), np.where(lo_fin, 0.0, ym).max())
    one_sided = qp.l != qp.u
    scale_y = 1.0 + (np.abs(y[one_sided]).max() if one_sided.any() else 0.0)
    # complementarity over the one-sided rows: an equality row's multiplier is free and its
    # residual is the primal measure (nearly dependent wheel rows carry multipliers ~1e13, whose
    # product with a 1e-9 residual is no complementarity gap)
    gap_hi = np.where(hi_fin & one_sided, qp.u - Ax, 0.0)
    gap_lo = np.where(lo_fin & one_sided, Ax - qp.l, 0.0)
    comp = np.maximum(np.abs(yp * gap_hi), np.abs(ym * gap_lo)).max()
    return dict(stationarity=float(np.abs(stat).max() / scale_d),
                primal=float(viol.max() / scale_p),
                dual=float(dual_inf / scale_y),
                complementarity=float(comp / (scale_d * scale_p)))


def _kkt_solve(K, rhs):
    """The working-set KKT system.  When the working set is linearly dependent -- a contact at
    the pyramid apex, where its four pyramid rows and fz >= 0 are all active on three forces --
    K is exactly singular: x is still unique (H > 0), the multipliers are not; least squares
    returns x and the minimum-norm multipliers.  (A nearly singular K can come back from the LU
    solve finite but wrong: its residual decides.)"""
    try:
        sol = np.linalg.solve(K, rhs)
        if np.all(np.isfinite(sol)):
            res = np.abs(K @ sol - rhs).max()
            if res <= 1e-9 * (np.abs(rhs).max() + np.abs(K).max() * np.abs(sol).max()):
                return sol
    except np.linalg.LinAlgError:
        pass
    return np.linalg.lstsq(K, rhs, rcond=None)[0]


def _primal_active_set(model: OSCModel, qp: QPData, M, C, J, eq, ineq, max_iter: int):
    """Primal active-set method (Nocedal & Wright, Alg. 16.3) from a strictly feasible point.
    Returns the working set (indices into ineq) and the iteration count; RuntimeError when it
    cycles past max_iter (degenerate working sets of the wheel rows)."""
    n = model.n
    A = qp.A
    x = (_feasible_start(model, qp, M, C, J) if qp.Aw is None else _phase1_start(qp, eq, ineq))
    # sanity: strictly feasible for all one-sided rows
    for (i, sg, bd) in ineq:
        assert sg * (A[i] @ x) < bd, "start point not strictly feasible"
    W: list[int] = []                     # indices into ineq
    Aeq, beq = A[eq], qp.u[eq]
    neq = Aeq.shape[0]
    degenerate = False
    it = 0
    for it in range(1, max_iter + 1):
        # Solve the equality-constrained QP on the working set directly for its minimiser x_W
        # (more accurate than solving for the step when K is ill-conditioned).
        rows = np.vstack([Aeq] + [ineq[w][1] * A[ineq[w][0]][None, :] for w in W])
        rhs_b = np.concatenate([beq] + [[ineq[w][2]] for w in W]) if W else beq
        k = rows.shape[0]
        K = np.zeros((n + k, n + k))
        K[:n, :n] = qp.H
        K[:n, n:] = rows.T
        K[n:, :n] = rows
        sol = _kkt_solve(K, np.concatenate([-qp.f, rhs_b]))
        p, lam = sol[:n] - x, sol[n:]
        if np.abs(p).max() <= 1e-9 * (1.0 + np.abs(x).max()):
            x = sol[:n]
            lam_in = lam[neq:]
            # the sign test is relative to the one-sided rows' own multipliers: the equality
            # multipliers (dynamics, and the wheel rows' ~1e6 when those rows fix dv) would hide
            # a wrong-signed contact multiplier of the W-scale (1e-4) under a tolerance of 1e-10
            if len(W) == 0:
                break
            tol_in = 1e-10 * (1.0 + np.abs(lam_in).max())
            if lam_in.min() >= -tol_in:
                break
            # Bland's rule after a degenerate step (alpha = 0: a dependent working set, where the
            # multipliers are not unique and the most negative one can cycle): the wrong-signed
            # row of lowest index leaves
            if degenerate:
                W.pop(min((j for j in range(len(W)) if lam_in[j] < -tol_in), key=lambda j: W[j]))
            else:
                W.pop(int(np.argmin(lam_in)))
            continue
        alpha, block = 1.0, None
        for j, (i, sg, bd) in enumerate(ineq):
            if j in W:
                continue
            ap = sg * (A[i] @ p)
            if ap > 1e-9 * np.abs(p).max():
                a = (bd - sg * (A[i] @ x)) / ap
                if a < alpha:   # (ties: the lowest index, j ascending -- Bland)
                    alpha, block = max(a, 0.0), j
        degenerate = block is not None and alpha <= 1e-14
        x = x + alpha * p
        if block is not None:
            W.append(block)
    else:
        raise RuntimeError("active set did not converge")
    return W, it


def _dual_active_set(qp: QPData, eq, ineq, max_iter: int = 5000):
    """Goldfarb & Idnani's dual active-set method (Math. Programming 27, 1983; the algorithm of
    quadprog) for the strictly convex QP: start at the unconstrained minimiser, add the equality
    rows, then repeatedly the most violated one-sided row, keeping the working set's multipliers
    non-negative.  A row linearly dependent on the working set is never added: a pure dual step
    first drops a working row (the degenerate pyramid apex; dependent wheel rows).  Every iterate
    is dual feasible and the dual objective rises strictly, so it terminates without the primal
    method's cycling.  Returns the working set (indices into ineq) and the iteration count.
    Rows as normals c'x >= b: a one-sided row sg a_i x <= bd is (-sg a_i) x >= -bd.
    (J, R recomputed per step by a QR of L^-T' N: n <= 46, cheap, no update formulas to get
    wrong.)"""
    import scipy.linalg as sla
    H, f, A = qp.H, qp.f, qp.A
    n = H.shape[0]
    Lc = np.linalg.cholesky(H)
    J0 = sla.solve_triangular(Lc, np.eye(n), lower=True).T          # L^-T: J0 J0' = H^-1
    x = -np.linalg.solve(H, f)
    normals = [A[i] for i in eq] + [-sg * A[i] for (i, sg, _) in ineq]
    rhs = [qp.u[i] for i in eq] + [-bd for (_, _, bd) in ineq]
    neq = len(eq)
    act: list[int] = []               # indices into normals
    u = np.zeros(0)

    def factor():
        q = len(act)
        if q == 0:
            return J0, np.zeros((0, 0))
        Q, R = np.linalg.qr(J0.T @ np.column_stack([normals[k] for k in act]), mode="complete")
        return J0 @ Q, R[:q, :q]

    def step_dirs(c):
        J, R = factor()
        q = len(act)
        d = J.T @ c
        z = J[:, q:] @ d[q:]
        r = sla.solve_triangular(R, d[:q]) if q else np.zeros(0)
        return z, r

    scale_c = [np.abs(c).max() for c in normals]
    it = 0
    for k in range(neq):              # equality rows: always active, multipliers of any sign
        c = normals[k]
        z, r = step_dirs(c)
        if np.abs(z).max() <= 1e-13 * scale_c[k]:
            continue                  # implied by the rows already in (consistent by construction)
        t = (rhs[k] - c @ x) / (z @ c)
        x = x + t * z
        u = np.append(u - t * r, t)
        act.append(k)
    while True:
        it += 1
        if it > max_iter:
            raise RuntimeError("dual active set did not converge")
        xs = np.abs(x).max()
        s = np.array([normals[k] @ x - rhs[k] for k in range(neq, len(normals))])
        viol = s / (1.0 + np.array(scale_c[neq:]) * xs + np.abs(rhs[neq:]))
        p = neq + int(np.argmin(viol)) if len(s) else None
        if p is None or viol[p - neq] >= -1e-14 or p in act:
            break
        c = normals[p]
        up = np.append(u, 0.0)
        while True:
            z, r = step_dirs(c)
            q = len(act)
            t1, kdrop = np.inf, None
            for j in range(q):
                if act[j] >= neq and r[j] > 1e-14 * (1.0 + np.abs(r).max()):
                    ratio = up[j] / r[j]
                    if ratio < t1:
                        t1, kdrop = ratio, j
            dependent = np.abs(z).max() <= 1e-13 * scale_c[p] * (1.0 + np.abs(J0).max())
            t2 = np.inf if dependent else -(c @ x - rhs[p]) / (z @ c)
            t = min(t1, t2)
            if not np.isfinite(t):
                raise RuntimeError("QP infeasible (dual unbounded)")
            if not dependent:
                x = x + t * z
            up[:q] -= t * r
            up[q] += t
            if t2 <= t1:              # full step: p joins the working set
                act.append(p)
                u = up
                break
            del act[kdrop]            # partial step: a working row whose multiplier hit 0 leaves
            up = np.delete(up, kdrop)
            if not dependent and c @ x - rhs[p] >= 0.0:
                u = up[:-1]           # (p satisfied without joining: cannot happen for t < t2)
                break
    return [k - neq for k in act if k >= neq], it


def _finish(model: OSCModel, qp: QPData, eq, ineq, W, it, refine_steps: int,
            basis: bool = False) -> ExactSolution:
    """Exact KKT solve on the identified working set W, polished by mixed-precision iterative
    refinement, with the multipliers mapped to OSQP's convention and the KKT certificate.
    basis=True (the retry when the first solve ends off the equality rows): the working set's rows
    are first reduced to a basis of their span by QR with column pivoting -- a nearly dependent
    working set (wheel rows next to an apex contact) makes the full KKT matrix numerically
    singular, while the optimum (unique, H > 0) satisfies every row of the span; the dropped rows
    get zero multipliers."""
    n = model.n
    A = qp.A
    Aeq = A[eq]
    neq = Aeq.shape[0]
    rows = np.vstack([Aeq] + [ineq[w][1] * A[ineq[w][0]][None, :] for w in W])
    rhs_b = np.concatenate([qp.u[eq]] + [[ineq[w][2]] for w in W]) if W else qp.u[eq]
    keep = np.arange(rows.shape[0])
    if basis and rows.shape[0]:
        import scipy.linalg
        un = rows / np.linalg.norm(rows, axis=1, keepdims=True)
        _, R, piv = scipy.linalg.qr(un.T, mode="economic", pivoting=True)
        d = np.abs(np.diag(R))
        keep = np.sort(piv[:int((d > 1e-9 * d[0]).sum())])
        rows, rhs_b = rows[keep], rhs_b[keep]
    k = rows.shape[0]
    K = np.zeros((n + k, n + k))
    K[:n, :n] = qp.H
    K[:n, n:] = rows.T
    K[n:, :n] = rows
    rhs = np.concatenate([-qp.f, rhs_b])
    if basis:   # (the retry: the whole solve in extended precision, then refined there)
        Kl = K.astype(np.longdouble)
        soll = _solve_ld(Kl, rhs)
        for _ in range(refine_steps):
            soll = soll + _solve_ld(Kl, rhs.astype(np.longdouble) - Kl @ soll)
        return _finish_tail(model, qp, eq, ineq, W, it, soll.astype(np.float64), keep, basis)
    sol = _kkt_solve(K, rhs)
    # Mixed-precision iterative refinement: residuals in x87 extended precision (eps ~1e-19),
    # corrections from the fp64 factorisation.  Converges to ~eps_ext * cond(K), i.e. well
    # below fp64 round-off for this QP (cond(K) ~ 1e8..1e10 with w_reg = 1e-4).
    Kl = K.astype(np.longdouble)
    rhsl = rhs.astype(np.longdouble)
    soll = sol.astype(np.longdouble)
    for _ in range(refine_steps):
        r = rhsl - Kl @ soll
        soll = soll + _kkt_solve(K, r.astype(np.float64)).astype(np.longdouble)
    return _finish_tail(model, qp, eq, ineq, W, it, soll.astype(np.float64), keep, basis)


def _finish_tail(model, qp, eq, ineq, W, it, sol, keep, basis):
    n = model.n
    A = qp.A
    neq = len(eq)
    x, lam_k = sol[:n], sol[n:]
    lam = np.zeros(neq + len(W))
    lam[keep] = lam_k
    # a degenerate working set whose KKT system came back inconsistent: once more on a basis of
    # its rows, then refuse rather than return a point off the equality rows
    eq_res = np.abs(A[eq] @ x - qp.u[eq]).max() if eq else 0.0
    if not eq_res <= 1e-8 * (1.0 + np.abs(qp.u[eq]).max() if eq else 1.0):
        if not basis:
            return _finish(model, qp, eq, ineq, W, it, 4, basis=True)
        raise RuntimeError(f"active set ended off the equality rows ({eq_res:.1e})")
    y = np.zeros(A.shape[0])
    y[eq] += lam[:neq]
    active = np.zeros(A.shape[0], bool)
    active[eq] = True
    for j, w in enumerate(W):
        i, sg, _ = ineq[w]
        y[i] += sg * lam[neq + j]
        active[i] = True
    cert = kkt_certificate(qp, x, y)
    return ExactSolution(x=x, y=y, active=active, iterations=it, cert=cert)


def _solve_ld(K, rhs):
    """Gaussian elimination with partial pivoting in x87 extended precision (eps ~1e-19), for the
    final KKT system of a working set that is nearly dependent (wheel rows whose smallest singular
    value is ~1e-8 of the largest: its fp64 factorisation cannot serve iterative refinement)."""
    A = np.array(K, dtype=np.longdouble)
    b = np.array(rhs, dtype=np.longdouble)
    n = A.shape[0]
    for k in range(n):
        p = k + int(np.argmax(np.abs(A[k:, k])))
        if p != k:
            A[[k, p]] = A[[p, k]]
            b[[k, p]] = b[[p, k]]
        if A[k, k] == 0:
            continue
        f = A[k + 1:, k] / A[k, k]
        A[k + 1:, k:] -= f[:, None] * A[k, k:][None, :]
        b[k + 1:] -= f * b[k]
    x = np.zeros(n, dtype=np.longdouble)
    for k in range(n - 1, -1, -1):
        x[k] = (b[k] - A[k, k + 1:] @ x[k + 1:]) / A[k, k] if A[k, k] != 0 else 0
    return x


def solve_exact(model: OSCModel, qp: QPData, M, C, J, max_iter: int = 500,
                refine_steps: int = 4, method: str = "auto") -> ExactSolution:
    """The QP's unique optimum with its KKT certificate.  method "primal": the primal active-set
    method; "dual": Goldfarb-Idnani; "auto": primal, and the dual method where the primal one
    cycles or ends on an inconsistent degenerate working set (a few wheel-row envs)."""
    eq, ineq = _constraints(qp)
    if method in ("primal", "auto"):
        try:
            W, it = _primal_active_set(model, qp, M, C, J, eq, ineq, max_iter)
            sol = _finish(model, qp, eq, ineq, W, it, refine_steps)
            # (auto: a primal working set whose certificate fails goes to the dual method too)
            if method == "primal" or certified(sol.cert, 1e-8):
                return sol
        except RuntimeError:
            if method == "primal":
                raise
    W, it = _dual_active_set(qp, eq, ineq)
    sol = _finish(model, qp, eq, ineq, W, it, refine_steps)
    # the fallback is held to the same certificate: an "exact" answer the KKT test refuses is an
    # error, never a silent return (a GPU fallback of the same algorithm would share its faults)
    if method == "auto" and not certified(sol.cert, 1e-8):
        raise RuntimeError(f"dual active set ended uncertified: {sol.cert}")
    return sol


def certified(cert: dict, tol: float = 1e-9) -> bool:
    return all(v <= tol for v in cert.values())
