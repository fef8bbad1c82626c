"""Numpy model of a Goldfarb-Idnani dual active-set solve of the reduced OSC QP (study).

    python tools/gi_model.py [robot] [scenario] [mask] [nenv]

The product's interior point takes 11-19 iterations of a full Newton step each (one 24x24 /
32x32 LDL^T and two triangular solves per iteration).  A dual active-set method (Goldfarb &
Idnani 1983, the algorithm of quadprog) starts from the unconstrained minimum and adds violated
rows one at a time, each add/drop an O(N^2) update of J = L^-T Q and R by Givens rotations.  This
model counts its adds / drops per env and the lockstep maximum over the four envs that share a
wavefront, and checks its torques against the exact oracle.
"""
from __future__ import annotations

import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

from osc_qp import BIG_NUMBER, b_matrix, build_qp, contact_jacobian, load_model, torque  # noqa: E402


def reduced_qp(model, M, C, J, b, T, mask):
    """min 1/2 y'Hr y + g'y s.t. G y <= h over y = (u, z of the contacts in touch); dv = X [y; 1]."""
    qp = build_qp(model, M, C, J, b, T, mask)
    nv, nu, nc = model.nv, model.nu, model.nc
    H_dv, f_dv = qp.H[:nv, :nv], qp.f[:nv]
    Jc = contact_jacobian(model, J)
    live = [k for k in range(nc) if mask[k] != 0.0]
    zcols = [3 * k + c for k in live for c in range(3)]
    Bm = np.hstack([b_matrix(model), Jc[:, zcols]])
    X = np.linalg.solve(M, Bm)
    x0 = np.linalg.solve(M, -np.asarray(C))
    ny = nu + len(zcols)
    Hr = X.T @ H_dv @ X
    Hr[np.arange(nu), np.arange(nu)] += 2 * (model.w_torque + model.w_reg)
    Hr[np.arange(nu, ny), np.arange(nu, ny)] += 2 * model.w_reg
    g = X.T @ (H_dv @ x0 + f_dv)
    rows, h = [], []
    for q in range(nu):
        e = np.zeros(ny); e[q] = 1.0
        rows += [e, -e]; h += [model.u_ub[q], -model.u_lb[q]]
    for i, k in enumerate(live):
        c0 = nu + 3 * i
        for sx, sy in ((1, 1), (-1, 1), (1, -1), (-1, -1)):
            r = np.zeros(ny); r[c0], r[c0 + 1], r[c0 + 2] = sx, sy, -model.mu
            rows.append(r); h.append(0.0)
        r = np.zeros(ny); r[c0 + 2] = -1.0; rows.append(r); h.append(0.0)
        r = np.zeros(ny); r[c0 + 2] = 1.0; rows.append(r); h.append(BIG_NUMBER * mask[k])
    return Hr, g, np.array(rows), np.array(h), X, x0, live


def givens(a, b):
    if b == 0.0:
        return 1.0, 0.0, a
    r = np.hypot(a, b)
    return a / r, b / r, r


def gi_solve(Hr, g, G, h, tol=1e-12, max_it=200):
    """Goldfarb-Idnani on  min 1/2 y'Hr y + g'y  s.t.  G y <= h  (rows as n'y >= b with n = -G_p,
    b = -h_p).  Returns y, the active rows, and the number of adds / drops."""
    N = Hr.shape[0]
    L = np.linalg.cholesky(Hr)
    Jm = np.linalg.inv(L).T                   # J = L^-T
    y = -np.linalg.solve(Hr, g)
    A: list[int] = []
    u = np.zeros(0)
    R = np.zeros((N, N))
    adds = drops = 0
    scale = 1.0 + np.abs(h[np.abs(h) < 1e20]).max() if len(h) else 1.0
    for _ in range(max_it):
        s = h - G @ y                          # slack: >= 0 feasible
        s[A] = np.inf
        p = int(np.argmin(s))
        if s[p] >= -tol * scale:
            return y, A, adds, drops
        n = -G[p]
        up = 0.0
        while True:
            q = len(A)
            d = Jm.T @ n
            z = Jm[:, q:] @ d[q:]
            r = np.linalg.solve(R[:q, :q], d[:q]) if q else np.zeros(0)
            t1, k = np.inf, -1
            for j in range(q):
                if r[j] > 0 and u[j] / r[j] < t1:
                    t1, k = u[j] / r[j], j
            zn = z @ n
            t2 = (-(n @ y - (-h[p])) / zn) if abs(zn) > 1e-14 * (1 + np.abs(z).max()) else np.inf
            t = min(t1, t2)
            if not np.isfinite(t):
                raise RuntimeError("infeasible")
            if t2 == np.inf:                       # dependent row: dual step, drop k
                u = u - t * r
                up += t
            else:
                y = y + t * z
                u = u - t * r
                up += t
                if t == t2:                        # add p
                    for j in range(N - 1, q, -1):  # zero d[j] into d[j-1]
                        c, sn, rr = givens(d[j - 1], d[j])
                        d[j - 1], d[j] = rr, 0.0
                        Jj1, Jj = Jm[:, j - 1].copy(), Jm[:, j].copy()
                        Jm[:, j - 1] = c * Jj1 + sn * Jj
                        Jm[:, j] = -sn * Jj1 + c * Jj
                    R[:q + 1, q] = d[:q + 1]
                    A.append(p)
                    u = np.append(u, up)
                    adds += 1
                    break
            # drop constraint k: remove column k of R, retriangularise by rotations
            A.pop(k)
            u = np.delete(u, k)
            R[:q, k:q - 1] = R[:q, k + 1:q].copy()
            R[:, q - 1] = 0.0
            for j in range(k, q - 1):
                c, sn, rr = givens(R[j, j], R[j + 1, j])
                Rj, Rj1 = R[j, j:q - 1].copy(), R[j + 1, j:q - 1].copy()
                R[j, j:q - 1] = c * Rj + sn * Rj1
                R[j + 1, j:q - 1] = -sn * Rj + c * Rj1
                Jj, Jj1 = Jm[:, j].copy(), Jm[:, j + 1].copy()
                Jm[:, j] = c * Jj + sn * Jj1
                Jm[:, j + 1] = -sn * Jj + c * Jj1
            R[q - 1, :] = 0.0
            drops += 1
            if t2 == np.inf and t == t1:
                continue
    raise RuntimeError("GI did not converge")


def main():
    from osc_amd.synth import SEED_BASE, generate
    from qp_exact import solve_exact
    robot = sys.argv[1] if len(sys.argv) > 1 else "unitree_go2"
    scen = sys.argv[2] if len(sys.argv) > 2 else "standing"
    mm = sys.argv[3] if len(sys.argv) > 3 else "ones"
    nenv = int(sys.argv[4]) if len(sys.argv) > 4 else 256
    model = load_model(robot)
    d = generate(robot, nenv, SEED_BASE + 2, scen, mm)
    its, errs = [], []
    for e in range(nenv):
        args = [d[k][e] for k in ("M", "C", "J", "b", "T", "mask")]
        Hr, g, G, h, X, x0, live = reduced_qp(model, *args)
        y, A, a_, d_ = gi_solve(Hr, g, G, h)
        its.append(a_ + d_)
        if e < 32:
            ref = torque(model, solve_exact(model, build_qp(model, *args), *args[:3]).x)
            errs.append(np.abs(y[:model.nu] - ref).max() / max(np.abs(ref).max(), 1.0))
    its = np.array(its)
    lock = its.reshape(-1, 4).max(axis=1)
    print(f"{robot} {scen} {mm}: adds+drops mean {its.mean():.2f} max {its.max()}  "
          f"lockstep(4) mean {lock.mean():.2f} max {lock.max()}  torque err max {max(errs):.2e}")


if __name__ == "__main__":
    main()
