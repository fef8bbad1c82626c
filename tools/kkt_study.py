"""Diagnostic (CPU): the joint-state failure class of the reduced-QP solve.

Joint states as the GPU tests draw them (random_states, joint_range 0.5, random base
orientation), oracle kinematics (oracle/kinematics.py, == the GPU's to 1e-12), the reduced QP in
torque coordinates and the numpy model of the interior point (tools/ipm_model.py), then
candidate refinements compared against the exact optimum (oracle/qp_exact.py).

    python tools/kkt_study.py [nenv] [joint_range] [seed_offset]
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tools"))
import numpy as np  # noqa: E402

import kinematics as okin  # noqa: E402
from ipm_model import ipm, reduce_qp_tau  # noqa: E402
from osc_amd.dist import shard_seed  # noqa: E402
from osc_amd.kinematics import load_tree, random_states  # noqa: E402
from osc_amd.synth import generate  # noqa: E402
from osc_qp import build_qp, load_model, torque  # noqa: E402
from qp_exact import solve_exact  # noqa: E402


def main():
    nenv = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    jr = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
    so = int(sys.argv[3]) if len(sys.argv) > 3 else 7
    robot = "unitree_go2"
    seed = shard_seed(0) + so
    km = okin.load(robot)
    tree = load_tree(robot)
    qpos, qvel = random_states(tree, nenv, seed, joint_range=jr)
    d = generate(robot, nenv, seed, "standing", "ones")
    model = load_model(robot)
    t0 = time.time()
    stats = []
    for e in range(nenv):
        M, C, J, b = okin.kinematics(km, qpos[e], qvel[e])
        args = (M, C, J, b, d["T"][e], d["mask"][e])
        Hr, g, G, h, P, p0 = reduce_qp_tau(model, *args)
        y, it, st = ipm(Hr, g, G, h, eps_mu=1e-9, max_iter=50)[:3]
        ex = solve_exact(model, build_qp(model, *args), M, C, J)
        ref = torque(model, ex.x)
        tau = y[:model.nu]
        err = np.abs(tau - ref).max() / max(np.abs(ref).max(), 1.0)
        ev = np.linalg.eigvalsh(Hr)
        evm = np.linalg.eigvalsh(M)
        stats.append((e, err, ev[-1] / ev[0], evm[-1] / evm[0], evm[0]))
    stats = np.array(stats)
    print(f"{nenv} envs in {time.time() - t0:.1f}s")
    bad = stats[stats[:, 1] > 1e-5]
    print(f"ipm err > 1e-5: {len(bad)}")
    for row in bad[np.argsort(-bad[:, 1])][:30]:
        print("env %5d err %.2e cond(Hr) %.2e cond(M) %.2e minEig(M) %.2e" % tuple(row))
    print("cond(Hr) percentiles", np.percentile(stats[:, 2], [50, 90, 99, 100]))


if __name__ == "__main__":
    main()


def detail(nenv=512, jr=0.5, so=7, envs=None):
    """Per failing env: the interior point's active set (lambda > s) vs the exact optimum's, and
    the exact reduced KKT solve on each."""
    import ipm_model
    robot = "unitree_go2"
    seed = shard_seed(0) + so
    km = okin.load(robot)
    qpos, qvel = random_states(load_tree(robot), nenv, seed, joint_range=jr)
    d = generate(robot, nenv, seed, "standing", "ones")
    model = load_model(robot)
    for e in envs:
        M, C, J, b = okin.kinematics(km, qpos[e], qvel[e])
        args = (M, C, J, b, d["T"][e], d["mask"][e])
        Hr, g, G, h, P, p0 = reduce_qp_tau(model, *args)
        y, it, st = ipm(Hr, g, G, h, eps_mu=1e-9, max_iter=50)[:3]
        s, lam = ipm_model.FINAL["s"], ipm_model.FINAL["lam"]
        ex = solve_exact(model, build_qp(model, *args), M, C, J)
        ys = np.concatenate([ex.x[model.nv:model.nv + model.nu], ex.x[model.nv + model.nu:]])
        sl = h - G @ ys
        act_ex = sl < 1e-9 * (1 + np.abs(h))
        act_ipm = lam > s
        print(f"env {e} it {it} |y-y*| {np.abs(y - ys).max():.2e} exact active {np.nonzero(act_ex)[0]}"
              f" ipm active {np.nonzero(act_ipm)[0]}")
        for name, A in (("ipm", act_ipm), ("exact", act_ex)):
            GA = G[A]
            nA = GA.shape[0]
            K = np.block([[Hr, GA.T], [GA, np.zeros((nA, nA))]])
            sol = np.linalg.lstsq(K, np.concatenate([-g, h[A]]), rcond=None)[0]
            yk = sol[:len(g)]
            print(f"   KKT on {name} set: |y-y*| {np.abs(yk - ys).max():.2e} "
                  f"maxviol {max((G @ yk - h).max(), 0):.2e} minmult {sol[len(g):].min() if nA else 0:.2e}")
        print("   s,lam on rows where they differ:",
              [(int(i), f"{s[i]:.1e}", f"{lam[i]:.1e}", f"{sl[i]:.1e}") for i in np.nonzero(act_ex != act_ipm)[0]])


def refine_sim(nenv=512, jr=0.5, so=7, envs=None, pens=(1e2, 1e4, 1e6), steps=12):
    """The kernel's refinement (method of multipliers on the active set, residual in factored
    form, one LDL^T of Hr + D G_A'G_A) run for `steps` steps without a restart: error per step."""
    import ipm_model
    from ipm_model import ldl_factor, ldl_solve
    robot = "unitree_go2"
    seed = shard_seed(0) + so
    km = okin.load(robot)
    qpos, qvel = random_states(load_tree(robot), nenv, seed, joint_range=jr)
    d = generate(robot, nenv, seed, "standing", "ones")
    model = load_model(robot)
    nv, nu = model.nv, model.nu
    for e in envs:
        M, C, J, b = okin.kinematics(km, qpos[e], qvel[e])
        args = (M, C, J, b, d["T"][e], d["mask"][e])
        qp = build_qp(model, *args)
        Hr, g, G, h, P, p0 = reduce_qp_tau(model, *args)
        y, it, st = ipm(Hr, g, G, h, eps_mu=1e-9, max_iter=50)[:3]
        s, lam = ipm_model.FINAL["s"], ipm_model.FINAL["lam"]
        ex = solve_exact(model, build_qp(model, *args), M, C, J)
        ys = np.concatenate([ex.x[nv:nv + nu], ex.x[nv + nu:]])
        X, x0 = P[:nv], p0[:nv]
        Hd, fd = qp.H[:nv, :nv], qp.f[:nv]
        wdiag = np.diag(qp.H)[nv:]
        A = lam > s
        GA, hA = G[A], h[A]

        def resid(yv, mu):
            return X.T @ (Hd @ (X @ yv + x0) + fd) + wdiag * yv + GA.T @ mu
        out = [f"env {e} e0 {np.abs(y - ys).max():.1e}"]
        for c in pens:
            Dp = c * np.abs(np.diag(Hr)).max()
            F = ldl_factor(Hr + Dp * GA.T @ GA)
            ya, mu = y.copy(), lam[A].copy()
            errs = []
            for k in range(steps):
                r = resid(ya, mu)
                R3 = GA @ ya - hA
                dy = ldl_solve(F, -r - Dp * GA.T @ R3)
                mu = mu + Dp * (GA @ dy + R3)
                ya = ya + dy
                errs.append(np.abs(ya - ys).max())
            out.append(f"D{c:.0e}: " + " ".join(f"{v:.0e}" for v in errs))
        print("\n   ".join(out))


def refine_new(Hr, G, h, resid, y, s, lam, pen=1e2, steps_min=2, steps_max=8, rounds=4,
               restart=True, neg_leave=True, one_change=False):
    """Candidate kernel refinement: method of multipliers on the active set with the factored
    residual, steps until converged, rows added (violated) / removed (negative multiplier) per
    round; accepted on a KKT test instead of a move bound.  Returns (y, ok, info)."""
    from ipm_model import ldl_factor, ldl_solve
    A = lam > s
    Dp = pen * np.abs(np.diag(Hr)).max()
    mu = np.where(A, lam, 0.0)
    ytol = 1e-9 * (1 + np.abs(y).max())
    ya = y.copy()
    info = {"rounds": 0, "steps": 0}
    for rnd in range(rounds):
        info["rounds"] += 1
        if restart:
            ya = y.copy()
        GA = G[A]
        F = ldl_factor(Hr + Dp * GA.T @ GA)
        conv = False
        for k in range(steps_max):
            info["steps"] += 1
            R3 = np.where(A, G @ ya - h, 0.0)
            r = resid(ya) + G.T @ mu
            dy = ldl_solve(F, -r - Dp * G.T @ R3)
            mu = mu + np.where(A, Dp * (G @ dy + R3), 0.0)
            ya = ya + dy
            dl = np.abs(dy).max()
            if k + 1 >= steps_min and dl <= 1e-10 * (1 + np.abs(ya).max()):
                conv = True
                break
        viol = (~A) & (G @ ya - h > ytol)
        mtol = 1e-9 * (1 + np.abs(mu).max())
        neg = A & (mu < -mtol) if neg_leave else np.zeros_like(A)
        if conv and not viol.any() and not neg.any():
            return ya, True, info
        if one_change:   # the most violated row joins, else the most negative multiplier leaves
            if viol.any():
                v = np.where(viol, G @ ya - h, -np.inf)
                viol = np.zeros_like(A)
                viol[np.argmax(v)] = True
                neg = np.zeros_like(A)
            elif neg.any():
                m = np.where(neg, mu, np.inf)
                neg = np.zeros_like(A)
                neg[np.argmin(m)] = True
        A = (A | viol) & ~neg
        mu = np.where(A, mu, 0.0)
    return ya, False, info


def sweep(robot="unitree_go2", nenv=1024, jr=0.5, so=7, synth=False, eps=1e-9, oracle=True, **kw):
    """IPM (numpy model) + refine_new over a joint-state batch: failures and worst error."""
    import ipm_model
    seed = shard_seed(0) + so
    model = load_model(robot)
    nv, nu = model.nv, model.nu
    if synth:
        dd = generate(robot, nenv, seed, *((synth.split(",")) if isinstance(synth, str)
                                            else ("tumbling", "bernoulli")))
    else:
        km = okin.load(robot)
        qpos, qvel = random_states(load_tree(robot), nenv, seed, joint_range=jr)
        dd = generate(robot, nenv, seed, "standing", "ones")
    worst, nfail, nref, steps, rounds, its = 0.0, 0, 0, [], [], []
    t0 = time.time()
    for e in range(nenv):
        if synth:
            M, C, J, b = dd["M"][e], dd["C"][e], dd["J"][e], dd["b"][e]
        else:
            M, C, J, b = okin.kinematics(km, qpos[e], qvel[e])
        args = (M, C, J, b, dd["T"][e], dd["mask"][e])
        qp = build_qp(model, *args)
        Hr, g, G, h, P, p0 = reduce_qp_tau(model, *args)
        y, it, st = ipm(Hr, g, G, h, eps_mu=eps, max_iter=50)[:3]
        its.append(it)
        s, lam = ipm_model.FINAL["s"], ipm_model.FINAL["lam"]
        X, x0 = P[:nv], p0[:nv]
        Hd, fd = qp.H[:nv, :nv], qp.f[:nv]
        wdiag = np.diag(qp.H)[nv:]

        def resid(yv):
            return X.T @ (Hd @ (X @ yv + x0) + fd) + wdiag * yv
        ya, ok, info = refine_new(Hr, G, h, resid, y, s, lam, **kw)
        steps.append(info["steps"]); rounds.append(info["rounds"])
        if not oracle:
            nfail += 0 if ok else 1
            continue
        try:
            ex = solve_exact(model, qp, M, C, J)
        except Exception:
            nref += 1
            continue
        ref = torque(model, ex.x)
        err = np.abs(ya[:nu] - ref).max() / max(np.abs(ref).max(), 1.0)
        if not ok:
            nfail += 1
            print(f"  env {e} not accepted, err {err:.1e}, info {info}")
        else:
            if err > 1e-7:
                print(f"  env {e} ACCEPTED but err {err:.1e} info {info}")
            worst = max(worst, err)
    print(f"{robot} jr {jr} synth {synth}: {nenv} envs {time.time()-t0:.0f}s  fail {nfail}  oracle refused {nref}"
          f"  worst accepted err {worst:.1e}  steps mean {np.mean(steps):.2f} max {max(steps)}"
          f"  rounds max {max(rounds)}  eps {eps:.0e}  ipm it mean {np.mean(its):.2f}"
          f" wave-max mean {np.mean(np.max(np.reshape(its, (-1, 4)), axis=1)):.2f} max {max(its)}"
          f"  wave steps mean {np.mean(np.max(np.reshape(steps, (-1, 4)), axis=1)):.2f}"
          f"  wave cost (it + 0.4 rounds + 0.15 steps) max "
          f"{np.max(np.max(np.reshape(its, (-1, 4)), 1) + 0.4 * np.max(np.reshape(rounds, (-1, 4)), 1) + 0.15 * np.max(np.reshape(steps, (-1, 4)), 1)):.2f}"
          f" p99 {np.percentile(np.max(np.reshape(its, (-1, 4)), 1) + 0.4 * np.max(np.reshape(rounds, (-1, 4)), 1) + 0.15 * np.max(np.reshape(steps, (-1, 4)), 1), 99):.2f}")
