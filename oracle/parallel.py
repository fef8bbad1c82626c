"""CPU oracle, part 3: the exact oracle over a whole batch, spread over the host's cores.

TEST INFRASTRUCTURE ONLY (see oracle/osc_qp.py header; parity unpinned vs reference outputs).
Only tests/ call this: it is how the GPU parity tests compare EVERY env of a BASELINE-size batch
(4,096 envs: configs[1], configs[2] and the joint-state batches) with the exact optimum of the
reference QP (oracle/qp_exact.solve_exact on oracle/osc_qp.build_qp, i.e. the QP of
unitree_go2/autogen/autogen.py:58-319 stacked as operational_space_controller.h:483-497).

At sizes where the full oracle would take minutes (65,536 envs), `seeded_batch` gets the same
exact optimum per env from the GPU's own answer: the rows the GPU's duals mark active are taken as
the working set, the oracle's exact KKT solve on that set (qp_exact._finish: extended-precision
iterative refinement) gives that face's optimum, and the oracle's KKT certificate decides whether
it is THE optimum (the QP is strictly convex: a certified KKT point is the unique optimum).  An env
whose set does not certify goes to the full oracle.  Either way the comparison is against the exact
optimum, never against the GPU's iterate.

Workers are fresh interpreters (multiprocessing "spawn": nothing of the parent's HIP state is
inherited; they import numpy/scipy only), each pinned to one BLAS thread, at most 16 of them (the
GPU box's CPU share).  Go2 takes ~20 ms per env on one core, so 4,096 envs take ~6 s on 16.
"""
from __future__ import annotations

import concurrent.futures as cf
import multiprocessing as mp
import os

import numpy as np

_CHUNK = 64


def default_workers() -> int:
    env = int(os.environ.get("OSC_ORACLE_WORKERS", "0"))
    if env > 0:
        return env
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:   # pragma: no cover
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def _init_worker():
    try:
        from threadpoolctl import threadpool_limits
        threadpool_limits(1)
    except ImportError:   # pragma: no cover
        pass


def _solve_chunk(robot, arrays, wheel=None, wd=None):
    """Worker: exact optimum (design vector x) and certificate of each env of one chunk."""
    from osc_qp import WheelRows, build_qp, load_model
    from qp_exact import certified, solve_exact
    model = load_model(robot)
    M, C, J, b, T, mask = arrays
    rows = None if wheel is None else WheelRows(dof=np.asarray(wheel[0]), radius=np.asarray(wheel[1]))
    xs, certs = [], []
    for e in range(M.shape[0]):
        a = (M[e], C[e], J[e], b[e], T[e], mask[e])
        qp = build_qp(model, *a) if rows is None else build_qp(model, *a, rows, wd[e])
        sol = solve_exact(model, qp, *a[:3])
        if not certified(sol.cert, 1e-8):
            raise RuntimeError(f"oracle solution not certified: {sol.cert}")
        xs.append(sol.x)
        certs.append(max(sol.cert.values()))
    return np.array(xs), np.array(certs)


def solve_batch(robot: str, M, C, J, b, T, mask, envs=None, workers: int | None = None,
                wheel=None, wheel_dir=None):
    """Exact optima of the reference QP for the envs `envs` (default: all) of a batch given as
    numpy arrays (env-major, the C-ABI's layout); `wheel` = (dof, radius) and `wheel_dir`
    (nenv, nc, 6) add the opt-in no-slip rows (walter_sr_wheels/autogen/autogen.py:128-240).
    Returns (x [len(envs), n], worst KKT residual per env)."""
    M, C, J, b, T, mask = (np.ascontiguousarray(a) for a in (M, C, J, b, T, mask))
    envs = np.arange(M.shape[0]) if envs is None else np.asarray(envs)
    chunks = [envs[i:i + _CHUNK] for i in range(0, len(envs), _CHUNK)]
    workers = workers or default_workers()
    ctx = mp.get_context("spawn")
    with cf.ProcessPoolExecutor(max_workers=min(workers, len(chunks)), mp_context=ctx,
                                initializer=_init_worker) as ex:
        futs = [ex.submit(_solve_chunk, robot, tuple(a[c] for a in (M, C, J, b, T, mask)),
                          wheel, None if wheel_dir is None else np.asarray(wheel_dir)[c])
                for c in chunks]
        res = [f.result() for f in futs]
    return np.concatenate([r[0] for r in res]), np.concatenate([r[1] for r in res])


def _seeded_chunk(robot, arrays, ys):
    """Worker: exact optimum of each env from the working set the GPU's duals mark active (rows
    with y_i != 0, on the bound its sign names), certified; full oracle otherwise."""
    from osc_qp import build_qp, load_model
    from qp_exact import _constraints, _finish, certified, solve_exact
    model = load_model(robot)
    M, C, J, b, T, mask = arrays
    xs, seeded = [], []
    for e in range(M.shape[0]):
        a = (M[e], C[e], J[e], b[e], T[e], mask[e])
        qp = build_qp(model, *a)
        eq, ineq = _constraints(qp)
        # active = a multiplier of the right sign above 1e-6 of the one-sided rows' largest: the
        # GPU's duals come from stationarity (osc_dual_kernel) and carry ~1e-9 residues on rows
        # the optimum leaves inactive (u box rows) -- with them the face is the wrong one
        ysc = 1.0 + max([abs(ys[e][i]) for (i, _, _) in ineq] + [0.0])
        W = [j for j, (i, sg, _) in enumerate(ineq) if sg * ys[e][i] > 1e-6 * ysc]
        ok = False
        try:
            sol = _finish(model, qp, eq, ineq, W, 0, 4)
            ok = certified(sol.cert, 1e-9)
        except RuntimeError:
            pass
        if not ok:
            sol = solve_exact(model, qp, *a[:3])
            if not certified(sol.cert, 1e-8):
                raise RuntimeError(f"oracle solution not certified: {sol.cert}")
        xs.append(sol.x)
        seeded.append(ok)
    return np.array(xs), np.array(seeded)


def seeded_batch(robot: str, M, C, J, b, T, mask, y, workers: int | None = None):
    """Exact optima of EVERY env of a batch (reference QP, no wheel rows), working sets seeded by
    the GPU's duals y [nenv, m] (OSQP convention over A = [Aeq; Aineq; I], include/osc_batch.h
    osc_solve_extras.y).  Returns (x [nenv, n], seeded [nenv] bool: the GPU's set certified)."""
    M, C, J, b, T, mask, y = (np.ascontiguousarray(a) for a in (M, C, J, b, T, mask, y))
    nenv = M.shape[0]
    chunk = max(_CHUNK, nenv // (4 * (workers or default_workers())) // _CHUNK * _CHUNK)
    chunks = [np.arange(i, min(i + chunk, nenv)) for i in range(0, nenv, chunk)]
    ctx = mp.get_context("spawn")
    with cf.ProcessPoolExecutor(max_workers=min(workers or default_workers(), len(chunks)),
                                mp_context=ctx, initializer=_init_worker) as ex:
        futs = [ex.submit(_seeded_chunk, robot, tuple(a[c] for a in (M, C, J, b, T, mask)), y[c])
                for c in chunks]
        res = [f.result() for f in futs]
    return np.concatenate([r[0] for r in res]), np.concatenate([r[1] for r in res])
