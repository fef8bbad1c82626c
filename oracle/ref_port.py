"""ctypes wrapper of oracle/osc_ref_port.c (CPU restatement of the reference's per-tick path:
CasADi-equivalent assembly + OSQP 0.6.3 ADMM, warm-started tick to tick).

TEST / BENCH INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg ("port") and oracle cross-checks.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from osc_qp import load_model, task_weights

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "build", "libosc_ref_port.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise ImportError(f"{LIB} missing: run `make -C oracle`")
        L = ctypes.CDLL(LIB)
        dp = ctypes.POINTER(ctypes.c_double)
        L.osc_cpu_create.argtypes = [ctypes.c_int] * 4 + [dp, ctypes.c_double, ctypes.c_double,
                                                          ctypes.c_double, dp, dp, ctypes.c_int]
        L.osc_cpu_create.restype = ctypes.c_void_p
        L.osc_cpu_destroy.argtypes = [ctypes.c_void_p]
        L.osc_cpu_step.argtypes = [ctypes.c_void_p] + [dp] * 8
        L.osc_cpu_step.restype = ctypes.c_int
        L.osc_cpu_set_tolerances.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_double,
                                             ctypes.c_int]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


class RefPort:
    """One reference controller instance (one environment, warm-started across ticks)."""

    def __init__(self, robot: str, adaptive_rho_interval: int = 25):
        self.model = m = load_model(robot)
        self._w = np.ascontiguousarray(task_weights(m))
        self._h = lib().osc_cpu_create(m.nv, m.nu, m.nc, m.ns, _p(self._w), m.w_torque, m.w_reg,
                                       m.mu, _p(np.ascontiguousarray(m.u_lb)),
                                       _p(np.ascontiguousarray(m.u_ub)), adaptive_rho_interval)
        self.tau = np.zeros(m.nu)
        self.x = np.zeros(m.n)

    def set_tolerances(self, eps_abs: float, eps_rel: float, max_iter: int):
        lib().osc_cpu_set_tolerances(self._h, eps_abs, eps_rel, max_iter)

    def step(self, M, C, J, b, T, mask, want_x=False):
        arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (M, C, J, b, T, mask)]
        it = lib().osc_cpu_step(self._h, *[_p(a) for a in arrs], _p(self.tau),
                                _p(self.x) if want_x else None)
        return self.tau.copy(), it

    def __del__(self):
        try:
            lib().osc_cpu_destroy(self._h)
        except Exception:
            pass


def timed_ticks(robot: str, seconds: float, seed: int) -> dict:
    """bench.py cpu_baseline worker: ONE environment ticking through a 64-tick 1 % random walk
    of its inputs (warm-started, no 500 Hz sleep) for `seconds` on the calling core."""
    import sys
    import time
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "operational-space-control_amd"))
    from osc_amd.synth import SEED_BASE, generate, random_walk
    rng = np.random.default_rng(SEED_BASE + seed)
    d = generate(robot, 1, SEED_BASE + 1 + seed, "standing", "ones")
    ticks = [d]
    for _ in range(63):
        ticks.append(random_walk(ticks[-1], rng))
    inputs = [[t[k][0] for k in ("M", "C", "J", "b", "T", "mask")] for t in ticks]
    port = RefPort(robot)
    for a in inputs[:4]:
        port.step(*a)
    n, iters, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        _, it = port.step(*inputs[n % len(inputs)])
        iters += it
        n += 1
    return {"ticks": n, "admm_iters": iters, "seconds": time.perf_counter() - t0}


if __name__ == "__main__":
    import argparse
    import json
    ap = argparse.ArgumentParser()
    ap.add_argument("--robot", default="unitree_go2")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    print(json.dumps(timed_ticks(a.robot, a.seconds, a.seed)), flush=True)
