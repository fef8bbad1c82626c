"""Host-fed batched control tick (include/osc_host_feed.h).

Every tick's inputs start in pinned host memory -- where the reference's control loop finds the
State and task targets the simulation thread wrote (unitree_go2/operational_space_controller.h:
546-573) -- cross PCIe in one copy, are solved on the GPU, and the torques come back.  Tick k's
copy overlaps tick k-1's solve (depth 2).  Two input forms: the post-kinematics QP inputs
(M, C, J, b, T, mask) or joint states (qpos, qvel, T, mask) through the GPU kinematics.

    feed = HostFeed(solver, nenv, form="qp", depth=2, warm=False)
    feed.inputs(k)["M"][:] = ...      # numpy views of the pinned slot of tick k
    feed.submit(k)
    tau, status, iters = feed.wait(k)  # numpy views of the pinned outputs (valid until k + depth)
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib


class HostFeed:
    def __init__(self, solver, nenv: int, form: str = "qp", depth: int = 2, warm: bool = False,
                 kin=None):
        """solver: an OSCBatchSolver (its model and device); kin: a KinematicsBatch for
        form="joint_states" (the same robot)."""
        import torch
        self.solver, self.nenv, self.form, self.depth = solver, nenv, form, depth
        d = solver.dims
        self.nu, self.nv, self.ns, self.nc = d["nu"], d["nv"], d["ns"], d["nc"]
        self.nq = kin.nq if kin is not None else None
        f = {"qp": _lib.FEED_QP, "joint_states": _lib.FEED_JOINT_STATES}[form]
        h = ctypes.c_void_p()
        with torch.cuda.device(solver.device):
            rc = _lib.lib().osc_host_feed_create(solver._h, kin._h if kin is not None else None,
                                                 nenv, f, _lib.FEED_WARM if warm else 0, depth,
                                                 ctypes.byref(h))
        if rc != 0:
            raise _lib.OSCError("osc_host_feed_create", rc)
        self._h = h
        self._kin = kin   # (kept alive: the feed holds its handle)
        self.next = 0
        self.in_bytes = 0
        self.out_bytes = 0

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.lib().osc_host_feed_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _view(addr, shape, dtype=np.float64):
        n = int(np.prod(shape))
        ct = ctypes.c_double if dtype == np.float64 else ctypes.c_int32
        return np.ctypeslib.as_array((ct * n).from_address(addr)).reshape(shape)

    def inputs(self, tick: int) -> dict:
        """Numpy views of tick `tick`'s pinned input slot (blocks until the slot is free)."""
        s = _lib.OscFeedInputs()
        rc = _lib.lib().osc_host_feed_inputs(self._h, tick, ctypes.byref(s))
        if rc != 0:
            raise _lib.OSCError("osc_host_feed_inputs", rc)
        self.in_bytes = s.bytes
        n = self.nenv
        out = {"T": self._view(s.T, (n, self.ns, 6)),
               "mask": self._view(s.contact_mask, (n, self.nc))}
        if self.form == "qp":
            out.update(M=self._view(s.M, (n, self.nv, self.nv)), C=self._view(s.C, (n, self.nv)),
                       J=self._view(s.J, (n, 6 * self.ns, self.nv)),
                       b=self._view(s.b, (n, 6 * self.ns)))
        else:
            out.update(qpos=self._view(s.qpos, (n, self.nq)), qvel=self._view(s.qvel, (n, self.nv)))
        return out

    def submit(self, tick: int) -> None:
        rc = _lib.lib().osc_host_feed_submit(self._h, tick)
        if rc != 0:
            raise _lib.OSCError("osc_host_feed_submit", rc)
        self.next = tick + 1

    def wait(self, tick: int):
        """(tau, status, iters) numpy views of tick `tick`'s pinned outputs."""
        o = _lib.OscFeedOutputs()
        rc = _lib.lib().osc_host_feed_wait(self._h, tick, ctypes.byref(o))
        if rc != 0:
            raise _lib.OSCError("osc_host_feed_wait", rc)
        self.out_bytes = o.bytes
        n = self.nenv
        return (self._view(o.tau, (n, self.nu)), self._view(o.status, (n,), np.int32),
                self._view(o.iters, (n,), np.int32))

    def timing(self, tick: int) -> dict:
        t = _lib.OscFeedTiming()
        rc = _lib.lib().osc_host_feed_timing(self._h, tick, ctypes.byref(t))
        if rc != 0:
            raise _lib.OSCError("osc_host_feed_timing", rc)
        return {"h2d_ms": t.h2d_ms, "solve_ms": t.solve_ms, "d2h_ms": t.d2h_ms,
                "kin_ms": t.kin_ms, "latency_ms": t.h2d_start_to_d2h_end_ms}
