"""Host-side batched OSC solver: the reference's per-tick QP for a whole batch of environments.

Reference interface this mirrors (paths relative to the reference's operational-space-control/):
  * OperationalSpaceController(xml_path, control_rate_us, OsqpSettings)   osc.h:108
      -> OSCBatchSolver(robot, yaml_path, eps_mu, max_iter)   (model from the same YAML schema)
  * update_optimization_data() + update_optimization() + solve_optimization()  osc.h:457-536
      -> OSCBatchSolver.solve(M, C, J, b, T, mask)          (all environments in one launch)
  * get_torque_command() -> tau;  get_solution() -> x        osc.h:230-238
  * OsqpSolver::dual_solution -> y (want_y)                  osc.h:534-535
  * wheel no-slip rows (walter_sr_wheels/autogen/autogen.py:128-240, commented out upstream):
    a model whose YAML switches them on takes the per-env wheel directions (wheel_dir)
  * absl::Status error convention -> OSCError with the osc_status code.

Inputs are torch float64 CUDA tensors already resident in HBM (numpy arrays are copied to the
current device for convenience).  Everything is launched through the C-ABI
(include/osc_batch.h) on the current torch stream.
"""
from __future__ import annotations

import ctypes
import dataclasses

import numpy as np
import torch

from . import _lib
from .robots import config_path, dims


@dataclasses.dataclass
class SolveResult:
    tau: torch.Tensor          # (nenv, nu)
    x: torch.Tensor | None     # (nenv, nv + nu + 3nc) design vector (dv, u, z)
    status: torch.Tensor       # (nenv,) int32, 0 = converged
    iters: torch.Tensor        # (nenv,) int32, interior-point iterations
    workspace: torch.Tensor | None = None   # device scratch (reduced QP per env)
    y: torch.Tensor | None = None           # (nenv, dual_rows) dual solution (OSQP convention)


class OSCBatchSolver:
    def __init__(self, robot: str, yaml_path: str | None = None, eps_mu: float | None = None,
                 max_iter: int | None = None, device: torch.device | int | None = None,
                 tuning: dict | None = None):
        """tuning: fields of osc_model_tuning (include/osc_batch.h) to change from the model's
        defaults, e.g. {"small_batch_max": 0} (solver policy only, never the QP)."""
        if not torch.cuda.is_available():
            raise RuntimeError("OSCBatchSolver needs a HIP device (no CPU fallback exists)")
        self.robot = robot
        self.dims = dims(robot)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else
                                   torch.device(device).index or 0)
        desc = _lib.desc_from_yaml(robot, yaml_path or config_path(robot))
        if eps_mu is not None:
            desc.eps_mu = float(eps_mu)
        if max_iter is not None:
            desc.max_iter = int(max_iter)
        self.desc = desc
        self.wheels = desc.wheel_rows != 0
        tune = _lib.OscModelTuning()
        rc = _lib.lib().osc_model_tuning_defaults(ctypes.byref(desc), ctypes.byref(tune))
        if rc != 0:
            raise _lib.OSCError("osc_model_tuning_defaults", rc)
        for k, v in (tuning or {}).items():
            if k not in dict(_lib.OscModelTuning._fields_):
                raise KeyError(f"osc_model_tuning has no field {k!r}")
            setattr(tune, k, v)
        self.tuning = tune
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            rc = _lib.lib().osc_model_create_tuned(ctypes.byref(desc), ctypes.byref(tune),
                                                   ctypes.byref(h))
        if rc != 0:
            raise _lib.OSCError("osc_model_create", rc)
        self._h = h
        rows = ctypes.c_int32()
        _lib.lib().osc_dual_rows(self._h, ctypes.byref(rows))
        self.dual_rows = rows.value

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.lib().osc_model_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _as_dev(self, a, shape, name):
        if isinstance(a, np.ndarray):
            a = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64))
        if not isinstance(a, torch.Tensor):
            raise TypeError(f"{name}: expected torch.Tensor or numpy array")
        a = a.to(device=self.device, dtype=torch.float64).contiguous()
        if tuple(a.shape) != shape:
            raise ValueError(f"{name}: expected shape {shape}, got {tuple(a.shape)}")
        return a

    def alloc_outputs(self, nenv: int, want_x: bool = False, want_y: bool = False):
        d = self.dims
        opts = dict(device=self.device)
        tau = torch.empty((nenv, d["nu"]), dtype=torch.float64, **opts)
        x = torch.empty((nenv, d["n"]), dtype=torch.float64, **opts) if (want_x or want_y) else None
        y = torch.empty((nenv, self.dual_rows), dtype=torch.float64, **opts) if want_y else None
        status = torch.empty((nenv,), dtype=torch.int32, **opts)
        iters = torch.empty((nenv,), dtype=torch.int32, **opts)
        nb = ctypes.c_size_t()
        rc = _lib.lib().osc_workspace_bytes(self._h, nenv, ctypes.byref(nb))
        if rc != 0:
            raise _lib.OSCError("osc_workspace_bytes", rc)
        ws = torch.empty((max(nb.value // 8, 2),), dtype=torch.float64, **opts)
        return SolveResult(tau, x, status, iters, ws, y)

    def solve_into(self, out: SolveResult, M, C, J, b, T, mask, stream=None,
                   wheel_dir=None) -> SolveResult:
        """Launch only (no allocation, no host sync): the benchmarked call.  osc_batch_solve, or
        osc_batch_solve_ex when the model has wheel rows or duals are wanted (out.y)."""
        nenv = out.tau.shape[0]
        s = (torch.cuda.current_stream(self.device) if stream is None else stream).cuda_stream
        ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
        wsb = ctypes.c_size_t(0 if out.workspace is None else out.workspace.numel() * 8)
        if wheel_dir is None and out.y is None:
            rc = _lib.lib().osc_batch_solve(self._h, nenv, ptr(M), ptr(C), ptr(J), ptr(b), ptr(T),
                                            ptr(mask), ptr(out.tau), ptr(out.x), ptr(out.status),
                                            ptr(out.iters), ptr(out.workspace), wsb,
                                            ctypes.c_void_p(s))
            if rc != 0:
                raise _lib.OSCError("osc_batch_solve", rc)
            return out
        ex = _lib.OscSolveExtras(wheel_dir.data_ptr() if wheel_dir is not None else None,
                                 out.y.data_ptr() if out.y is not None else None)
        rc = _lib.lib().osc_batch_solve_ex(self._h, nenv, ptr(M), ptr(C), ptr(J), ptr(b), ptr(T),
                                           ptr(mask), ctypes.byref(ex), ptr(out.tau), ptr(out.x),
                                           ptr(out.status), ptr(out.iters), ptr(out.workspace), wsb,
                                           ctypes.c_void_p(s))
        if rc != 0:
            raise _lib.OSCError("osc_batch_solve_ex", rc)
        return out

    def assemble_into(self, out: SolveResult, M, C, J, b, T, mask, stream=None,
                      wheel_dir=None) -> SolveResult:
        """First half of solve_into: every env's reduced QP into out.workspace."""
        nenv = out.tau.shape[0]
        s = (torch.cuda.current_stream(self.device) if stream is None else stream).cuda_stream
        ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
        wsb = ctypes.c_size_t(out.workspace.numel() * 8)
        if wheel_dir is None:
            rc = _lib.lib().osc_batch_assemble(self._h, nenv, ptr(M), ptr(C), ptr(J), ptr(b),
                                               ptr(T), ptr(mask), ptr(out.workspace), wsb,
                                               ctypes.c_void_p(s))
        else:
            rc = _lib.lib().osc_batch_assemble_ex(self._h, nenv, ptr(M), ptr(C), ptr(J), ptr(b),
                                                  ptr(T), ptr(mask), ptr(wheel_dir),
                                                  ptr(out.workspace), wsb, ctypes.c_void_p(s))
        if rc != 0:
            raise _lib.OSCError("osc_batch_assemble", rc)
        return out

    def solve_assembled_into(self, out: SolveResult, mask, stream=None) -> SolveResult:
        """Second half of solve_into: interior-point solve of the assembled workspace."""
        nenv = out.tau.shape[0]
        s = (torch.cuda.current_stream(self.device) if stream is None else stream).cuda_stream
        ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
        rc = _lib.lib().osc_batch_solve_assembled(self._h, nenv, ptr(mask), ptr(out.tau),
                                                  ptr(out.x), ptr(out.status), ptr(out.iters),
                                                  ptr(out.workspace),
                                                  ctypes.c_size_t(out.workspace.numel() * 8),
                                                  ctypes.c_void_p(s))
        if rc != 0:
            raise _lib.OSCError("osc_batch_solve_assembled", rc)
        return out

    def alloc_warm_state(self, nenv: int) -> torch.Tensor:
        """Zero-filled warm state (osc_warm_state_bytes): every env starts cold on its first tick."""
        nb = ctypes.c_size_t()
        rc = _lib.lib().osc_warm_state_bytes(self._h, nenv, ctypes.byref(nb))
        if rc != 0:
            raise _lib.OSCError("osc_warm_state_bytes", rc)
        return torch.zeros((max(nb.value // 8, 2),), dtype=torch.float64, device=self.device)

    def solve_warm_into(self, out: SolveResult, warm: torch.Tensor, M, C, J, b, T, mask,
                        stream=None, wheel_dir=None) -> SolveResult:
        """osc_batch_solve_warm: as solve_into, starting from (and updating) `warm`, the previous
        tick's solution (the reference's SetWarmStart, operational_space_controller.h:519-526);
        osc_batch_solve_warm_ex with wheel rows or duals (out.y)."""
        nenv = out.tau.shape[0]
        s = (torch.cuda.current_stream(self.device) if stream is None else stream).cuda_stream
        ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
        if wheel_dir is not None or out.y is not None:
            ex = _lib.OscSolveExtras(wheel_dir.data_ptr() if wheel_dir is not None else None,
                                     out.y.data_ptr() if out.y is not None else None)
            rc = _lib.lib().osc_batch_solve_warm_ex(
                self._h, nenv, ptr(M), ptr(C), ptr(J), ptr(b), ptr(T), ptr(mask),
                ctypes.byref(ex), ptr(out.tau), ptr(out.x), ptr(out.status), ptr(out.iters),
                ptr(warm), ctypes.c_size_t(warm.numel() * 8), ptr(out.workspace),
                ctypes.c_size_t(0 if out.workspace is None else out.workspace.numel() * 8),
                ctypes.c_void_p(s))
            if rc != 0:
                raise _lib.OSCError("osc_batch_solve_warm_ex", rc)
            return out
        rc = _lib.lib().osc_batch_solve_warm(self._h, nenv, ptr(M), ptr(C), ptr(J), ptr(b), ptr(T),
                                             ptr(mask), ptr(out.tau), ptr(out.x), ptr(out.status),
                                             ptr(out.iters), ptr(warm),
                                             ctypes.c_size_t(0 if warm is None else warm.numel() * 8),
                                             ptr(out.workspace),
                                             ctypes.c_size_t(0 if out.workspace is None else
                                                             out.workspace.numel() * 8),
                                             ctypes.c_void_p(s))
        if rc != 0:
            raise _lib.OSCError("osc_batch_solve_warm", rc)
        return out

    def solve_assembled_warm_into(self, out: SolveResult, warm: torch.Tensor, mask,
                                  stream=None) -> SolveResult:
        nenv = out.tau.shape[0]
        s = (torch.cuda.current_stream(self.device) if stream is None else stream).cuda_stream
        ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
        rc = _lib.lib().osc_batch_solve_assembled_warm(
            self._h, nenv, ptr(mask), ptr(out.tau), ptr(out.x), ptr(out.status), ptr(out.iters),
            ptr(warm), ctypes.c_size_t(0 if warm is None else warm.numel() * 8),
            ptr(out.workspace), ctypes.c_size_t(out.workspace.numel() * 8),
            ctypes.c_void_p(s))
        if rc != 0:
            raise _lib.OSCError("osc_batch_solve_assembled_warm", rc)
        return out

    def prepare(self, M, C, J, b, T, mask):
        d = self.dims
        nenv = int(M.shape[0])
        return (self._as_dev(M, (nenv, d["nv"], d["nv"]), "M"),
                self._as_dev(C, (nenv, d["nv"]), "C"),
                self._as_dev(J, (nenv, d["s"], d["nv"]), "J"),
                self._as_dev(b, (nenv, d["s"]), "b"),
                self._as_dev(T, (nenv, d["ns"], 6), "T"),
                self._as_dev(mask, (nenv, d["nc"]), "mask"))

    def solve(self, M, C, J, b, T, mask, want_x: bool = False, want_y: bool = False,
              wheel_dir=None) -> SolveResult:
        args = self.prepare(M, C, J, b, T, mask)
        nenv = int(args[0].shape[0])
        if wheel_dir is not None:
            wheel_dir = self._as_dev(wheel_dir, (nenv, self.dims["nc"], 6), "wheel_dir")
        out = self.alloc_outputs(nenv, want_x, want_y)
        with torch.cuda.device(self.device):
            return self.solve_into(out, *args, wheel_dir=wheel_dir)


def solve_multi_into(jobs, stream=None) -> None:
    """osc_batch_solve_multi: several models' batches in one call on one stream (BASELINE
    configs[4]: Go2 + WaLTER Sr per GPU).  `jobs` = [(solver, SolveResult, (M, C, J, b, T,
    mask)[, wheel_dir]), ...] with device tensors from solver.prepare / solver.alloc_outputs
    (wheel_dir: the wheel-row models' directions, [nenv, nc, 6])."""
    arr = (_lib.OscBatchJob * len(jobs))()
    ptr = lambda t: t.data_ptr() if t is not None else None
    dev = None
    for j, job in zip(arr, jobs):
        solver, out, inputs = job[:3]
        j.wheel_dir = ptr(job[3]) if len(job) > 3 else None
        M, C, J, b, T, mask = inputs
        j.model = solver._h.value
        j.nenv = out.tau.shape[0]
        j.M, j.C, j.J, j.b, j.T, j.contact_mask = (ptr(t) for t in (M, C, J, b, T, mask))
        j.tau, j.x, j.status, j.iters = ptr(out.tau), ptr(out.x), ptr(out.status), ptr(out.iters)
        j.workspace = ptr(out.workspace)
        j.workspace_bytes = out.workspace.numel() * 8
        dev = solver.device
    s = (torch.cuda.current_stream(dev) if stream is None else stream).cuda_stream
    rc = _lib.lib().osc_batch_solve_multi(arr, len(jobs), ctypes.c_void_p(s))
    if rc != 0:
        raise _lib.OSCError("osc_batch_solve_multi", rc)
