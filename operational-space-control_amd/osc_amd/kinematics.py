"""Host side of the GPU kinematics front end (include/osc_kinematics.h).

Reference interface this mirrors (paths relative to the reference's operational-space-control/):
  * update_mj_data()   unitree_go2/operational_space_controller.h:350-374
      -> KinematicsBatch.state_to_qpos(...) (qpos = [0,0,0, quat, q_m], qvel = [v, w, qd_m])
  * update_osc_data()  :376-455 (mj_fullM, qfrc_bias, mj_jac / mj_jacDot per site)
      -> KinematicsBatch.compute(qpos, qvel) -> (M, C, J, b, site_xpos), the inputs of
         OSCBatchSolver.solve
  * the whole tick (update_mj_data .. solve_optimization, :546-573)
      -> KinematicsBatch.solve(solver, qpos, qvel, T, mask)   (osc_batch_solve_qpos)
The kinematic tree comes from operational-space-control_amd/config/<robot>_kinematics.json
(illustrative trees: the reference's MJCF files are not vendored) or from any osc_kin_desc.
Launches go through the C-ABI on the current torch stream; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import dataclasses
import json
import os

import numpy as np
import torch

from . import _lib
from .robots import CONFIG_DIR

KIN_ROBOTS = {"unitree_go2": "unitree_go2", "walter_sr": "walter_sr",
              "walter_sr_wheels": "walter_sr"}   # wheels config: same robot, other weights


def kin_json_path(robot: str) -> str:
    return os.path.join(CONFIG_DIR, f"{KIN_ROBOTS.get(robot, robot)}_kinematics.json")


def load_tree(robot: str) -> dict:
    with open(kin_json_path(robot)) as f:
        return json.load(f)


@dataclasses.dataclass
class KinOutputs:
    M: torch.Tensor            # (nenv, nv, nv)
    C: torch.Tensor            # (nenv, nv)
    J: torch.Tensor            # (nenv, 6ns, nv)
    b: torch.Tensor            # (nenv, 6ns)
    site_xpos: torch.Tensor | None = None   # (nenv, ns, 3)


class KinematicsBatch:
    def __init__(self, robot: str | None = None, tree: dict | None = None,
                 device: torch.device | int | None = None):
        if not torch.cuda.is_available():
            raise RuntimeError("KinematicsBatch needs a HIP device (no CPU fallback exists)")
        if tree is None and robot is None:
            raise ValueError("robot or tree required")
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else
                                   torch.device(device).index or 0)
        desc = (_lib.kin_desc_from_dict(tree) if tree is not None else
                _lib.kin_desc_from_json(None, kin_json_path(robot)))
        self.desc = desc
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            rc = _lib.lib().osc_kin_model_create(ctypes.byref(desc), ctypes.byref(h))
        if rc != 0:
            raise _lib.OSCError("osc_kin_model_create", rc)
        self._h = h
        nq, nv, ns = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        _lib.lib().osc_kin_model_dims(h, ctypes.byref(nq), ctypes.byref(nv), ctypes.byref(ns))
        self.nq, self.nv, self.ns = nq.value, nv.value, ns.value

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.lib().osc_kin_model_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _dev(self, a, shape, name):
        if isinstance(a, np.ndarray):
            a = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64))
        a = a.to(device=self.device, dtype=torch.float64).contiguous()
        if tuple(a.shape) != tuple(shape):
            raise ValueError(f"{name}: expected shape {tuple(shape)}, got {tuple(a.shape)}")
        return a

    @staticmethod
    def _stream(stream, device):
        return (torch.cuda.current_stream(device) if stream is None else stream).cuda_stream

    def alloc(self, nenv: int, want_sites: bool = False) -> KinOutputs:
        o = dict(device=self.device, dtype=torch.float64)
        nv, s = self.nv, 6 * self.ns
        return KinOutputs(torch.empty((nenv, nv, nv), **o), torch.empty((nenv, nv), **o),
                          torch.empty((nenv, s, nv), **o), torch.empty((nenv, s), **o),
                          torch.empty((nenv, self.ns, 3), **o) if want_sites else None)

    def compute_into(self, out: KinOutputs, qpos, qvel, stream=None) -> KinOutputs:
        nenv = out.M.shape[0]
        ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
        rc = _lib.lib().osc_batch_kinematics(self._h, nenv, ptr(qpos), ptr(qvel), ptr(out.M),
                                             ptr(out.C), ptr(out.J), ptr(out.b),
                                             ptr(out.site_xpos),
                                             ctypes.c_void_p(self._stream(stream, self.device)))
        if rc != 0:
            raise _lib.OSCError("osc_batch_kinematics", rc)
        return out

    def compute(self, qpos, qvel, want_sites: bool = True) -> KinOutputs:
        nenv = int(qpos.shape[0])
        qpos = self._dev(qpos, (nenv, self.nq), "qpos")
        qvel = self._dev(qvel, (nenv, self.nv), "qvel")
        with torch.cuda.device(self.device):
            return self.compute_into(self.alloc(nenv, want_sites), qpos, qvel)

    def state_to_qpos(self, body_rotation, linear_body_velocity, angular_body_velocity,
                      motor_position, motor_velocity, stream=None):
        """update_mj_data's packing (osc.h:357-361) for SoA batches of State fields."""
        nenv = int(body_rotation.shape[0])
        nu = self.nq - 7
        args = [self._dev(body_rotation, (nenv, 4), "body_rotation"),
                self._dev(linear_body_velocity, (nenv, 3), "linear_body_velocity"),
                self._dev(angular_body_velocity, (nenv, 3), "angular_body_velocity"),
                self._dev(motor_position, (nenv, nu), "motor_position"),
                self._dev(motor_velocity, (nenv, nu), "motor_velocity")]
        qpos = torch.empty((nenv, self.nq), dtype=torch.float64, device=self.device)
        qvel = torch.empty((nenv, self.nv), dtype=torch.float64, device=self.device)
        rc = _lib.lib().osc_state_to_qpos(nenv, nu, *[ctypes.c_void_p(a.data_ptr()) for a in args],
                                          ctypes.c_void_p(qpos.data_ptr()),
                                          ctypes.c_void_p(qvel.data_ptr()),
                                          ctypes.c_void_p(self._stream(stream, self.device)))
        if rc != 0:
            raise _lib.OSCError("osc_state_to_qpos", rc)
        return qpos, qvel

    def workspace_bytes(self, solver, nenv: int) -> int:
        nb = ctypes.c_size_t()
        rc = _lib.lib().osc_qpos_workspace_bytes(solver._h, self._h, nenv, ctypes.byref(nb))
        if rc != 0:
            raise _lib.OSCError("osc_qpos_workspace_bytes", rc)
        return nb.value

    def solve_into(self, solver, out, qpos, qvel, T, mask, workspace, stream=None):
        """osc_batch_solve_qpos: kinematics + QP assembly + interior point, launch only."""
        nenv = out.tau.shape[0]
        ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
        rc = _lib.lib().osc_batch_solve_qpos(
            solver._h, self._h, nenv, ptr(qpos), ptr(qvel), ptr(T), ptr(mask), ptr(out.tau),
            ptr(out.x), ptr(out.status), ptr(out.iters), ptr(workspace),
            ctypes.c_size_t(0 if workspace is None else workspace.numel() * 8),
            ctypes.c_void_p(self._stream(stream, self.device)))
        if rc != 0:
            raise _lib.OSCError("osc_batch_solve_qpos", rc)
        return out

    def solve_warm_into(self, solver, out, warm, qpos, qvel, T, mask, workspace, stream=None):
        """osc_batch_solve_qpos_warm: the tick from joint states, warm-started from `warm`."""
        nenv = out.tau.shape[0]
        ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
        rc = _lib.lib().osc_batch_solve_qpos_warm(
            solver._h, self._h, nenv, ptr(qpos), ptr(qvel), ptr(T), ptr(mask), ptr(out.tau),
            ptr(out.x), ptr(out.status), ptr(out.iters), ptr(warm),
            ctypes.c_size_t(0 if warm is None else warm.numel() * 8), ptr(workspace),
            ctypes.c_size_t(0 if workspace is None else workspace.numel() * 8),
            ctypes.c_void_p(self._stream(stream, self.device)))
        if rc != 0:
            raise _lib.OSCError("osc_batch_solve_qpos_warm", rc)
        return out

    def solve(self, solver, qpos, qvel, T, mask, want_x: bool = False):
        d = solver.dims
        nenv = int(qpos.shape[0])
        qpos = self._dev(qpos, (nenv, self.nq), "qpos")
        qvel = self._dev(qvel, (nenv, self.nv), "qvel")
        T = self._dev(T, (nenv, d["ns"], 6), "T")
        mask = self._dev(mask, (nenv, d["nc"]), "mask")
        out = solver.alloc_outputs(nenv, want_x)
        ws = torch.empty((max(self.workspace_bytes(solver, nenv) // 8, 2),), dtype=torch.float64,
                         device=self.device)
        with torch.cuda.device(self.device):
            return self.solve_into(solver, out, qpos, qvel, T, mask, ws)


def _tree_joints(tree: dict):
    """(type, body) of every joint in qpos order: a body's "joints" list, else its "joint"."""
    out = []
    for i, b in enumerate(tree["bodies"]):
        if "joints" in b:
            out += [(j["type"], i) for j in b["joints"]]
        elif b["joint"] != "none":
            out.append((b["joint"], i))
    return out


def random_states(tree: dict, nenv: int, seed: int, base_pos_zero: bool = True,
                  joint_range: float = 1.0, vel_scale: float = 1.0):
    """Seeded synthetic joint states for a tree: unit base / ball quaternions, hinge angles
    uniform in +-joint_range, slides in +-0.3 joint_range, velocities N(0, vel_scale^2); base
    position 0 as update_mj_data sets it (osc.h:358-359) unless base_pos_zero is False."""
    rng = np.random.default_rng(seed)
    joints = _tree_joints(tree)
    nqj = {"free": 7, "ball": 4, "slide": 1, "hinge": 1}
    nvj = {"free": 6, "ball": 3, "slide": 1, "hinge": 1}
    nq = sum(nqj[t] for t, _ in joints)
    nv = sum(nvj[t] for t, _ in joints)
    qpos = np.zeros((nenv, nq))
    qvel = vel_scale * rng.standard_normal((nenv, nv))
    qa = 0
    for t, _ in joints:
        if t == "free":
            if not base_pos_zero:
                qpos[:, qa:qa + 3] = 0.3 * rng.standard_normal((nenv, 3))
            q = rng.standard_normal((nenv, 4))
            qpos[:, qa + 3:qa + 7] = q / np.linalg.norm(q, axis=1, keepdims=True)
        elif t == "ball":
            q = rng.standard_normal((nenv, 4))
            qpos[:, qa:qa + 4] = q / np.linalg.norm(q, axis=1, keepdims=True)
        elif t == "hinge":
            qpos[:, qa] = rng.uniform(-joint_range, joint_range, size=nenv)
        else:
            qpos[:, qa] = rng.uniform(-0.3 * joint_range, 0.3 * joint_range, size=nenv)
        qa += nqj[t]
    return qpos, qvel
