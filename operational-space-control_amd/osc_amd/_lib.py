"""ctypes binding of the C-ABI in include/osc_batch.h (libosc_batch.so, built in-tree).

This is the Python twin of the binding a maintainer would add on the reference side
(INTEGRATION.md).  There is deliberately NO fallback: if the HIP library is missing the import
fails, and solving on a machine without a GPU raises.
"""
from __future__ import annotations

import ctypes
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("OSC_LIB_PATH", os.path.join(PKG_DIR, "lib", "libosc_batch.so"))

OSC_MAX_SITES = 32
OSC_MAX_NU = 16

STATUS_NAMES = {0: "OSC_OK", 1: "OSC_ERR_INVALID_ARGUMENT", 2: "OSC_ERR_UNSUPPORTED_DIMS",
                3: "OSC_ERR_IO", 4: "OSC_ERR_DEVICE", 5: "OSC_ERR_NO_DEVICE"}
SOLVE_OK, SOLVE_MAX_ITER, SOLVE_NUMERICAL, SOLVE_UNREFINED = 0, 1, 2, 3

EXPORTED_SYMBOLS = ("osc_desc_from_yaml", "osc_model_create", "osc_model_create_from_yaml",
                    "osc_model_destroy", "osc_model_get_desc", "osc_workspace_bytes",
                    "osc_workspace_env_bytes",
                    "osc_batch_solve", "osc_batch_assemble", "osc_batch_solve_assembled",
                    "osc_status_string", "osc_abi_version",
                    "osc_pd_base_targets", "osc_contact_mask_from_contacts",
                    "osc_kin_desc_from_json", "osc_kin_model_create",
                    "osc_kin_model_create_from_json", "osc_kin_model_destroy",
                    "osc_kin_model_dims", "osc_batch_kinematics", "osc_state_to_qpos",
                    "osc_qpos_workspace_bytes", "osc_batch_solve_qpos",
                    "osc_warm_state_bytes", "osc_batch_solve_warm", "osc_batch_solve_assembled_warm",
                    "osc_batch_solve_qpos_warm", "osc_batch_solve_multi",
                    "osc_kin_desc_from_mjcf", "osc_kin_desc_from_mjcf_robot",
                    "osc_contact_geom_table", "osc_tumbling_params_default",
                    "osc_tumbling_targets", "osc_dual_rows", "osc_batch_solve_ex",
                    "osc_batch_assemble_ex", "osc_model_tuning_defaults",
                    "osc_model_create_tuned", "osc_batch_solve_warm_ex",
                    "osc_host_feed_create", "osc_host_feed_destroy", "osc_host_feed_inputs",
                    "osc_host_feed_submit", "osc_host_feed_wait", "osc_host_feed_timing")

OSC_KIN_MAX_BODIES = 16
OSC_KIN_MAX_DOFS = 32
OSC_KIN_MAX_SITES = 32
JOINT_NONE, JOINT_FREE, JOINT_BALL, JOINT_SLIDE, JOINT_HINGE = -1, 0, 1, 2, 3   # mjtJoint


class OscModelDesc(ctypes.Structure):
    _fields_ = [
        ("nv", ctypes.c_int32), ("nu", ctypes.c_int32), ("nc", ctypes.c_int32),
        ("ns", ctypes.c_int32),
        ("mu", ctypes.c_double),
        ("w_pos", ctypes.c_double * OSC_MAX_SITES),
        ("w_rot", ctypes.c_double * OSC_MAX_SITES),
        ("w_torque", ctypes.c_double), ("w_reg", ctypes.c_double),
        ("u_lb", ctypes.c_double * OSC_MAX_NU), ("u_ub", ctypes.c_double * OSC_MAX_NU),
        ("z_lb", ctypes.c_double * 3), ("z_ub", ctypes.c_double * 3),
        ("infinity", ctypes.c_double),
        ("eps_mu", ctypes.c_double),
        ("max_iter", ctypes.c_int32),
        ("wheel_rows", ctypes.c_int32),
        ("wheel_dof", ctypes.c_int32 * OSC_MAX_SITES),
        ("wheel_radius", ctypes.c_double * OSC_MAX_SITES),
    ]


class OscModelTuning(ctypes.Structure):
    """osc_model_tuning (include/osc_batch.h, ABI 3): solver policy knobs, no QP change."""
    _fields_ = [
        ("refine_steps", ctypes.c_int32), ("refine_max_move", ctypes.c_double),
        ("eps_mu", ctypes.c_double), ("restart_iter", ctypes.c_int32),
        ("warm_restart", ctypes.c_int32), ("warm_delta", ctypes.c_double),
        ("warm_center", ctypes.c_double), ("wheel_tol", ctypes.c_double),
        ("small_batch_max", ctypes.c_int32), ("park_it", ctypes.c_int32),
    ]


class OscSolveExtras(ctypes.Structure):
    """osc_solve_extras (include/osc_batch.h): per-call extras of osc_batch_solve_ex."""
    _fields_ = [("wheel_dir", ctypes.c_void_p), ("y", ctypes.c_void_p)]


class OscTumblingParams(ctypes.Structure):
    """osc_tumbling_params (include/osc_producers.h)."""
    _fields_ = [(n, ctypes.c_double) for n in (
        "shin_rot_vel", "shin_kp", "shin_kv", "thigh_lin_vel", "thigh_lin_kp", "thigh_lin_kv",
        "thigh_height_offset", "torso_lin_vel", "torso_lin_kp", "torso_lin_kv", "torso_ang_kp",
        "torso_ang_kv")] + [("shin_qadr", ctypes.c_int32 * 4)]


class OscBatchJob(ctypes.Structure):
    """osc_batch_job (include/osc_batch.h): one model's batch inside osc_batch_solve_multi."""
    _fields_ = [("model", ctypes.c_void_p), ("nenv", ctypes.c_int32)] + \
        [(n, ctypes.c_void_p) for n in ("M", "C", "J", "b", "T", "contact_mask", "tau", "x",
                                         "status", "iters", "workspace")] + \
        [("workspace_bytes", ctypes.c_size_t), ("wheel_dir", ctypes.c_void_p)]


_B, _S = OSC_KIN_MAX_BODIES, OSC_KIN_MAX_SITES


class OscKinDesc(ctypes.Structure):
    """osc_kin_desc (include/osc_kinematics.h): mjModel's body / joint / site fields."""
    _fields_ = [
        ("nbody", ctypes.c_int32), ("nsite", ctypes.c_int32),
        ("gravity", ctypes.c_double * 3),
        ("parent", ctypes.c_int32 * _B), ("jnt_type", ctypes.c_int32 * _B),
        ("pos", (ctypes.c_double * 3) * _B), ("quat", (ctypes.c_double * 4) * _B),
        ("axis", (ctypes.c_double * 3) * _B), ("jnt_pos", (ctypes.c_double * 3) * _B),
        ("armature", ctypes.c_double * _B), ("mass", ctypes.c_double * _B),
        ("ipos", (ctypes.c_double * 3) * _B), ("iquat", (ctypes.c_double * 4) * _B),
        ("inertia", (ctypes.c_double * 3) * _B),
        ("site_body", ctypes.c_int32 * _S), ("site_pos", (ctypes.c_double * 3) * _S),
        ("has_jac_body", ctypes.c_int32), ("site_jac_body", ctypes.c_int32 * _S),
    ]


class OscFeedInputs(ctypes.Structure):
    """osc_feed_inputs (include/osc_host_feed.h): pinned host pointers of one slot's inputs."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("M", "C", "J", "b", "qpos", "qvel", "T",
                                                "contact_mask")] + [("bytes", ctypes.c_size_t)]


class OscFeedOutputs(ctypes.Structure):
    """osc_feed_outputs (include/osc_host_feed.h): pinned host pointers of one tick's outputs."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("tau", "status", "iters")] + \
        [("bytes", ctypes.c_size_t)]


class OscFeedTiming(ctypes.Structure):
    """osc_feed_timing (include/osc_host_feed.h): per-stage HIP-event durations (ms)."""
    _fields_ = [(n, ctypes.c_float) for n in ("h2d_ms", "solve_ms", "d2h_ms",
                                               "h2d_start_to_d2h_end_ms", "kin_ms")]


FEED_QP, FEED_JOINT_STATES, FEED_WARM = 0, 1, 1


class OSCError(RuntimeError):
    def __init__(self, where: str, code: int):
        super().__init__(f"{where} failed: {STATUS_NAMES.get(code, code)}")
        self.code = code


_lib = None


def lib() -> ctypes.CDLL:
    """Load libosc_batch.so (raises if it has not been built -- no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built; run __graft_entry__.build() "
                          "(hipcc --offload-arch=gfx950)")
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, dp = ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(OscModelDesc)
    L.osc_desc_from_yaml.argtypes = [ctypes.c_char_p, ctypes.c_char_p, dp]
    L.osc_desc_from_yaml.restype = ctypes.c_int
    L.osc_model_create.argtypes = [dp, ctypes.POINTER(vp)]
    L.osc_model_create.restype = ctypes.c_int
    L.osc_model_tuning_defaults.argtypes = [dp, ctypes.POINTER(OscModelTuning)]
    L.osc_model_tuning_defaults.restype = ctypes.c_int
    L.osc_model_create_tuned.argtypes = [dp, ctypes.POINTER(OscModelTuning), ctypes.POINTER(vp)]
    L.osc_model_create_tuned.restype = ctypes.c_int
    L.osc_model_create_from_yaml.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(vp)]
    L.osc_model_create_from_yaml.restype = ctypes.c_int
    L.osc_model_destroy.argtypes = [vp]
    L.osc_model_destroy.restype = ctypes.c_int
    L.osc_model_get_desc.argtypes = [vp, dp]
    L.osc_model_get_desc.restype = ctypes.c_int
    L.osc_workspace_bytes.argtypes = [vp, i32, ctypes.POINTER(ctypes.c_size_t)]
    L.osc_workspace_bytes.restype = ctypes.c_int
    L.osc_workspace_env_bytes.argtypes = [vp, ctypes.POINTER(ctypes.c_size_t)]
    L.osc_workspace_env_bytes.restype = ctypes.c_int
    L.osc_batch_solve.argtypes = [vp, i32] + [vp] * 10 + [vp, ctypes.c_size_t, vp]
    L.osc_batch_solve.restype = ctypes.c_int
    L.osc_status_string.argtypes = [ctypes.c_int]
    L.osc_status_string.restype = ctypes.c_char_p
    L.osc_abi_version.argtypes = []
    L.osc_abi_version.restype = ctypes.c_int
    L.osc_batch_assemble.argtypes = [vp, i32] + [vp] * 6 + [vp, ctypes.c_size_t, vp]
    L.osc_batch_assemble.restype = ctypes.c_int
    L.osc_batch_solve_assembled.argtypes = [vp, i32] + [vp] * 5 + [vp, ctypes.c_size_t, vp]
    L.osc_batch_solve_assembled.restype = ctypes.c_int
    L.osc_pd_base_targets.argtypes = [i32, i32] + [vp] * 5 + [i32, vp, i32, vp, vp, vp]
    L.osc_pd_base_targets.restype = ctypes.c_int
    L.osc_contact_mask_from_contacts.argtypes = [i32, i32, i32, vp, vp, i32, vp, vp, vp]
    L.osc_contact_mask_from_contacts.restype = ctypes.c_int
    ip32 = ctypes.POINTER(ctypes.c_int32)
    L.osc_contact_geom_table.argtypes = [i32, ip32, i32, ip32, i32, ip32, ip32]
    L.osc_contact_geom_table.restype = ctypes.c_int
    L.osc_tumbling_params_default.argtypes = [ctypes.POINTER(OscTumblingParams)]
    L.osc_tumbling_params_default.restype = None
    L.osc_tumbling_targets.argtypes = [i32, i32, i32, i32] + [vp] * 7 + \
        [ctypes.POINTER(OscTumblingParams), vp, vp]
    L.osc_tumbling_targets.restype = ctypes.c_int
    L.osc_warm_state_bytes.argtypes = [vp, i32, ctypes.POINTER(ctypes.c_size_t)]
    L.osc_warm_state_bytes.restype = ctypes.c_int
    L.osc_batch_solve_warm.argtypes = [vp, i32] + [vp] * 11 + [ctypes.c_size_t, vp,
                                                               ctypes.c_size_t, vp]
    L.osc_batch_solve_warm.restype = ctypes.c_int
    L.osc_batch_solve_warm_ex.argtypes = [vp, i32] + [vp] * 6 + [ctypes.POINTER(OscSolveExtras)] + \
        [vp] * 5 + [ctypes.c_size_t, vp, ctypes.c_size_t, vp]
    L.osc_batch_solve_warm_ex.restype = ctypes.c_int
    L.osc_batch_solve_assembled_warm.argtypes = [vp, i32] + [vp] * 6 + [ctypes.c_size_t, vp,
                                                                         ctypes.c_size_t, vp]
    L.osc_batch_solve_assembled_warm.restype = ctypes.c_int
    L.osc_dual_rows.argtypes = [vp, ctypes.POINTER(i32)]
    L.osc_dual_rows.restype = ctypes.c_int
    L.osc_batch_solve_ex.argtypes = [vp, i32] + [vp] * 6 + [ctypes.POINTER(OscSolveExtras)] + \
        [vp] * 4 + [vp, ctypes.c_size_t, vp]
    L.osc_batch_solve_ex.restype = ctypes.c_int
    L.osc_batch_assemble_ex.argtypes = [vp, i32] + [vp] * 7 + [vp, ctypes.c_size_t, vp]
    L.osc_batch_assemble_ex.restype = ctypes.c_int
    L.osc_batch_solve_multi.argtypes = [ctypes.POINTER(OscBatchJob), i32, vp]
    L.osc_batch_solve_multi.restype = ctypes.c_int
    kp = ctypes.POINTER(OscKinDesc)
    L.osc_kin_desc_from_json.argtypes = [ctypes.c_char_p, ctypes.c_char_p, kp]
    L.osc_kin_desc_from_json.restype = ctypes.c_int
    L.osc_kin_desc_from_mjcf.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p),
                                         ctypes.POINTER(ctypes.c_char_p), i32, i32, kp]
    L.osc_kin_desc_from_mjcf.restype = ctypes.c_int
    L.osc_kin_desc_from_mjcf_robot.argtypes = [ctypes.c_char_p, ctypes.c_char_p,
                                               ctypes.c_char_p, kp]
    L.osc_kin_desc_from_mjcf_robot.restype = ctypes.c_int
    L.osc_kin_model_create.argtypes = [kp, ctypes.POINTER(vp)]
    L.osc_kin_model_create.restype = ctypes.c_int
    L.osc_kin_model_create_from_json.argtypes = [ctypes.c_char_p, ctypes.c_char_p,
                                                 ctypes.POINTER(vp)]
    L.osc_kin_model_create_from_json.restype = ctypes.c_int
    L.osc_kin_model_destroy.argtypes = [vp]
    L.osc_kin_model_destroy.restype = ctypes.c_int
    ip = ctypes.POINTER(ctypes.c_int32)
    L.osc_kin_model_dims.argtypes = [vp, ip, ip, ip]
    L.osc_kin_model_dims.restype = ctypes.c_int
    L.osc_batch_kinematics.argtypes = [vp, i32] + [vp] * 7 + [vp]
    L.osc_batch_kinematics.restype = ctypes.c_int
    L.osc_state_to_qpos.argtypes = [i32, i32] + [vp] * 7 + [vp]
    L.osc_state_to_qpos.restype = ctypes.c_int
    L.osc_qpos_workspace_bytes.argtypes = [vp, vp, i32, ctypes.POINTER(ctypes.c_size_t)]
    L.osc_qpos_workspace_bytes.restype = ctypes.c_int
    L.osc_batch_solve_qpos.argtypes = [vp, vp, i32] + [vp] * 9 + [ctypes.c_size_t, vp]
    L.osc_batch_solve_qpos.restype = ctypes.c_int
    L.osc_batch_solve_qpos_warm.argtypes = [vp, vp, i32] + [vp] * 9 + [ctypes.c_size_t, vp,
                                                                      ctypes.c_size_t, vp]
    L.osc_batch_solve_qpos_warm.restype = ctypes.c_int
    L.osc_host_feed_create.argtypes = [vp, vp, i32, i32, ctypes.c_uint32, i32, ctypes.POINTER(vp)]
    L.osc_host_feed_create.restype = ctypes.c_int
    L.osc_host_feed_destroy.argtypes = [vp]
    L.osc_host_feed_destroy.restype = ctypes.c_int
    L.osc_host_feed_inputs.argtypes = [vp, i32, ctypes.POINTER(OscFeedInputs)]
    L.osc_host_feed_inputs.restype = ctypes.c_int
    L.osc_host_feed_submit.argtypes = [vp, i32]
    L.osc_host_feed_submit.restype = ctypes.c_int
    L.osc_host_feed_wait.argtypes = [vp, i32, ctypes.POINTER(OscFeedOutputs)]
    L.osc_host_feed_wait.restype = ctypes.c_int
    L.osc_host_feed_timing.argtypes = [vp, i32, ctypes.POINTER(OscFeedTiming)]
    L.osc_host_feed_timing.restype = ctypes.c_int
    _lib = L
    return L


def desc_from_yaml(robot: str, yaml_path: str | None = None) -> OscModelDesc:
    d = OscModelDesc()
    rc = lib().osc_desc_from_yaml(robot.encode(), yaml_path.encode() if yaml_path else None,
                                  ctypes.byref(d))
    if rc != 0:
        raise OSCError("osc_desc_from_yaml", rc)
    return d


def kin_desc_from_json(robot: str, json_path: str | None = None) -> OscKinDesc:
    d = OscKinDesc()
    rc = lib().osc_kin_desc_from_json(robot.encode() if robot else None,
                                      json_path.encode() if json_path else None, ctypes.byref(d))
    if rc != 0:
        raise OSCError("osc_kin_desc_from_json", rc)
    return d


def kin_desc_from_dict(tree: dict) -> OscKinDesc:
    """osc_kin_desc from the <robot>_kinematics.json schema already parsed into a dict."""
    d = OscKinDesc()
    bodies, sites = tree["bodies"], tree["sites"]
    d.nbody, d.nsite = len(bodies), len(sites)
    d.gravity[:] = tree["gravity"]
    jt = {"free": JOINT_FREE, "ball": JOINT_BALL, "slide": JOINT_SLIDE, "hinge": JOINT_HINGE,
          "none": JOINT_NONE}
    for i, b in enumerate(bodies):
        d.parent[i] = b["parent"]
        d.jnt_type[i] = jt[b["joint"]]
        d.pos[i][:] = b["pos"]
        d.quat[i][:] = b["quat"]
        d.axis[i][:] = b.get("axis", [0.0, 0.0, 1.0])
        d.jnt_pos[i][:] = b.get("jnt_pos", [0.0, 0.0, 0.0])
        d.armature[i] = b.get("armature", 0.0)
        d.mass[i] = b["mass"]
        d.ipos[i][:] = b["ipos"]
        d.iquat[i][:] = b["iquat"]
        d.inertia[i][:] = b["diaginertia"]
    for k, s in enumerate(sites):
        d.site_body[k] = s["body"]
        d.site_pos[k][:] = s["pos"]
        d.site_jac_body[k] = s.get("jac_body", s["body"])
        if "jac_body" in s:
            d.has_jac_body = 1
    return d


def kin_desc_to_dict(d: OscKinDesc, name: str = "") -> dict:
    """The <robot>_kinematics.json schema of a descriptor (inverse of kin_desc_from_dict)."""
    jt = {JOINT_FREE: "free", JOINT_BALL: "ball", JOINT_SLIDE: "slide", JOINT_HINGE: "hinge",
          JOINT_NONE: "none"}
    bodies = []
    for i in range(d.nbody):
        bodies.append({"parent": d.parent[i], "joint": jt[d.jnt_type[i]], "pos": list(d.pos[i]),
                       "quat": list(d.quat[i]), "axis": list(d.axis[i]),
                       "jnt_pos": list(d.jnt_pos[i]), "armature": d.armature[i],
                       "mass": d.mass[i], "ipos": list(d.ipos[i]), "iquat": list(d.iquat[i]),
                       "diaginertia": list(d.inertia[i])})
    sites = []
    for k in range(d.nsite):
        s = {"body": d.site_body[k], "pos": list(d.site_pos[k])}
        if d.has_jac_body:
            s["jac_body"] = d.site_jac_body[k]
        sites.append(s)
    return {"name": name, "gravity": list(d.gravity), "bodies": bodies, "sites": sites}


def kin_desc_from_mjcf(xml_path: str, body_names, site_names, model_order: bool) -> OscKinDesc:
    """osc_kin_desc_from_mjcf (host-only MJCF reader; include/osc_kinematics.h)."""
    d = OscKinDesc()
    n = len(site_names)
    bn = (ctypes.c_char_p * n)(*[x.encode() for x in body_names])
    sn = (ctypes.c_char_p * n)(*[x.encode() for x in site_names])
    rc = lib().osc_kin_desc_from_mjcf(xml_path.encode(), bn, sn, n, 1 if model_order else 0,
                                      ctypes.byref(d))
    if rc != 0:
        raise OSCError("osc_kin_desc_from_mjcf", rc)
    return d


def kin_desc_from_mjcf_robot(robot: str, xml_path: str, yaml_path: str | None = None) -> OscKinDesc:
    d = OscKinDesc()
    rc = lib().osc_kin_desc_from_mjcf_robot(robot.encode(),
                                            yaml_path.encode() if yaml_path else None,
                                            xml_path.encode(), ctypes.byref(d))
    if rc != 0:
        raise OSCError("osc_kin_desc_from_mjcf_robot", rc)
    return d
