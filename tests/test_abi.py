"""CPU tests of the drop-in boundary: libosc_batch.so loads, exports every symbol the header
declares, parses the reference's YAML schema, and reports errors the documented way.  No
compute calls (no GPU here)."""
import ctypes
import os
import re

import numpy as np
import pytest

from osc_amd import _lib
from osc_qp import load_model

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(REPO, "include", h) for h in ("osc_batch.h", "osc_producers.h", "osc_kinematics.h",
                                                               "osc_host_feed.h")]
REF_CONFIG = "/root/reference/config"


def test_library_loads_and_exports_header_symbols():
    L = _lib.lib()
    declared = set()
    for h in HEADERS:
        declared |= set(re.findall(r"^\s*(?:int|void|const char\*)\s+(osc_\w+)\s*\(", open(h).read(), re.M))
    assert declared == set(_lib.EXPORTED_SYMBOLS)
    for name in declared:
        assert hasattr(L, name), name
    assert L.osc_abi_version() == 4
    assert L.osc_status_string(2) == b"OSC_ERR_UNSUPPORTED_DIMS"


@pytest.mark.parametrize("robot", ["unitree_go2", "walter_sr", "walter_sr_wheels"])
def test_tuning_defaults(robot):
    """osc_model_tuning_defaults (ABI 3): the model's solver-policy defaults, host-only."""
    L = _lib.lib()
    d = _lib.desc_from_yaml(robot)
    t = _lib.OscModelTuning()
    assert L.osc_model_tuning_defaults(ctypes.byref(d), ctypes.byref(t)) == 0
    assert t.refine_steps == (12 if d.wheel_rows else 2)
    assert t.refine_max_move == 1e300 and t.eps_mu == d.eps_mu
    assert (t.restart_iter, t.warm_restart, t.warm_delta, t.warm_center) == (28, 22, 1.0, 1.0)
    assert t.wheel_tol == 1e-6 and t.small_batch_max == -1 and t.park_it == -1
    assert L.osc_model_tuning_defaults(None, ctypes.byref(t)) == 1
    # invalid tuning is refused before any device call
    h = ctypes.c_void_p()
    t.refine_steps = -1
    assert L.osc_model_create_tuned(ctypes.byref(d), ctypes.byref(t), ctypes.byref(h)) in (1, 5)


def test_release_library_reads_no_tuning_variables():
    """The release library reads no OSC_* tuning environment variable: the knobs
    live in osc_model_tuning; the OSC_TUNING_ENV diagnostic build alone reads them."""
    blob = open(_lib.LIB_PATH, "rb").read()
    for name in (b"OSC_REFINE_STEPS", b"OSC_EPS_MU", b"OSC_RESTART_ITER", b"OSC_WARM_RESTART",
                 b"OSC_WARM_DELTA", b"OSC_WARM_CENTER", b"OSC_REFINE_MAX_MOVE", b"OSC_WHEEL_TOL",
                 b"OSC_SMALL_BATCH_MAX", b"OSC_PARK_IT", b"OSC_TICK_GRAPH"):
        assert name not in blob, name
    ctrl = os.path.join(os.path.dirname(_lib.LIB_PATH), "libosc_controller.so")
    if os.path.exists(ctrl):
        assert b"OSC_TICK_GRAPH" not in open(ctrl, "rb").read()


@pytest.mark.parametrize("robot", ["unitree_go2", "walter_sr", "walter_sr_wheels"])
def test_desc_from_yaml_matches_oracle(robot):
    d = _lib.desc_from_yaml(robot)          # default config next to the library
    m = load_model(robot)                   # oracle's independent reader (PyYAML)
    assert (d.nv, d.nu, d.nc, d.ns) == (m.nv, m.nu, m.nc, m.ns)
    assert d.mu == m.mu and d.w_torque == m.w_torque and d.w_reg == m.w_reg
    np.testing.assert_array_equal(np.array(d.w_pos[:m.ns]), m.w_pos)
    np.testing.assert_array_equal(np.array(d.w_rot[:m.ns]), m.w_rot)
    np.testing.assert_array_equal(np.array(d.u_lb[:m.nu]), m.u_lb)
    np.testing.assert_array_equal(np.array(d.u_ub[:m.nu]), m.u_ub)
    assert list(d.z_lb) == [-1e30, -1e30, 0.0] and list(d.z_ub) == [1e30, 1e30, 1e4]


@pytest.mark.skipif(not os.path.isdir(REF_CONFIG), reason="reference tree not mounted")
@pytest.mark.parametrize("robot,rel", [
    ("unitree_go2", "unitree_go2/unitree_go2_config.yaml"),
    ("walter_sr", "walter_sr/walter_sr_config.yaml"),
    ("walter_sr_wheels", "walter_sr_wheels/walter_sr_wheels_config.yaml"),
    ("walter_sr", "walter_sr/true_tumbling_mjjoint.yaml"),
    # every WaLTER scenario config of the reference (same shape, different weights / targets)
    ("walter_sr", "walter_sr/base_bad_stairs_climbing.yaml"),
    ("walter_sr", "walter_sr/forward_velocity_front_tumbling.yaml"),
    ("walter_sr", "walter_sr/forward_velocity_front_tumbling2.yaml"),
    ("walter_sr", "walter_sr/slowtumbling.yaml"),
    ("walter_sr", "walter_sr/slowtumbling_with_bodytargets_maybe_stairs.yaml"),
    ("walter_sr", "walter_sr/stairclimbing_slightlybetter.yaml"),
    ("walter_sr", "walter_sr/torso_tumbling_fail.yaml"),
])
def test_reads_reference_yaml_files(robot, rel):
    """The native loader reads the reference's own config files (block lists, comments) and
    agrees with PyYAML on every weight."""
    path = os.path.join(REF_CONFIG, rel)
    d = _lib.desc_from_yaml(robot, path)
    m = load_model(robot, path)
    np.testing.assert_array_equal(np.array(d.w_pos[:m.ns]), m.w_pos)
    np.testing.assert_array_equal(np.array(d.w_rot[:m.ns]), m.w_rot)
    assert d.mu == m.mu
    # a model the library has a kernel for (select_kernel, csrc/osc_device.hpp)
    h = ctypes.c_void_p()
    rc = _lib.lib().osc_model_create(ctypes.byref(d), ctypes.byref(h))
    assert rc != 2, rel            # not OSC_ERR_UNSUPPORTED_DIMS (CPU-only: OSC_ERR_NO_DEVICE)
    if rc == 0:
        _lib.lib().osc_model_destroy(h)


def test_wheel_no_slip_yaml_keys(tmp_path):
    """The opt-in wheel rows (walter_sr_wheels/autogen/autogen.py:64-94, 128-240) come from three
    optional YAML keys; the reference's own configs (no such keys) leave them off."""
    from osc_amd.robots import config_path
    from osc_amd.synth import WALTER_WHEEL_DOFS, WHEEL_RADIUS
    assert _lib.desc_from_yaml("walter_sr_wheels").wheel_rows == 0
    d = _lib.desc_from_yaml("walter_sr_wheels", os.path.join(
        os.path.dirname(config_path("walter_sr_wheels")), "walter_sr_wheels_noslip_config.yaml"))
    assert d.wheel_rows == 1
    assert list(d.wheel_dof[:8]) == WALTER_WHEEL_DOFS and list(d.wheel_radius[:8]) == [WHEEL_RADIUS] * 8
    base = open(config_path("walter_sr_wheels")).read()
    for extra, ok in [("wheel_no_slip: true\nwheel_radius: [1, 2, 3, 4, 5, 6, 7, 8]\n"
                       "wheel_dofs: [-1, -1, 6, 7, 8, 9, 10, 11]\n", True),
                      ("wheel_no_slip: true\nwheel_radius: 0.1\nwheel_dofs: [1, 2]\n", False),
                      ("wheel_no_slip: true\nwheel_radius: 0.1\n"
                       "wheel_dofs: [0, 0, 0, 0, 0, 0, 0, 14]\n", False),
                      ("wheel_no_slip: maybe\n", False),
                      ("wheel_no_slip: false\n", True)]:
        f = tmp_path / "w.yaml"
        f.write_text(base + extra)
        if ok:
            _lib.desc_from_yaml("walter_sr_wheels", str(f))
        else:
            with pytest.raises(_lib.OSCError):
                _lib.desc_from_yaml("walter_sr_wheels", str(f))
    d = _lib.desc_from_yaml("walter_sr_wheels", str(tmp_path / "w.yaml"))
    assert d.wheel_rows == 0
    # models with wheel rows: only the WaLTER dimensions have a kernel; bad dof indices refused
    h = ctypes.c_void_p()
    g = _lib.desc_from_yaml("unitree_go2")
    g.wheel_rows = 1
    assert _lib.lib().osc_model_create(ctypes.byref(g), ctypes.byref(h)) == 2
    d.wheel_rows, d.wheel_dof[0] = 1, 14
    assert _lib.lib().osc_model_create(ctypes.byref(d), ctypes.byref(h)) == 1


def test_error_codes():
    L = _lib.lib()
    d = _lib.OscModelDesc()
    assert L.osc_desc_from_yaml(b"no_such_robot", None, ctypes.byref(d)) == 1
    assert L.osc_desc_from_yaml(b"unitree_go2", b"/nonexistent.yaml", ctypes.byref(d)) == 3
    h = ctypes.c_void_p()
    d = _lib.desc_from_yaml("unitree_go2")
    d.nv = 17                                   # no compiled kernel for these dimensions
    assert L.osc_model_create(ctypes.byref(d), ctypes.byref(h)) == 2
    d = _lib.desc_from_yaml("unitree_go2")
    d.z_ub[0] = 5.0                             # finite fx bound: not in the reference QP
    assert L.osc_model_create(ctypes.byref(d), ctypes.byref(h)) == 1
    assert L.osc_batch_solve(None, 1, *([None] * 10), None, 0, None) == 1
    assert L.osc_batch_assemble(None, 1, *([None] * 6), None, 0, None) == 1
    assert L.osc_batch_solve_assembled(None, 1, *([None] * 5), None, 0, None) == 1
    assert L.osc_batch_solve_ex(None, 1, *([None] * 6), None, *([None] * 4), None, 0, None) == 1
    assert L.osc_batch_assemble_ex(None, 1, *([None] * 7), None, 0, None) == 1
    rows = ctypes.c_int32()
    assert L.osc_dual_rows(None, ctypes.byref(rows)) == 1
    assert L.osc_pd_base_targets(1, 5, *([None] * 5), 0, None, 0, None, None, None) == 1
    assert L.osc_contact_mask_from_contacts(1, 4, 2, None, None, 0, None, None, None) == 1
    assert L.osc_model_destroy(None) == 1


def test_no_device_is_reported_not_faked():
    """On a host without a HIP device model creation fails loudly (no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("device present")
    h = ctypes.c_void_p()
    d = _lib.desc_from_yaml("unitree_go2")
    assert _lib.lib().osc_model_create(ctypes.byref(d), ctypes.byref(h)) == 5


@pytest.mark.parametrize("robot", ["unitree_go2", "walter_sr"])
def test_kin_desc_from_json_matches_python_reader(robot):
    """The library's JSON reader and the Python one fill identical descriptors."""
    import ctypes as ct
    from osc_amd.kinematics import kin_json_path, load_tree
    a = _lib.kin_desc_from_json(None, kin_json_path(robot))
    b = _lib.kin_desc_from_dict(load_tree(robot))
    assert ct.string_at(ct.addressof(a), ct.sizeof(a)) == ct.string_at(ct.addressof(b), ct.sizeof(b))
    assert _lib.kin_desc_from_json(robot).nbody == a.nbody    # default path next to the library


def test_kin_desc_errors():
    with pytest.raises(_lib.OSCError) as e:
        _lib.kin_desc_from_json(None, "/nonexistent/tree.json")
    assert e.value.code == 3
    import ctypes as ct
    from kin_trees import random_tree
    L = _lib.lib()
    bad = [lambda d: setattr(d, "nbody", 17),
           lambda d: d.parent.__setitem__(3, 5),            # parent after child
           lambda d: d.jnt_type.__setitem__(2, 0),          # free joint below the root
           lambda d: d.jnt_type.__setitem__(2, 5),          # not an mjtJoint value
           lambda d: [d.jnt_type.__setitem__(1, 2)] +       # slide without an axis
                     [d.axis[1].__setitem__(i, 0.0) for i in range(3)],
           lambda d: d.site_body.__setitem__(0, 40),
           lambda d: [d.axis[1].__setitem__(i, 0.0) for i in range(3)]]
    for mutate in bad:
        d = _lib.kin_desc_from_dict(random_tree(1, weld_p=0.0))
        mutate(d)
        h = ct.c_void_p()
        assert L.osc_kin_model_create(ct.byref(d), ct.byref(h)) == 1
    assert L.osc_batch_kinematics(None, 1, *([None] * 7), None) == 1


@pytest.mark.parametrize("text", ['{"bodies": [', '{"gravity": [0, 0], "bodies": [], "sites": []}',
                                  '{"gravity": [0, 0, -9.81], "bodies": [{"parent": -1}], "sites": []}',
                                  '[1, 2, 3]', ''])
def test_kin_desc_from_json_rejects_malformed(tmp_path, text):
    f = tmp_path / "tree.json"
    f.write_text(text)
    with pytest.raises(_lib.OSCError) as e:
        _lib.kin_desc_from_json(None, str(f))
    assert e.value.code == 3   # OSC_ERR_IO


def test_kin_desc_joint_strings_and_defaults(tmp_path):
    import json
    from kin_trees import random_tree
    t = random_tree(3, nbody=4, nsite=2)
    for b in t["bodies"][1:]:                  # optional keys may be omitted
        b.pop("armature"); b.pop("jnt_pos")
    f = tmp_path / "tree.json"
    f.write_text(json.dumps(t))
    d = _lib.kin_desc_from_json(None, str(f))
    assert d.nbody == 4 and d.nsite == 2
    assert list(d.jnt_type[:4]) == [{"free": 0, "hinge": 3, "none": -1}[b["joint"]] for b in t["bodies"]]
    assert all(d.armature[i] == 0.0 for i in range(1, 4))
