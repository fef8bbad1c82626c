"""OperationalSpaceController shim (include/osc_controller.h): the
reference's lifecycle/precondition semantics (unitree_go2/operational_space_controller.h:112-238)
on CPU, and on the GPU one synchronous tick plus the fixed-rate control thread (:546-589)
against the golden oracle torques.  Driven through the C++ program tests/cpp/osc_controller_test.cpp
(built here with hipcc against the in-tree libraries)."""
import json
import os
import subprocess

import numpy as np
import pytest

from osc_amd import build as osc_build
from osc_amd.robots import dims

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tests", "cpp", "osc_controller_test.cpp")
EXE = os.path.join(REPO, "tests", "cpp", "build", "osc_controller_test")
LIB = os.path.dirname(osc_build.OUT)
GOLDEN = os.path.join(REPO, "tests", "golden")

# absl::StatusCode values the shim's Status mirrors
OK, INVALID_ARGUMENT, FAILED_PRECONDITION, INTERNAL = 0, 3, 9, 13


def driver():
    osc_build.build()
    deps = [SRC, osc_build.OUT_CTRL, os.path.join(REPO, "include", "osc_controller.h"),
            os.path.join(REPO, "include", "osc_kinematics.h")]
    if not os.path.exists(EXE) or any(os.path.getmtime(p) > os.path.getmtime(EXE) for p in deps):
        os.makedirs(os.path.dirname(EXE), exist_ok=True)
        subprocess.run([osc_build.HIPCC, "-std=c++17", "-O2", "-I", os.path.join(REPO, "include"),
                        SRC, "-L", LIB, "-losc_controller", "-losc_batch",
                        f"-Wl,-rpath,{LIB}", "-o", EXE], check=True)
    return EXE


def run(*args, graph=None):
    if graph is not None:    # "1": the tick replayed as one captured hipGraph (set_tick_graph)
        args = (*args, graph)
    r = subprocess.run([driver(), *args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


@pytest.mark.parametrize("robot", ["unitree_go2", "walter_sr"])
def test_lifecycle_preconditions(robot):
    import torch
    out = run("lifecycle", robot)
    assert out["pre_opt"] == FAILED_PRECONDITION          # osc.h:164-165
    assert out["pre_thread"] == FAILED_PRECONDITION       # :180-182
    assert out["pre_stop"] == FAILED_PRECONDITION         # :190-191
    assert out["pre_clean"] == FAILED_PRECONDITION        # :211-212
    assert out["bad_mask"] == INVALID_ARGUMENT
    assert out["init"] == OK and out["initialized"] == 1
    assert out["thread_before_opt"] == FAILED_PRECONDITION
    assert out["step_before_opt"] == FAILED_PRECONDITION
    assert out["bad_robot"] == INTERNAL                   # load failure: InternalError (:117)
    assert out["torque0"] == dims(robot)["nu"]            # torque_command starts at Zero (:244)
    if torch.cuda.is_available():
        assert out["opt"] == OK and out["opt_initialized"] == 1
    else:                                                 # no device: reported, not faked
        assert out["opt"] == INTERNAL and out["opt_initialized"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("graph", ["0", "1"])
@pytest.mark.parametrize("case", ["go2_standing", "go2_tumbling_mask", "walter_standing"])
def test_controller_tick_and_thread_match_oracle(gpu, case, graph, tmp_path):
    g = np.load(os.path.join(GOLDEN, case + ".npz"))
    robot = str(g["robot"])
    fx = tmp_path / "fixture.bin"
    parts = [g[k][0].astype(np.float64).ravel() for k in ("M", "C", "J", "b", "T", "mask", "tau")]
    np.concatenate(parts).tofile(fx)
    out = run("solve", robot, str(fx), graph=graph)
    assert out["status"] == 0 and out["iters"] > 0
    assert out["err_step"] <= 1e-5 and out["err_thread"] <= 1e-5, out   # tests/test_gpu_parity.py
    assert out["slice"] == 0.0                            # torque = solution[nv:nv+nu] (osc.h:573)
    assert out["n"] == dims(robot)["n"]
    assert out["thread"] == OK and out["stop"] == OK and out["clean"] == OK
    assert out["ticks_60ms"] >= 10, out                   # 2000 us control rate


@pytest.mark.parametrize("robot", ["unitree_go2", "walter_sr"])
def test_gpu_kinematics_controller_arguments(robot):
    import torch
    out = run("gpu_lifecycle", robot)
    assert out["bad_state"] == INVALID_ARGUMENT           # State sized for another robot
    assert out["init"] == OK
    # a missing kinematic tree fails initialize() with InternalError, as the reference's XML
    # load does (osc.h:114-117); the optimization then has its precondition unmet (:164-165)
    assert out["init_nt"] == INTERNAL
    assert out["opt_nt"] == FAILED_PRECONDITION


@pytest.mark.gpu
@pytest.mark.parametrize("graph", ["0", "1"])
@pytest.mark.parametrize("robot", ["unitree_go2", "walter_sr", "walter_sr_wheels"])
def test_gpu_kinematics_controller_matches_oracle(gpu, robot, graph, tmp_path):
    """The controller without a KinematicsFn: State -> qpos/qvel (update_mj_data) -> GPU
    kinematics -> QP -> torque, against the oracle chain (kinematics oracle -> reference QP ->
    exact optimum)."""
    import kinematics as kin
    from osc_amd.kinematics import load_tree, random_states
    from osc_qp import build_qp, load_model, torque
    from qp_exact import solve_exact
    tree = load_tree(robot)
    qpos, qvel = random_states(tree, 1, 31, joint_range=0.5)
    model = load_model(robot)
    rng = np.random.default_rng(31)
    T = np.zeros((model.ns, 6))
    T[0] = 10.0 * rng.standard_normal(6)
    mask = np.ones(model.nc)
    mask[1] = 0.0
    M, C, J, b = kin.kinematics(kin.KinModel(tree), qpos[0], qvel[0])
    tau = torque(model, solve_exact(model, build_qp(model, M, C, J, b, T, mask), M, C, J).x)
    fx = tmp_path / "fixture.bin"
    np.concatenate([qpos[0], qvel[0], T.ravel(), mask, tau]).astype(np.float64).tofile(fx)
    out = run("qpos", robot, str(fx), graph=graph)
    assert out["status"] == 0
    assert out["err_step"] <= 1e-5 and out["err_thread"] <= 1e-5, out
    assert out["thread"] == OK and out["stop"] == OK and out["clean"] == OK
