"""Drop-in controller headers (include/operational-space-control/<robot>/):
tests/cpp/dropin_standing.cpp writes out the controller calls of the reference's
examples/standing.cc:86-164 and walter_sr_standing.cc:88-163 -- same includes, namespaces,
Eigen-typed State / TaskspaceTargets / Vector<nu>, absl::Status, the (xml_path) constructor --
and is compiled with plain g++ against the headers (Eigen / absl from tests/cpp/stubs/, the
image has neither) and linked with -losc_controller -losc_batch.

CPU: all three robots compile; the lifecycle preconditions match the reference's
(osc.h:112-218; an unreadable XML is InternalError as mj_loadXML's failure at :114-117).
GPU: the example loop runs its control thread on config/<robot>.xml for a joint state, and the
last torque command equals the oracle chain on the same inputs -- the MJCF read by the same
convention (Go2 model-order site rows, G/osc.h:373), the kinematics oracle, the reference QP,
its exact optimum -- within the 1e-5 normwise tolerance of tests/test_gpu_parity.py."""
import json
import os
import subprocess

import numpy as np
import pytest

from osc_amd import build as osc_build

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tests", "cpp", "dropin_standing.cpp")
OUT = os.path.join(REPO, "tests", "cpp", "build")
LIB = os.path.dirname(osc_build.OUT)
CFG = os.path.join(REPO, "operational-space-control_amd", "config")
ROBOTS = {"unitree_go2": 0, "walter_sr": 1, "walter_sr_wheels": 2}
XML = {"unitree_go2": "unitree_go2.xml", "walter_sr": "walter_sr.xml",
       "walter_sr_wheels": "walter_sr.xml"}
OK, INVALID_ARGUMENT, FAILED_PRECONDITION, INTERNAL = 0, 3, 9, 13


def build_driver(robot: str) -> str:
    """g++ (no HIP compiler needed by a user of the headers); rebuilt when a source is newer."""
    osc_build.build()
    exe = os.path.join(OUT, f"dropin_standing_{robot}")
    hdr = os.path.join(REPO, "include", "operational-space-control")
    deps = [SRC, osc_build.OUT_CTRL, os.path.join(REPO, "include", "osc_controller.h")]
    for root, _, files in os.walk(hdr):
        deps += [os.path.join(root, f) for f in files]
    if not os.path.exists(exe) or any(os.path.getmtime(p) > os.path.getmtime(exe) for p in deps):
        os.makedirs(OUT, exist_ok=True)
        subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-Werror",
                        f"-DOSC_DROPIN_ROBOT={ROBOTS[robot]}",
                        "-I", os.path.join(REPO, "tests", "cpp", "stubs"),
                        "-I", os.path.join(REPO, "include"), SRC, "-L", LIB, "-losc_controller",
                        "-losc_batch", f"-Wl,-rpath,{LIB}", "-Wl,-rpath-link,/opt/rocm/lib",
                        "-o", exe], check=True)
    return exe


def run(robot, *args):
    r = subprocess.run([build_driver(robot), *args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


@pytest.mark.parametrize("robot", list(ROBOTS))
def test_headers_compile_and_lifecycle(robot):
    from osc_amd.robots import dims
    out = run(robot, "lifecycle", os.path.join(CFG, XML[robot]))
    d = dims(robot)
    assert out["load"] == INTERNAL                      # mj_loadXML failure (osc.h:114-117)
    assert out["pre_opt"] == FAILED_PRECONDITION        # :164-165
    assert out["pre_thread"] == FAILED_PRECONDITION     # :180-182
    assert out["pre_stop"] == FAILED_PRECONDITION       # :190-191
    assert out["pre_clean"] == FAILED_PRECONDITION      # :211-212
    assert out["init"] == OK and out["initialized"] == 1
    assert out["torque0_norm"] == 0.0                   # torque_command starts at Zero (:244)
    assert (out["nu"], out["ns"], out["n"]) == (d["nu"], d["ns"], d["n"])


@pytest.mark.gpu
@pytest.mark.parametrize("robot", list(ROBOTS))
def test_standing_loop_matches_oracle(gpu, robot, tmp_path):
    import kinematics as kin
    from osc_amd.mjcf import load_mjcf_robot
    from osc_qp import build_qp, load_model, torque
    from qp_exact import solve_exact

    xml = os.path.join(CFG, XML[robot])
    tree = load_mjcf_robot(robot, xml)
    km = kin.KinModel(tree)
    rng = np.random.default_rng(31 + ROBOTS[robot])
    qpos, qvel = kin.random_state(km, rng, base_pos_zero=False)   # standing.cc reads qpos[0:3]
    qvel *= 0.3
    np.savetxt(tmp_path / "qpos.txt", qpos)
    np.savetxt(tmp_path / "qvel.txt", qvel)
    out = run(robot, "run", xml, str(tmp_path / "qpos.txt"), str(tmp_path / "qvel.txt"))
    model = load_model(robot)
    T = np.asarray(out["targets"]).reshape(model.ns, 6)
    q0 = qpos.copy()
    q0[0:3] = 0.0                                   # update_mj_data zeroes the base position
    M, C, J, b = kin.kinematics(km, q0, qvel)
    mask = np.ones(model.nc)
    ref = torque(model, solve_exact(model, build_qp(model, M, C, J, b, T, mask), M, C, J).x)
    tau = np.asarray(out["torque"])
    err = np.abs(tau - ref).max() / max(np.abs(ref).max(), 1.0)
    assert err <= 1e-5, (err, tau, ref)
    assert np.array_equal(np.asarray(out["solution"])[model.nv:model.nv + model.nu], tau)
    if robot == "unitree_go2":
        assert np.abs(T[0]).max() > 0 and np.all(T[1:] == 0)   # the base PD row only


def test_eigen_stub_is_as_strict_as_eigen(tmp_path):
    """The stub rejects what real Eigen rejects for the calls the harness makes: Map<M> needs
    mutable storage (examples/standing.cc:90-92 maps mj_data->qpos, a double*); read-only storage
    needs Map<const M>."""
    stub = os.path.join(REPO, "tests", "cpp", "stubs")
    cases = {"mutable": ("double a[3] = {1, 2, 3};\n"
                         "Eigen::Matrix<double, 3, 1> v = Eigen::Map<Eigen::Matrix<double, 3, 1>>(a);", 0),
             "const_view": ("const double a[3] = {1, 2, 3};\n"
                            "Eigen::Matrix<double, 3, 1> v = Eigen::Map<const Eigen::Matrix<double, 3, 1>>(a);", 0),
             "const_into_mutable": ("const double a[3] = {1, 2, 3};\n"
                                    "Eigen::Matrix<double, 3, 1> v = Eigen::Map<Eigen::Matrix<double, 3, 1>>(a);", 1)}
    for name, (body, fails) in cases.items():
        src = tmp_path / f"{name}.cpp"
        src.write_text("#include <Eigen/Dense>\nint main() {\n" + body + "\nreturn v(0) > 0 ? 0 : 1;\n}\n")
        r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I", stub, str(src)],
                           capture_output=True, text=True)
        assert (r.returncode != 0) == bool(fails), (name, r.stderr[-500:])
