"""The reference's OWN example programs compile and link, unchanged, against the drop-in headers
(BASELINE north_star: "walter_sr_standing and go2 standing link against it unchanged"; SURVEY.md
§8(b)).  The files are compiled where they lie under /root/reference/examples (never
copied into this repo); the test is skipped where the reference tree is absent (the GPU box).

Third-party headers the image lacks are declaration-only test stubs under tests/cpp/stubs/
(MuJoCo's C API subset the examples call, GLFW, Bazel's runfiles, and the Eigen / absl subsets the
drop-in headers already use); tests/cpp/stubs/mujoco_stub.cpp defines them so the link step
resolves every symbol -- the controller's against the real libosc_controller.so / libosc_batch.so.
BAZEL_CURRENT_REPOSITORY is the macro Bazel itself passes on the command line.

Warnings: -Wall -Wextra -Werror, except two that the examples' own code raises whatever the headers
(an unused `argc` in main, -Wunused-parameter; `initial_position` in walter_sr_standing.cc:96, set
but unused once the lines that read it are commented out, :148-158, -Wunused-but-set-variable)."""
import os
import subprocess

import pytest

from osc_amd import build as osc_build

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXAMPLES = "/root/reference/examples"
STUBS = os.path.join(REPO, "tests", "cpp", "stubs")
FLAGS = ["-std=c++20", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
         "-Wno-unused-but-set-variable", '-DBAZEL_CURRENT_REPOSITORY=""', "-I", STUBS,
         "-I", os.path.join(REPO, "include")]

pytestmark = pytest.mark.skipif(not os.path.isdir(EXAMPLES), reason="reference tree not mounted")

# the two the north star names, plus the other examples whose MuJoCo / Eigen use the stubs cover
NAMED = ["standing.cc", "walter_sr_standing.cc"]
ALSO = ["push_up.cc", "walter_sr_tumbling.cc"]


@pytest.mark.parametrize("example", NAMED + ALSO)
def test_example_compiles_unchanged(example):
    src = os.path.join(EXAMPLES, example)
    r = subprocess.run(["g++", *FLAGS, "-fsyntax-only", src], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]


@pytest.mark.parametrize("example", NAMED)
def test_example_links_unchanged(example, tmp_path):
    """Linked against the real controller library: every OperationalSpaceController member the
    example calls resolves in libosc_controller.so.  Run, it stops at mj_loadXML (no MuJoCo here)
    exactly as the example does on a missing model file (examples/standing.cc:37-41)."""
    osc_build.build()
    lib = os.path.dirname(osc_build.OUT)
    exe = tmp_path / example.replace(".cc", "")
    r = subprocess.run(["g++", *FLAGS, os.path.join(EXAMPLES, example),
                        os.path.join(STUBS, "mujoco_stub.cpp"), "-L", lib, "-losc_controller",
                        "-losc_batch", f"-Wl,-rpath,{lib}", "-Wl,-rpath-link,/opt/rocm/lib",
                        "-o", str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    run = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert run.returncode == 1 and "stub: no MuJoCo" in run.stdout, (run.returncode, run.stdout)
