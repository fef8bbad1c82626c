"""Static check of the IPM kernels' inline-asm DPP statements (CPU only: cross-compiles gfx950).

hipcc's hazard recognizer does not look inside inline asm, so every DPP read of a VGPR that a
VALU instruction wrote must be padded by the asm itself (osc_device.hpp: fmac_bcast<K, NOP>,
bcast_guarded).  tools/check_dpp_hazards.py walks the generated listing and fails on any DPP
source written by a VALU instruction less than 2 wait states earlier."""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
from osc_amd.build import UNIT_FLAGS  # noqa: E402

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None,
                    reason="hipcc not available")
@pytest.mark.parametrize("unit", ["osc_ipm_go2", "osc_ipm_walter", "osc_ipm_wheels", "osc_multi",
                                  "osc_setup", "osc_dual", "osc_gi"])
def test_no_dpp_hazards_in_kernels(tmp_path, unit):
    out = tmp_path / f"{unit}.s"
    src = os.path.join(REPO, "operational-space-control_amd", "csrc", f"{unit}.hip")
    subprocess.run([HIPCC, "-std=c++17", "-O3", "--offload-arch=gfx950", "--cuda-device-only",
                    *UNIT_FLAGS.get(f"{unit}.hip", []),   # the flags the product build uses
                    "-S", "-I", os.path.join(REPO, "include"), "-o", str(out), src],
                   check=True, capture_output=True)
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "check_dpp_hazards.py"),
                        str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:]
    assert "0 DPP hazards" in r.stdout
