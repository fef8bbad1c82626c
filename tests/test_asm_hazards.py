"""Static check of the IPM kernels' inline-asm DPP statements (CPU only: cross-compiles gfx950).

hipcc's hazard recognizer does not look inside inline asm, so every DPP read of a VGPR that a
VALU instruction wrote must be padded by the asm itself (osc_batch.hip: fmac_bcast<K, NOP>,
bcast_guarded).  tools/check_dpp_hazards.py walks the generated listing and fails on any DPP
source written by a VALU instruction less than 2 wait states earlier."""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None,
                    reason="hipcc not available")
def test_no_dpp_hazards_in_kernels(tmp_path):
    out = tmp_path / "osc_batch.s"
    src = os.path.join(REPO, "operational-space-control_amd", "csrc", "osc_batch.hip")
    subprocess.run([HIPCC, "-std=c++17", "-O3", "--offload-arch=gfx950", "--cuda-device-only",
                    "-S", "-I", os.path.join(REPO, "include"), "-o", str(out), src],
                   check=True, capture_output=True)
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "check_dpp_hazards.py"),
                        str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:]
    assert "0 DPP hazards" in r.stdout
