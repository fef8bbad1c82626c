"""Per-kernel register / scratch / occupancy table of a HIP source, from the compiler's
kernel-resource-usage remarks (no GPU needed).

    python tools/kernel_resources.py [operational-space-control_amd/csrc/osc_ipm_go2.hip] [-D...]
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
from osc_amd.build import UNIT_FLAGS  # noqa: E402


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names),
                         capture_output=True, text=True).stdout.splitlines()
    return out if len(out) == len(names) else names


def main(argv):
    src = next((a for a in argv[1:] if not a.startswith("-")),
               os.path.join(REPO, "operational-space-control_amd", "csrc", "osc_ipm_go2.hip"))
    defs = [a for a in argv[1:] if a.startswith("-D")]
    with tempfile.TemporaryDirectory() as td:
        r = subprocess.run(["/opt/rocm/bin/hipcc", "-std=c++17", "-O3", "--offload-arch=gfx950",
                            "-fPIC", "-c", "--cuda-device-only", "-I", os.path.join(REPO, "include"),
                            *defs, *UNIT_FLAGS.get(os.path.basename(src), []), src, "-o", os.path.join(td, "k.o"),
                            "-Rpass-analysis=kernel-resource-usage"],
                           capture_output=True, text=True)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy "
                      r"\[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
        if not m:
            continue
        k, v = m.group(1), m.group(2)
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k.split()[0]] = v
    names = demangle([x["name"] for x in rows])
    for x, n in zip(rows, names):
        n = n.replace("(anonymous namespace)::", "").split("(")[0]
        print(f"{x.get('VGPRs', '?'):>4} v {x.get('AGPRs', '?'):>4} a {x.get('ScratchSize', '?'):>5} "
              f"scr {x.get('Occupancy', '?'):>2} occ {x.get('LDS', '?'):>6} lds  {n}")
    if r.returncode != 0:
        print(r.stderr[-2000:])
    return r.returncode


if __name__ == "__main__":
    sys.exit(main(sys.argv))
