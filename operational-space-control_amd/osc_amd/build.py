"""Build the in-tree native libraries: libosc_batch.so (HIP kernels for gfx950 + C-ABI + YAML
loader) and libosc_controller.so (the OperationalSpaceController shim over the C-ABI).

    python -m osc_amd.build          (from operational-space-control_amd/)

Plain hipcc, no cmake: five translation units.  The .so files land in
operational-space-control_amd/lib/ so that it travels to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
OUT = os.path.join(PKG_DIR, "lib", "libosc_batch.so")
OUT_CTRL = os.path.join(PKG_DIR, "lib", "libosc_controller.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("OSC_OFFLOAD_ARCH", "gfx950")

SOURCES = ["osc_batch.hip", "osc_model.cpp", "osc_mjcf.cpp", "osc_producers.hip",
           "osc_kinematics.hip"]


def build(verbose: bool = False, force: bool = False) -> str:
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    hdrs = [os.path.join(REPO, "include", h) for h in ("osc_batch.h", "osc_producers.h", "osc_kinematics.h")]
    if not force and os.path.exists(OUT):
        t_out = os.path.getmtime(OUT)
        if all(os.path.getmtime(p) <= t_out for p in srcs + hdrs + [__file__]):
            build_controller()
            build_tick_latency()
            return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cmd = [HIPCC, "-std=c++17", "-O3", f"--offload-arch={ARCH}", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-result", "-I", os.path.join(REPO, "include"),
           *srcs, "-o", OUT]
    if verbose:
        cmd.append("-Rpass-analysis=kernel-resource-usage")
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    build_controller(force=True)
    build_tick_latency(force=True)
    return OUT


OUT_TICK = os.path.join(PKG_DIR, "bin", "osc_tick_latency")


def build_tick_latency(force: bool = False) -> str:
    """Host program timing single-env ticks through the controller (BASELINE configs[0])."""
    src = os.path.join(CSRC, "osc_tick_latency.cpp")
    deps = [src, OUT_CTRL, os.path.join(REPO, "include", "osc_controller.h")]
    if not force and os.path.exists(OUT_TICK) and \
            all(os.path.getmtime(p) <= os.path.getmtime(OUT_TICK) for p in deps):
        return OUT_TICK
    os.makedirs(os.path.dirname(OUT_TICK), exist_ok=True)
    lib = os.path.dirname(OUT)
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-I", os.path.join(REPO, "include"), src,
                    "-L", lib, "-losc_controller", "-losc_batch", "-Wl,-rpath,$ORIGIN/../lib",
                    "-Wl,-rpath-link,/opt/rocm/lib", "-o", OUT_TICK], check=True)
    return OUT_TICK


def build_controller(force: bool = False) -> str:
    """Host-only C++ (HIP runtime API); links libosc_batch.so next to it via $ORIGIN."""
    src = os.path.join(CSRC, "osc_controller.cpp")
    hdrs = [os.path.join(REPO, "include", h) for h in ("osc_batch.h", "osc_controller.h")]
    if not force and os.path.exists(OUT_CTRL):
        t_out = os.path.getmtime(OUT_CTRL)
        if all(os.path.getmtime(p) <= t_out for p in [src, OUT] + hdrs):
            return OUT_CTRL
    cmd = [HIPCC, "-std=c++17", "-O2", "-fPIC", "-shared", "-Wall", "-Wno-unused-result",
           "-I", os.path.join(REPO, "include"), src, "-L", os.path.dirname(OUT), "-losc_batch",
           "-Wl,-rpath,$ORIGIN", "-o", OUT_CTRL]
    subprocess.run(cmd, check=True)
    return OUT_CTRL


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv, force="-f" in sys.argv))
