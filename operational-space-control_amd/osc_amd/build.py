"""Build the in-tree native libraries: libosc_batch.so (HIP kernels for gfx950 + C-ABI + YAML
loader + kinematics + producers) and libosc_controller.so (the OperationalSpaceController shim
over the C-ABI).

    python -m osc_amd.build [-f] [-v]            (from operational-space-control_amd/)
    python -m osc_amd.build -f --out DIR -DFLAG  (a variant library for A/B timing or stamps)

Plain hipcc, no cmake: every translation unit compiles to its own object, in parallel (the
interior-point kernel is instantiated in one unit per robot model for that reason), then one
link.  The .so files land in operational-space-control_amd/lib/ so that they travel to the GPU
box with the repo snapshot.
"""
from __future__ import annotations

import concurrent.futures as cf
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

# kernel units (csrc/osc_device.hpp lists what each holds) + host units
SOURCES = ["osc_ipm_go2.hip", "osc_ipm_walter.hip", "osc_ipm_wheels.hip", "osc_multi.hip",
           "osc_setup.hip", "osc_gi.hip", "osc_dual.hip", "osc_kinematics.hip",
           "osc_producers.hip", "osc_api.hip", "osc_model.cpp", "osc_mjcf.cpp", "osc_host_feed.cpp"]
HEADERS = ["osc_device.hpp", "osc_internal.hpp", "osc_setup.hpp", "osc_ipm.hpp", "osc_ipm_asm.hpp",
           "osc_kin_device.hpp",
           "osc_qpos.hpp", "osc_wave_sum.hpp"]
# Per-unit compiler flags (variant builds may pass their own map to build()).  The interior-point
# units use LLVM's iterative ILP scheduler (round 6): bitwise the same results, faster per solve
# (profiles/r06/sched/); ldl_rows' column barrier keeps its schedule clear of DPP hazards
# (tests/test_asm_hazards.py compiles with these flags).  Not the assembly's unit: slower with it.
# The two-model unit (configs[4]'s pair kernels) too: mixed 24.09 -> 24.75 M solves/s, its GPU tests
# bitwise against the solo solves (profiles/r06/sched/multi/).
_ILP = ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]
UNIT_FLAGS: dict = {"osc_ipm_go2.hip": _ILP, "osc_ipm_walter.hip": _ILP, "osc_ipm_wheels.hip": _ILP,
              "osc_multi.hip": _ILP}
# device-code units, for the static checks that read the generated assembly
DEVICE_SOURCES = [s for s in SOURCES if s.endswith(".hip")]


def _jobs() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:   # pragma: no cover
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def compile_flags(defines=()) -> list:
    return ["-std=c++17", "-O3", f"--offload-arch={ARCH}", "-fPIC", "-Wall", "-Wno-unused-result",
            "-I", os.path.join(REPO, "include"), *defines]


def build(verbose: bool = False, force: bool = False, out: str | None = None,
          defines=(), unit_flags: dict | None = None) -> str:
    out = out or OUT
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    deps = srcs + [os.path.join(CSRC, h) for h in HEADERS] + \
        [os.path.join(REPO, "include", h) for h in ("osc_batch.h", "osc_producers.h",
                                                     "osc_kinematics.h", "osc_host_feed.h")] + [__file__]
    variant = out != OUT
    if not force and os.path.exists(out):
        t_out = os.path.getmtime(out)
        if all(os.path.getmtime(p) <= t_out for p in deps):
            if not variant:
                build_controller()
                build_tick_latency()
            return out
    objdir = os.path.join(os.path.dirname(out), "obj")
    os.makedirs(objdir, exist_ok=True)
    flags = compile_flags(defines)
    if verbose:
        flags.append("-Rpass-analysis=kernel-resource-usage")

    def compile_one(src):
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        extra = (UNIT_FLAGS if unit_flags is None else unit_flags).get(os.path.basename(src), [])
        cmd = [HIPCC, *flags, *extra, "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        return obj

    with cf.ThreadPoolExecutor(max_workers=_jobs()) as ex:
        objs = list(ex.map(compile_one, srcs))
    subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", out],
                   check=True)
    if not variant:
        build_controller(force=True)
        build_tick_latency(force=True)
    return out


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


def main(argv) -> None:
    out, defines = None, []
    it = iter(argv)
    for a in it:
        if a == "--out":
            out = os.path.join(next(it), "libosc_batch.so")
        elif a.startswith("-D"):
            defines.append(a)
    print(build(verbose="-v" in argv, force="-f" in argv, out=out, defines=defines))


if __name__ == "__main__":
    main(sys.argv[1:])
