"""MI355X-native batched operational-space-control (OSC) solver -- host side.

The solve runs in HIP kernels for gfx950 behind the C-ABI in include/osc_batch.h
(libosc_batch.so, built in-tree by osc_amd.build).  Importing this package does not need a GPU;
creating an OSCBatchSolver does.
"""
from .robots import ROBOTS, dims, config_path, bytes_per_solve  # noqa: F401
from . import synth  # noqa: F401


def __getattr__(name):
    # torch-dependent pieces load lazily so CPU-only tooling stays light
    if name in ("OSCBatchSolver", "SolveResult"):
        from . import solver
        return getattr(solver, name)
    raise AttributeError(name)
