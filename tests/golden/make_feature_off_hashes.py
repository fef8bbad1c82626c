"""Bitwise fingerprints of the product's cold solve on fixed seeded batches (GPU only).

    OSC_LIB_PATH=<libosc_batch.so> python tests/golden/make_feature_off_hashes.py > out.json

Each entry is the SHA-256 of the bytes of (tau, x, status, iters) for one (robot, scenario,
mask, nenv, seed) batch.  tests/test_gpu_wheels.py checks that the current build reproduces
them, i.e. that models without wheel no-slip rows -- the feature-off path -- are bitwise what
they were.  History: made with the round-2 build; regenerated once in round 3 for the
intentional change of the LDL factor's storage (row k pre-scaled by -1/D_k, multiply-free
triangular solves: DESIGN.md §5), and again for the refinement rounds settling per env (an env
whose round ends without a violation keeps that round's result when a wave-mate asks for another
round: results no longer depend on which envs share a wavefront); the wheel rows' changes do not
reach models without them.  Regenerated once in round 4 (profiles/run_r04d.sh, in git history at cfe45c1) for the
refinement accepted on a KKT test instead of a per-lane move bound, the interior point's earlier
stops (Go2 eps_mu 1e-6, WaLTER 1e-8) and the multipliers of rows leaving the refinement's active
set zeroed.  Regenerated once in round 5 (profiles/run_r05h.sh) for the
refinement's one-change rounds (the most violated row joins, else the most negative multiplier
leaves: tests/golden/go2_unrefined_joint_states.npz).  Regenerated once in round 6 for the
interior point's carried dual residual (rd formed from scratch only where rp is: DESIGN.md §3.2), and again for the torque rows'
diagonal terms added to the pivots inside the factorisation.
Regenerate
only for an intentional numerical change of the default kernels, and say so in the commit.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))

CASES = [
    ("unitree_go2", "standing", "ones", 4096, 21),
    ("unitree_go2", "tumbling", "bernoulli", 8192, 22),
    ("walter_sr", "tumbling", "bernoulli", 4096, 23),
    ("walter_sr_wheels", "tumbling", "bernoulli", 1024, 24),
]


def fingerprint(solver, d) -> str:
    import torch
    res = solver.solve(**d, want_x=True)
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for t in (res.tau, res.x, res.status, res.iters):
        h.update(t.cpu().numpy().tobytes())
    return h.hexdigest()


def main() -> None:
    from osc_amd.solver import OSCBatchSolver
    from osc_amd.synth import SEED_BASE, generate
    out = {"lib": os.environ.get("OSC_LIB_PATH", "in-tree"), "cases": []}
    solvers = {}
    for robot, scen, mask, nenv, seed in CASES:
        if robot not in solvers:
            solvers[robot] = OSCBatchSolver(robot)
        d = generate(robot, nenv, SEED_BASE + seed, scen, mask)
        out["cases"].append({"robot": robot, "scenario": scen, "mask": mask, "nenv": nenv,
                             "seed": SEED_BASE + seed, "sha256": fingerprint(solvers[robot], d)})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
