"""The wheel-row fallback's algorithm on the CPU (tools/gi_fallback_model.py restates osc_gi_kernel's
sequence in numpy): on the envs the GPU interior point leaves at max_iter (round-4 census, seed
offset 86) and on ordinary ones, its torques match the exact oracle and its iterate holds every
equality row -- the check that the restated method itself is right, independent of the GPU."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in ("tools", "oracle", "operational-space-control_amd"):
    sys.path.insert(0, os.path.join(REPO, p))

from gi_fallback_model import gi_full, rows_of  # noqa: E402
from osc_amd.synth import SEED_BASE, WALTER_WHEEL_DOFS, WHEEL_RADIUS, generate, wheel_directions  # noqa: E402
from osc_qp import WheelRows, build_qp, load_model, torque  # noqa: E402
from qp_exact import solve_exact  # noqa: E402


@pytest.mark.parametrize("envs", [(37, 357, 1157), (0, 9, 18)])
def test_gi_full_qp_matches_oracle(envs):
    model = load_model("walter_sr_wheels")
    wheel = WheelRows(dof=np.array(WALTER_WHEEL_DOFS), radius=np.full(8, WHEEL_RADIUS))
    d = generate("walter_sr_wheels", 2048, SEED_BASE + 86, "tumbling", "bernoulli")
    wd = wheel_directions("walter_sr_wheels", d, wheel.dof, wheel.radius, SEED_BASE + 87)
    for e in envs:
        a = [d[k][e] for k in ("M", "C", "J", "b", "T", "mask")]
        qp = build_qp(model, *a, wheel, wd[e])
        cs, bs, eqs = rows_of(qp, model.n, model)
        x, act, steps, ok = gi_full(qp.H, qp.f, cs, bs, eqs)
        assert ok, (e, steps)
        eq_res = max(abs(cs[k] @ x - bs[k]) / (1 + abs(bs[k])) for k in range(int(eqs.sum())))
        assert eq_res <= 1e-9, (e, eq_res)
        ref = torque(model, solve_exact(model, qp, *a[:3]).x)
        err = np.abs(torque(model, x) - ref).max() / max(np.abs(ref).max(), 1.0)
        assert err <= 1e-9, (e, err)
