"""EVERY env of the BASELINE single-GPU batches against the exact oracle.

configs[1] (Go2 standing, 4,096 envs) and configs[2] (WaLTER Sr standing, 4,096 envs), the
bench's own batches (seed shard_seed(0), osc_amd.synth.generate): the HIP path's torques through
the C-ABI (osc_batch_solve) against the exact optimum of the reference QP (oracle/qp_exact.py on
oracle/osc_qp.build_qp -- unitree_go2/autogen/autogen.py:58-319 stacked as
operational_space_controller.h:483-497, torque slice :573), solved for every env over a host
process pool (oracle/parallel.py).  The joint-state batches get the same treatment in
tests/test_gpu_joint_states.py.

Tolerances (tests/test_gpu_parity.py): contract 1e-5 normwise and elementwise above the 1 %
floor; achieved bars normwise <= 1e-9, elementwise <= 1e-7.  The worst env is printed (pytest -s).
Tumbling configs[3] batches (8,192 envs, masks redrawn) get the same check on every env too.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from osc_amd.dist import shard_seed
from osc_amd.synth import generate
from osc_qp import load_model
from parallel import solve_batch
from test_gpu_parity import ELEM_ACH, NORM_ACH, _check, _rel_errors, solver

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("robot,nenv,scenario,mask_mode,seed", [
    ("unitree_go2", 4096, "standing", "ones", shard_seed(0)),      # configs[1], the bench batch
    ("walter_sr", 4096, "standing", "ones", shard_seed(0)),        # configs[2]
    ("walter_sr", 8192, "tumbling", "bernoulli", shard_seed(0)),   # configs[3] (first step's masks)
])
def test_every_env_vs_oracle(gpu, robot, nenv, scenario, mask_mode, seed):
    d = generate(robot, nenv, seed, scenario, mask_mode)
    res = solver(robot).solve(**d, want_x=True)
    torch.cuda.synchronize()
    st = res.status.cpu().numpy()
    assert (st == 0).all(), (np.bincount(st), np.nonzero(st)[0][:20])
    model = load_model(robot)
    xo, cert = solve_batch(robot, d["M"], d["C"], d["J"], d["b"], d["T"], d["mask"])
    tau_ref = xo[:, model.nv:model.nv + model.nu]
    nw, el = _rel_errors(res.tau.cpu().numpy(), tau_ref)
    x = res.x.cpu().numpy()
    nx = (np.abs(x - xo) / np.maximum(np.abs(xo).max(axis=1, keepdims=True), 1.0)).max(axis=1)
    print(f"\n{robot} {scenario} {nenv} envs: every env vs the exact oracle (worst oracle KKT "
          f"residual {cert.max():.1e}): torques worst normwise {nw.max():.2e} (env "
          f"{int(np.argmax(nw))}), worst elementwise {el.max():.2e} (env {int(np.argmax(el))}); "
          f"design vector worst normwise {nx.max():.2e}")
    _check(nw, el, robot)
    assert nw.max() <= NORM_ACH and el.max() <= ELEM_ACH
