"""Diagnostic (GPU): A/B of osc_model_tuning settings on one batch -- kernel time per solve (HIP
events around 30 launches), status counts, interior-point iterations, and the normwise torque
difference against the first setting.  Replaces the OSC_* environment-variable sweeps of rounds
1-3 (the release library reads no environment).

    python tools/tune_ab.py ROBOT NENV SCENARIO MASK '{"eps_mu": 1e-9}' '{"eps_mu": 1e-6}' ...
    (SCENARIO standing|tumbling|qpos<range>: joint states through the GPU kinematics;
     OSC_AB_ROUNDS=R: R interleaved rounds over the settings, the median time per setting -- one
     round's first setting also pays the clocks' ramp)
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from osc_amd.dist import shard_seed  # noqa: E402
from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import SEED_BASE, generate  # noqa: E402


def inputs(robot, nenv, scenario, mask_mode):
    if scenario.startswith("qpos"):
        from osc_amd.kinematics import KinematicsBatch, load_tree, random_states
        tree = load_tree(robot)
        seed = shard_seed(0) + 7
        qpos, qvel = random_states(tree, nenv, seed, joint_range=float(scenario[4:] or 0.5))
        d = generate(robot, nenv, seed, "standing", mask_mode)
        k = KinematicsBatch(tree=tree).compute(qpos, qvel, want_sites=False)
        return dict(M=k.M, C=k.C, J=k.J, b=k.b, T=d["T"], mask=d["mask"])
    return generate(robot, nenv, SEED_BASE + 2, scenario, mask_mode)


def main():
    robot, nenv, scenario, mask_mode = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4]
    tunings = [json.loads(a) for a in sys.argv[5:]] or [{}]
    d = inputs(robot, nenv, scenario, mask_mode)
    ref = None
    rounds = int(os.environ.get("OSC_AB_ROUNDS", "1"))
    solvers = [OSCBatchSolver(robot, tuning=tn) for tn in tunings]
    argss = [s.prepare(**d) for s in solvers]
    outs = [s.alloc_outputs(nenv) for s in solvers]
    times = [[] for _ in tunings]
    for _ in range(rounds):
        for k, s in enumerate(solvers):
            for _ in range(5):
                s.solve_into(outs[k], *argss[k])
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(30):
                s.solve_into(outs[k], *argss[k])
            b.record()
            torch.cuda.synchronize()
            times[k].append(a.elapsed_time(b) / 30)
    for k, tn in enumerate(tunings):
        s, out = solvers[k], outs[k]
        tau = out.tau.cpu().numpy()
        st = out.status.cpu().numpy()
        it = out.iters.cpu().numpy()
        row = {"robot": robot, "nenv": nenv, "scenario": scenario, "tuning": tn,
               "ms": round(float(np.median(times[k])), 4), "ms_rounds": [round(t, 4) for t in times[k]],
               "status": {int(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
               "iters_mean": round(float(it.mean()), 3), "iters_max": int(it.max()),
               "wave_iters_mean": round(float(np.max(np.reshape(it[:nenv // 4 * 4], (-1, 4)), 1).mean()), 3)}
        if ref is None:
            ref = tau
        else:
            nrm = np.maximum(np.abs(ref).max(axis=1), 1.0)
            row["vs_first_normwise_max"] = float((np.abs(tau - ref).max(axis=1) / nrm).max())
        print(json.dumps(row), flush=True)
        s.close()


if __name__ == "__main__":
    main()
