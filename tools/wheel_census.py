"""Diagnostic (GPU): census of the opt-in wheel no-slip rows on one batch -- status counts, the
OSQP-form KKT certificate of every env reported OK (tests/test_gpu_wheels._kkt), and for the envs
not reported OK (or OK but not certified) their status, iterations and torque error against the
exact oracle.  One parameterised tool in place of round 3's wheel_* one-offs.

    python tools/wheel_census.py [nenv] [seed] [scenario] [mask] [warm_ticks] [tuning-json] [--brief]
(--brief: the per-tick summary lines only, no oracle solves; --dump=OUT.npz: x, y, status and the
inputs of every env not certified, for a CPU look at its certificate)
"""
import hashlib
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("operational-space-control_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, p))
import torch  # noqa: E402

from osc_amd.robots import config_path  # noqa: E402
from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import (SEED_BASE, WALTER_WHEEL_DOFS, WHEEL_RADIUS, generate,  # noqa: E402
                           random_walk, wheel_directions)
from osc_qp import WheelRows, build_qp, load_model, torque  # noqa: E402
from qp_exact import solve_exact  # noqa: E402
from test_gpu_wheels import KKT_COMP, KKT_DUAL, KKT_PRIMAL, KKT_STAT, _batched_qp, _kkt  # noqa: E402

YAML = os.path.join(os.path.dirname(config_path("walter_sr_wheels")),
                    "walter_sr_wheels_noslip_config.yaml")


def main():
    brief = "--brief" in sys.argv
    dump = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--dump=")), None)
    sys.argv = [a for a in sys.argv if a != "--brief" and not a.startswith("--dump=")]
    dumps = {}
    nenv = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    seed = SEED_BASE + (int(sys.argv[2]) if len(sys.argv) > 2 else 86)
    scenario = sys.argv[3] if len(sys.argv) > 3 else "tumbling"
    mask_mode = sys.argv[4] if len(sys.argv) > 4 else "bernoulli"
    ticks = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    tuning = json.loads(sys.argv[6]) if len(sys.argv) > 6 else None
    model = load_model("walter_sr_wheels")
    wheel = WheelRows(dof=np.array(WALTER_WHEEL_DOFS), radius=np.full(8, WHEEL_RADIUS))
    tn = dict(tuning or {})
    max_iter = tn.pop("max_iter", None)   # (a descriptor field, not osc_model_tuning)
    s = OSCBatchSolver("walter_sr_wheels", YAML, max_iter=max_iter, tuning=tn or None)
    d = generate("walter_sr_wheels", nenv, seed, scenario, mask_mode)
    rng = np.random.default_rng(seed)
    warm = s.alloc_warm_state(nenv) if ticks > 1 else None
    for tick in range(ticks):
        wd = wheel_directions("walter_sr_wheels", d, wheel.dof, wheel.radius, seed + 1)
        args = s.prepare(**d)
        wdt = torch.from_numpy(wd).cuda()
        out = s.alloc_outputs(nenv, want_y=True)
        if warm is None:
            s.solve_into(out, *args, wheel_dir=wdt)
        else:
            s.solve_warm_into(out, warm, *args, wheel_dir=wdt)
        torch.cuda.synchronize()
        ms = None
        if brief and warm is None:   # time 10 cold solves of this batch (HIP events)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(10):
                s.solve_into(out, *args, wheel_dir=wdt)
            ev[1].record()
            torch.cuda.synchronize()
            ms = ev[0].elapsed_time(ev[1]) / 10
        st = out.status.cpu().numpy()
        cert = _kkt(*_batched_qp("walter_sr_wheels", *args, wheel, wdt), out.x, out.y)
        good = torch.ones(nenv, dtype=torch.bool, device=out.x.device)
        worst = {}
        for k, tol in (("stationarity", KKT_STAT), ("primal", KKT_PRIMAL), ("dual", KKT_DUAL),
                       ("complementarity", KKT_COMP)):
            good &= cert[k] <= tol
            worst[k] = float(cert[k][torch.from_numpy(st == 0).cuda()].max().item()) if (st == 0).any() else 0.0
        good = good.cpu().numpy()
        row = {"tick": tick, "nenv": nenv, "seed": seed, "scenario": scenario, "tuning": tuning,
               "status": {int(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
               "ok_uncertified": int(((st == 0) & ~good).sum()), "worst_cert_of_ok": worst,
               "iters_mean": float(out.iters.float().mean().item()),
               "iters_max": int(out.iters.max().item()), "ms": ms,
               "tau_x_sha": hashlib.sha1(out.tau.cpu().numpy().tobytes() +
                                         out.x.cpu().numpy().tobytes()).hexdigest()[:16],
               "y_sha": hashlib.sha1(out.y.cpu().numpy().tobytes()).hexdigest()[:16]}
        print(json.dumps(row), flush=True)
        tau = out.tau.cpu().numpy()
        it = out.iters.cpu().numpy()
        if dump:
            for e in np.nonzero(~good)[0]:
                key = f"t{tick}_e{e}"
                dumps[key + "_x"] = out.x[e].cpu().numpy()
                dumps[key + "_y"] = out.y[e].cpu().numpy()
                dumps[key + "_wd"] = wd[e]
                for k in ("M", "C", "J", "b", "T", "mask"):
                    dumps[f"{key}_{k}"] = np.asarray(d[k][e])
        for e in [] if brief else np.nonzero((st != 0) | ~good)[0][:24]:
            a = [d[k][e] for k in ("M", "C", "J", "b", "T", "mask")]
            ref = torque(model, solve_exact(model, build_qp(model, *a, wheel, wd[e]), *a[:3]).x)
            err = float(np.abs(tau[e] - ref).max() / max(np.abs(ref).max(), 1.0))
            print(json.dumps({"tick": tick, "env": int(e), "status": int(st[e]), "iters": int(it[e]),
                              "certified": bool(good[e]), "err": err,
                              "cert": {k: float(v[e].item()) for k, v in cert.items()},
                              "ncontact": int(d["mask"][e].sum())}), flush=True)
        d = random_walk(d, rng)
    if dump:
        np.savez(dump, **dumps)


if __name__ == "__main__":
    main()
