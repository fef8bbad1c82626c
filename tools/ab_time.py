"""A/B kernel timing of the cold solve for builds of libosc_batch.so given on the command line
(raw ctypes: only osc_desc_from_yaml / osc_model_create / osc_workspace_bytes / osc_batch_solve,
so older builds load too).  Diagnostic only.

    python tools/ab_time.py lib1.so [lib2.so ...]
    AB_CONFIGS="unitree_go2:4096,unitree_go2:8192"   configurations (default Go2 4,096 / 65,536,
                                                     WaLTER 4,096); AB_ONLY=one of them (rocprof)
    AB_ROUNDS=R      R interleaved rounds over the libraries (default 3); every round times 30
                     solves per library after 5 warmup solves; the JSON lines give each round,
                     the summary line the median per library and configuration
    AB_CHECK=1       also compare each library's torques with the first one's (bitwise flag)
    AB_WARM=1        warm-started ticks instead (osc_batch_solve_warm, the warm state carried,
                     inputs alternating between the batch and a 1 % perturbed copy)
"""
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "operational-space-control_amd"))
import torch  # noqa: E402

from osc_amd._lib import OscModelDesc  # noqa: E402
from osc_amd.robots import config_path  # noqa: E402
from osc_amd.synth import SEED_BASE, generate  # noqa: E402

vp = ctypes.c_void_p


def configs():
    only = os.environ.get("AB_ONLY")
    spec = os.environ.get("AB_CONFIGS", "unitree_go2:4096,unitree_go2:65536,walter_sr:4096")
    out = []
    for c in spec.split(","):
        if only and only != c:
            continue
        robot, nenv = c.split(":")
        out.append((robot, int(nenv)))
    return out


class Lib:
    def __init__(self, path):
        self.path = path
        self.L = ctypes.CDLL(path)
        self.L.osc_batch_solve.argtypes = [vp, ctypes.c_int32] + [vp] * 10 + [vp, ctypes.c_size_t, vp]
        self.L.osc_batch_solve_warm.argtypes = [vp, ctypes.c_int32] + [vp] * 10 + \
            [vp, ctypes.c_size_t, vp, ctypes.c_size_t, vp]
        self.models = {}

    def model(self, robot):
        if robot not in self.models:
            d = OscModelDesc()
            assert self.L.osc_desc_from_yaml(robot.encode(), config_path(robot).encode(),
                                             ctypes.byref(d)) == 0
            h = vp()
            assert self.L.osc_model_create(ctypes.byref(d), ctypes.byref(h)) == 0
            self.models[robot] = h
        return self.models[robot]


def main():
    libs = [Lib(p) for p in sys.argv[1:]]
    rounds = int(os.environ.get("AB_ROUNDS", "3"))
    check = os.environ.get("AB_CHECK") == "1"
    warm_mode = os.environ.get("AB_WARM") == "1"
    times = {}
    for robot, nenv in configs():
        g = generate(robot, nenv, SEED_BASE + 2)
        t = [torch.from_numpy(g[k]).cuda().contiguous() for k in ("M", "C", "J", "b", "T", "mask")]
        p = [vp(x.data_ptr()) for x in t]
        gen = torch.Generator(device="cuda").manual_seed(5)
        t2 = [x if i == 5 else (x * (1.0 + 0.01 * torch.randn(x.shape, generator=gen, device="cuda",
                                                               dtype=x.dtype))).contiguous()
              for i, x in enumerate(t)]
        # M by a congruence A M A' (SPD kept; an elementwise 1 % perturbation made ~1 % of the
        # WaLTER M indefinite or near-singular: unphysical QPs the reduction flags)
        nv = t[0].shape[1]
        A = torch.eye(nv, dtype=torch.float64, device="cuda") + 0.01 / nv ** 0.5 * torch.randn(
            t[0].shape, generator=gen, device="cuda", dtype=torch.float64)
        t2[0] = A @ t[0] @ A.transpose(1, 2)
        t2[0] = (0.5 * (t2[0] + t2[0].transpose(1, 2))).contiguous()
        p2 = [vp(x.data_ptr()) for x in t2]
        nu = {"unitree_go2": 12, "walter_sr": 8}[robot]
        taus = []
        for lib in libs:
            nb = ctypes.c_size_t()
            lib.L.osc_workspace_bytes(lib.model(robot), nenv, ctypes.byref(nb))
            lib.ws = torch.empty((nb.value // 8 + 2,), dtype=torch.float64, device="cuda")
            lib.tau = torch.empty((nenv, nu), dtype=torch.float64, device="cuda")
            if warm_mode:
                wb = ctypes.c_size_t()
                lib.L.osc_warm_state_bytes(lib.model(robot), nenv, ctypes.byref(wb))
                lib.warm = torch.zeros((wb.value // 8 + 2,), dtype=torch.float64, device="cuda")
                lib.tick = 0
        for r in range(rounds):
            for lib in libs:
                h = lib.model(robot)

                def call():
                    if warm_mode:
                        lib.tick += 1
                        rc = lib.L.osc_batch_solve_warm(
                            h, nenv, *(p if lib.tick % 2 else p2), vp(lib.tau.data_ptr()), None,
                            None, None, vp(lib.warm.data_ptr()),
                            ctypes.c_size_t(lib.warm.numel() * 8), vp(lib.ws.data_ptr()),
                            ctypes.c_size_t(lib.ws.numel() * 8),
                            vp(torch.cuda.current_stream().cuda_stream))
                    else:
                        rc = lib.L.osc_batch_solve(h, nenv, *p, vp(lib.tau.data_ptr()), None, None,
                                                   None, vp(lib.ws.data_ptr()),
                                                   ctypes.c_size_t(lib.ws.numel() * 8),
                                                   vp(torch.cuda.current_stream().cuda_stream))
                    assert rc == 0
                for _ in range(5):
                    call()
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(30):
                    call()
                b.record()
                torch.cuda.synchronize()
                ms = a.elapsed_time(b) / 30
                times.setdefault((lib.path, robot, nenv), []).append(ms)
                print(json.dumps({"lib": lib.path[-45:], "robot": robot, "nenv": nenv, "round": r,
                                  "ms": round(ms, 4)}), flush=True)
        if check:
            ref = libs[0].tau
            for lib in libs[1:]:
                print(json.dumps({"lib": lib.path[-45:], "robot": robot, "nenv": nenv,
                                  "bitwise_equal_to_first": bool(torch.equal(ref, lib.tau))}),
                      flush=True)
    for (path, robot, nenv), ms in times.items():
        print(json.dumps({"summary": True, "lib": path[-45:], "robot": robot, "nenv": nenv,
                          "median_ms": round(statistics.median(ms), 4),
                          "min_ms": round(min(ms), 4), "rounds": len(ms)}), flush=True)


if __name__ == "__main__":
    main()
