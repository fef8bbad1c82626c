"""Diagnostic (CPU): exact-oracle torques of every env of one seeded synthetic batch, saved for
tools/dump_tau.py's on-box comparison (so sweeps ship back per-env errors, not torques).
Usage: python tools/ref_tau.py robot scenario mask nenv seed_offset out.npz [workers]"""
import multiprocessing as mp
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from hardest_envs import init, ref  # noqa: E402

if __name__ == "__main__":
    robot, scenario, mask, nenv, off, out = sys.argv[1:7]
    workers = int(sys.argv[7]) if len(sys.argv) > 7 else os.cpu_count()
    with mp.Pool(workers, initializer=init,
                 initargs=(robot, scenario, mask, int(nenv), int(off))) as p:
        refs = np.array(p.map(ref, range(int(nenv)), chunksize=64))
    np.savez(out, tau=refs)
    print("saved", out, refs.shape)
