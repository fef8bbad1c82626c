"""Static per-robot facts used by the host side (dimensions, site order, synthetic structure).

The numeric model (weights, friction, bounds) is owned by the native library
(csrc/osc_model.cpp), which reads the reference's YAML schema at run time.  This table only
carries what the Python host needs to size buffers and to synthesise inputs.

  unitree_go2 : nv 18, nu 12, 4 contacts, 5 sites   (unitree_go2/autogen/autogen.py:44-56)
  walter_sr   : nv 14, nu 8, 8 contacts, 17 sites    (walter_sr/autogen/autogen.py:44-60)
"""
from __future__ import annotations

import os

CONFIG_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "config")


def _walter_site_dofs():
    base = list(range(6))
    leg = lambda l: [6 + 2 * l, 7 + 2 * l]
    dofs = [base]
    dofs += [base + leg(l) for l in range(4)]            # shins
    dofs += [base + leg(l)[:1] for l in range(4)]        # thighs
    dofs += [base + leg(l // 2) for l in range(8)]       # wheels (2 per leg)
    return dofs


_WALTER_SITES = ["torso", "tls", "trs", "hls", "hrs", "tlh", "trh", "hlh", "hrh",
                 "tlf", "tlr", "trf", "trr", "hlf", "hlr", "hrf", "hrr"]

ROBOTS = {
    "unitree_go2": dict(
        nv=18, nu=12, nc=4, site_keys=["base", "fr", "fl", "hr", "hl"],
        config="unitree_go2_config.yaml", base_mass=15.0,
        site_dofs=[list(range(6))] + [list(range(6)) + list(range(6 + 3 * l, 9 + 3 * l)) for l in range(4)],
    ),
    "walter_sr": dict(
        nv=14, nu=8, nc=8, site_keys=_WALTER_SITES, config="walter_sr_config.yaml",
        base_mass=10.0, site_dofs=_walter_site_dofs(),
    ),
    "walter_sr_wheels": dict(
        nv=14, nu=8, nc=8, site_keys=_WALTER_SITES, config="walter_sr_wheels_config.yaml",
        base_mass=10.0, site_dofs=_walter_site_dofs(),
    ),
}


def dims(robot: str) -> dict:
    r = ROBOTS[robot]
    ns = len(r["site_keys"])
    nz = 3 * r["nc"]
    n = r["nv"] + r["nu"] + nz
    return dict(nv=r["nv"], nu=r["nu"], nc=r["nc"], ns=ns, s=6 * ns, nz=nz, n=n,
                m=r["nv"] + 4 * r["nc"] + n)


def config_path(robot: str) -> str:
    return os.path.join(CONFIG_DIR, ROBOTS[robot]["config"])


def bytes_per_solve(robot: str) -> int:
    """Algorithmic HBM bytes per solve: inputs M, C, J, b, T, mask + output tau."""
    d = dims(robot)
    return 8 * (d["nv"] ** 2 + d["nv"] + d["s"] * d["nv"] + d["s"] + 6 * d["ns"] + d["nc"] + d["nu"])
