"""Random kinematic trees (test data) in the <robot>_kinematics.json schema.

The illustrative Go2 / WaLTER trees have identity body quaternions, zero joint anchors and
diagonal inertias; these exercise every term the kernel and the oracle carry: rotated body
frames, hinge anchors off the body origin, rotated principal axes, welded bodies, non-unit
axes, armature, a fixed-base (hinge-rooted) variant and deeper chains."""
import numpy as np


def _unit_quat(rng):
    q = rng.standard_normal(4)
    return list(q / np.linalg.norm(q))


def random_tree(seed: int, nbody: int = 11, free_root: bool = True, nsite: int = 9,
                weld_p: float = 0.15) -> dict:
    rng = np.random.default_rng(seed)
    bodies = []
    for i in range(nbody):
        if i == 0:
            parent, joint = -1, ("free" if free_root else "hinge")
        else:
            parent = int(rng.integers(0, i))
            joint = "none" if rng.uniform() < weld_p else "hinge"
        bodies.append(dict(
            name=f"b{i}", parent=parent, pos=list(0.2 * rng.standard_normal(3)),
            quat=_unit_quat(rng), joint=joint,
            axis=list(rng.standard_normal(3) * rng.uniform(0.5, 2.0)),
            jnt_pos=list(0.05 * rng.standard_normal(3)),
            armature=float(rng.uniform(0.0, 0.05)) if joint != "free" else 0.0,
            mass=float(rng.uniform(0.2, 3.0)), ipos=list(0.05 * rng.standard_normal(3)),
            iquat=_unit_quat(rng), diaginertia=list(rng.uniform(1e-3, 2e-2, size=3))))
    sites = [dict(name=f"s{k}", body=int(rng.integers(0, nbody)),
                  pos=list(0.1 * rng.standard_normal(3))) for k in range(nsite)]
    return dict(name=f"random tree {seed}", gravity=[0.0, 0.0, -9.81], bodies=bodies,
                sites=sites)


def chain_tree(seed: int, nbody: int = 16) -> dict:
    """A single 15-hinge chain under a free root: the deepest tree the kernel allows."""
    t = random_tree(seed, nbody=nbody, nsite=12, weld_p=0.0)
    for i, b in enumerate(t["bodies"][1:], start=1):
        b["parent"] = i - 1
    return t


def free_body(mass=2.0, diag=(0.1, 0.2, 0.3), iquat=(1.0, 0.0, 0.0, 0.0)) -> dict:
    """A single free body with its COM at the body origin and one site there."""
    return dict(name="free body", gravity=[0.0, 0.0, -9.81], bodies=[dict(
        name="b", parent=-1, pos=[0, 0, 0], quat=[1, 0, 0, 0], joint="free", axis=[0, 0, 1],
        jnt_pos=[0, 0, 0], armature=0.0, mass=mass, ipos=[0, 0, 0], iquat=list(iquat),
        diaginertia=list(diag))], sites=[dict(name="s", body=0, pos=[0, 0, 0])])


def pendulum(mass=1.5, length=0.7, izz=1e-3, armature=0.05) -> dict:
    """A point-like mass on a hinge about the world y axis, COM at -length along z, welded to the
    world (fixed base), one site at the COM."""
    return dict(name="pendulum", gravity=[0.0, 0.0, -9.81], bodies=[dict(
        name="arm", parent=-1, pos=[0, 0, 0], quat=[1, 0, 0, 0], joint="hinge", axis=[0, 1, 0],
        jnt_pos=[0, 0, 0], armature=armature, mass=mass, ipos=[0, 0, -length],
        iquat=[1, 0, 0, 0], diaginertia=[izz, izz, izz])],
        sites=[dict(name="bob", body=0, pos=[0, 0, -length])])


def mixed_tree(seed: int, nbody: int = 12, nsite: int = 9, free_root: bool = True) -> dict:
    """A random tree whose joints mix hinge, slide and ball (one per body: the JSON schema and
    the kernel's descriptor), with welded bodies."""
    t = random_tree(seed, nbody=nbody, nsite=nsite, free_root=free_root, weld_p=0.1)
    kinds = ["slide", "ball", "hinge"]
    for i, b in enumerate(t["bodies"][1:]):
        if b["joint"] != "none":
            b["joint"] = kinds[(i + seed) % 3]
    return t


def multi_joint_tree(seed: int, nbody: int = 8, nsite: int = 8) -> dict:
    """A random tree whose bodies carry MuJoCo-style joint lists ("joints": applied in order):
    hinge / slide pairs and triples, a ball as the last rotating joint of a body, single joints
    and a welded body.  The oracle reads the lists directly; the MJCF reader splits each such
    body into a chain (osc_mjcf.cpp)."""
    t = random_tree(seed, nbody=nbody, nsite=nsite, weld_p=0.0)
    rng = np.random.default_rng(2000 + seed)
    patterns = [["hinge", "hinge"], ["slide", "hinge"], ["hinge", "slide", "hinge"],
                ["hinge", "ball"], ["ball", "slide"], ["slide", "slide"], ["hinge"], ["none"]]
    for i, b in enumerate(t["bodies"][1:], start=1):
        pat = patterns[(i - 1 + seed) % len(patterns)]
        if pat == ["none"]:
            b["joint"] = "none"
            continue
        b["joints"] = [dict(type=k, axis=list(rng.standard_normal(3)),
                            pos=list(0.05 * rng.standard_normal(3)),
                            armature=float(rng.uniform(0.0, 0.05))) for k in pat]
        del b["joint"]
    return t


def slider(mass=1.3, axis=(0.6, 0.0, 0.8), armature=0.02) -> dict:
    """A point-like mass on a slide joint along a tilted world-fixed axis (fixed base), one site
    at the COM."""
    return dict(name="slider", gravity=[0.0, 0.0, -9.81], bodies=[dict(
        name="carriage", parent=-1, pos=[0.1, 0.2, 0.3], quat=[1, 0, 0, 0], joint="slide",
        axis=list(axis), jnt_pos=[0, 0, 0], armature=armature, mass=mass, ipos=[0, 0, 0],
        iquat=[1, 0, 0, 0], diaginertia=[1e-3, 1e-3, 1e-3])],
        sites=[dict(name="c", body=0, pos=[0, 0, 0])])


def spherical_pendulum(mass=0.8, length=0.5, i_small=1e-4) -> dict:
    """A point-like mass below a ball joint (fixed base): one body, COM at -length z."""
    return dict(name="spherical pendulum", gravity=[0.0, 0.0, -9.81], bodies=[dict(
        name="bob", parent=-1, pos=[0, 0, 0], quat=[1, 0, 0, 0], joint="ball", axis=[0, 0, 1],
        jnt_pos=[0, 0, 0], armature=0.0, mass=mass, ipos=[0, 0, -length], iquat=[1, 0, 0, 0],
        diaginertia=[i_small, i_small, i_small])],
        sites=[dict(name="tip", body=0, pos=[0, 0, -length])])


def two_joint_body(mass=1.1, length=0.6, i_small=1e-4, arm=(0.01, 0.03)) -> dict:
    """One body with two joints, MuJoCo style: a hinge about world x then a hinge about the
    (rotated) body y, both through the origin, point-like mass at -length z (a universal-joint
    pendulum)."""
    return dict(name="two-joint body", gravity=[0.0, 0.0, -9.81], bodies=[dict(
        name="u", parent=-1, pos=[0, 0, 0], quat=[1, 0, 0, 0],
        joints=[dict(type="hinge", axis=[1, 0, 0], pos=[0, 0, 0], armature=arm[0]),
                dict(type="hinge", axis=[0, 1, 0], pos=[0, 0, 0], armature=arm[1])],
        mass=mass, ipos=[0, 0, -length], iquat=[1, 0, 0, 0],
        diaginertia=[i_small, i_small, i_small])],
        sites=[dict(name="tip", body=0, pos=[0, 0, -length])])
