"""Write the kinematic-tree descriptions used by the GPU kinematics front end (SURVEY.md §8(f)
row 1) to operational-space-control_amd/config/<robot>_kinematics.json.

The reference loads its robots from MJCF files of the external vannem95/mujoco-models archive
(MODULE.bazel:32-38), which is not vendored, so these are ILLUSTRATIVE trees with the same
topology, joint types, dof order and site order as the reference's models use:
  * unitree_go2: free trunk + 4 legs (hip about x, thigh and calf about y), sites
    [imu, FR foot, FL foot, HR foot, HL foot] (the weight order of unitree_go2/autogen.py:160-219);
    dimensions and inertias approximate the public Go2 description.
  * walter_sr: free torso + 4 legs (thigh, shin about y), sites [torso, 4 shins, 4 thighs,
    8 wheel contacts] (walter_sr/autogen/autogen.py:163-330 order); dimensions are made up.
Parity against MuJoCo therefore stays unpinned; the kinematics oracle is pinned by physical
identities instead (tests/test_kinematics_oracle.py).

Schema (MJCF semantics): per body parent (-1 = world), pos/quat (w, x, y, z) in the parent
frame, joint "free" | "hinge" | "none", hinge axis and anchor in the body frame, armature per
hinge dof, mass, COM ipos and principal inertia (iquat, diaginertia) in the body frame; per site
body and pos.  Bodies are listed parents first; dofs follow body order.
"""
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "operational-space-control_amd", "config")
Q1 = [1.0, 0.0, 0.0, 0.0]


def body(name, parent, pos, joint, axis=(0, 0, 1), mass=1.0, ipos=(0, 0, 0),
         diag=(1e-3, 1e-3, 1e-3), quat=Q1, iquat=Q1, armature=0.0, jnt_pos=(0, 0, 0)):
    return dict(name=name, parent=parent, pos=list(pos), quat=list(quat), joint=joint,
                axis=list(axis), jnt_pos=list(jnt_pos), armature=armature, mass=mass,
                ipos=list(ipos), iquat=list(iquat), diaginertia=list(diag))


def go2():
    b = [body("trunk", -1, (0, 0, 0), "free", mass=6.921, ipos=(0.021112, 0.0, -0.005366),
              diag=(0.02448, 0.098077, 0.107))]
    sites = [dict(name="imu", body=0, pos=[-0.02557, 0.0, 0.04232])]
    legs = {"FL": (1, 1), "FR": (1, -1), "RL": (-1, 1), "RR": (-1, -1)}
    feet = {}
    for leg, (sx, sy) in legs.items():
        hip = len(b)
        b.append(body(f"{leg}_hip", 0, (0.1934 * sx, 0.0465 * sy, 0), "hinge", axis=(1, 0, 0),
                      mass=0.678, ipos=(-0.0054 * sx, 0.00194 * sy, -0.000105),
                      diag=(0.00048, 0.000884, 0.000596), armature=0.01))
        thigh = len(b)
        b.append(body(f"{leg}_thigh", hip, (0, 0.0955 * sy, 0), "hinge", axis=(0, 1, 0),
                      mass=1.152, ipos=(-0.00374, -0.0223 * sy, -0.0327),
                      diag=(0.00584, 0.0058, 0.00103), armature=0.01))
        calf = len(b)
        b.append(body(f"{leg}_calf", thigh, (0, 0, -0.213), "hinge", axis=(0, 1, 0),
                      mass=0.154, ipos=(0.00548, -0.000975, -0.115),
                      diag=(0.00108, 0.0011, 3.29e-05), armature=0.01))
        feet[leg] = dict(name=f"{leg}_foot", body=calf, pos=[0.0, 0.0, -0.213])
    sites += [feet["FR"], feet["FL"], feet["RR"], feet["RL"]]   # reference order FR FL HR HL
    return dict(name="unitree_go2 (illustrative tree)", gravity=[0, 0, -9.81], bodies=b,
                sites=sites)


def walter():
    b = [body("torso", -1, (0, 0, 0), "free", mass=6.0, ipos=(0.0, 0.0, 0.02),
              diag=(0.05, 0.12, 0.14))]
    legs = {"tl": (1, 1), "tr": (1, -1), "hl": (-1, 1), "hr": (-1, -1)}
    thigh_s, shin_s, wheel_s = {}, {}, {}
    for leg, (sx, sy) in legs.items():
        th = len(b)
        b.append(body(f"{leg}_thigh", 0, (0.22 * sx, 0.12 * sy, 0.0), "hinge", axis=(0, 1, 0),
                      mass=0.9, ipos=(0.0, 0.0, -0.09), diag=(0.004, 0.004, 0.0008),
                      armature=0.02))
        sh = len(b)
        b.append(body(f"{leg}_shin", th, (0.0, 0.0, -0.18), "hinge", axis=(0, 1, 0),
                      mass=0.6, ipos=(0.0, 0.0, -0.08), diag=(0.002, 0.002, 0.0004),
                      armature=0.02))
        thigh_s[leg] = dict(name=f"{leg}_thigh_site", body=th, pos=[0.0, 0.0, -0.09])
        shin_s[leg] = dict(name=f"{leg}_shin_site", body=sh, pos=[0.0, 0.0, -0.08])
        wheel_s[leg] = [dict(name=f"{leg}f_wheel_site", body=sh, pos=[0.05, 0.0, -0.17]),
                        dict(name=f"{leg}r_wheel_site", body=sh, pos=[-0.05, 0.0, -0.17])]
    order = ["tl", "tr", "hl", "hr"]
    sites = [dict(name="torso_site", body=0, pos=[0.0, 0.0, 0.0])]
    sites += [shin_s[k] for k in order] + [thigh_s[k] for k in order]
    for k in order:
        sites += wheel_s[k]
    return dict(name="walter_sr (illustrative tree)", gravity=[0, 0, -9.81], bodies=b,
                sites=sites)


def main():
    for robot, m in (("unitree_go2", go2()), ("walter_sr", walter())):
        path = os.path.join(OUT, f"{robot}_kinematics.json")
        with open(path, "w") as f:
            json.dump(m, f, indent=1)
        print(path)


if __name__ == "__main__":
    main()
