"""Float64 numpy model of the Franka Panda chain (tooling only: fixture and query
generation, model tuning). The product evaluates kinematics in the HIP kernels
(rbe550_final_project_amd/csrc/rp_math.h); the test oracle in oracle/rbe_oracle.c.

Kinematic constants: SURVEY.md Appendix A.2 (public Franka / MuJoCo-Menagerie
panda.xml that Genesis loads at code/scenes.py:85).
"""
import numpy as np

# body offsets (pos, rotation about x in degrees applied before the joint rotation)
_CHAIN = [
    ((0.0, 0.0, 0.333), 0.0),
    ((0.0, 0.0, 0.0), -90.0),
    ((0.0, -0.316, 0.0), 90.0),
    ((0.0825, 0.0, 0.0), 90.0),
    ((-0.0825, 0.384, 0.0), -90.0),
    ((0.0, 0.0, 0.0), 90.0),
    ((0.088, 0.0, 0.0), 90.0),
]

LINK_NAMES = ["link0", "link1", "link2", "link3", "link4", "link5", "link6", "link7",
              "hand", "left_finger", "right_finger"]


def _rx(deg):
    a = np.deg2rad(deg)
    c, s = np.cos(a), np.sin(a)
    return np.array([[1, 0, 0], [0, c, -s], [0, s, c]])


def _rz(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


def link_frames(q, base=(0.0, 0.0, 0.01)):
    """Return list of 11 (R, p) world frames for q (9,)."""
    q = np.asarray(q, dtype=float)
    R = np.eye(3)
    p = np.array(base, dtype=float)
    frames = [(R.copy(), p.copy())]
    for j, (t, rx) in enumerate(_CHAIN):
        p = p + R @ np.array(t)
        R = R @ _rx(rx) @ _rz(q[j])
        frames.append((R.copy(), p.copy()))
    # hand: flange 0.107 along z, rotated -45 deg about z
    p = p + R @ np.array([0, 0, 0.107])
    R = R @ _rz(-np.pi / 4)
    frames.append((R.copy(), p.copy()))
    Rh, ph = R, p
    pf = ph + Rh @ np.array([0, 0, 0.0584])
    frames.append((Rh.copy(), pf + Rh @ np.array([0, q[7], 0])))
    Rr = Rh @ _rz(np.pi)
    frames.append((Rr, pf + Rh @ np.array([0, -q[8], 0])))
    return frames


def hand_pose(q, base=(0.0, 0.0, 0.01)):
    R, p = link_frames(q, base)[8]
    return R, p


def mat_to_quat(R):
    """(w, x, y, z) of a rotation matrix."""
    w = np.sqrt(max(0.0, 1 + R[0, 0] + R[1, 1] + R[2, 2])) / 2
    x = np.sqrt(max(0.0, 1 + R[0, 0] - R[1, 1] - R[2, 2])) / 2
    y = np.sqrt(max(0.0, 1 - R[0, 0] + R[1, 1] - R[2, 2])) / 2
    z = np.sqrt(max(0.0, 1 - R[0, 0] - R[1, 1] + R[2, 2])) / 2
    x = np.copysign(x, R[2, 1] - R[1, 2])
    y = np.copysign(y, R[0, 2] - R[2, 0])
    z = np.copysign(z, R[1, 0] - R[0, 1])
    return np.array([w, x, y, z])


def quat_to_mat(qt):
    w, x, y, z = np.asarray(qt, dtype=float) / np.linalg.norm(qt)
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
        [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)],
    ])


def ik_hand(pos, quat, q_seed, lo, hi, base=(0.0, 0.0, 0.01), iters=400, tol=1e-6):
    """Damped-least-squares IK of the hand link (7 arm joints, fingers kept from
    q_seed) — tooling stand-in for Genesis' inverse_kinematics used by
    code/motion_primitives.py:131-134 to make goal configurations."""
    q = np.array(q_seed, dtype=float)
    Rt = quat_to_mat(quat)
    pt = np.asarray(pos, dtype=float)
    lam = 1e-3
    for _ in range(iters):
        R, p = hand_pose(q, base)
        ep = pt - p
        Re = Rt @ R.T
        # rotation error as axis-angle vector
        ang = np.arccos(np.clip((np.trace(Re) - 1) / 2, -1, 1))
        if ang < 1e-9:
            er = np.zeros(3)
        else:
            er = ang / (2 * np.sin(ang)) * np.array([Re[2, 1] - Re[1, 2], Re[0, 2] - Re[2, 0], Re[1, 0] - Re[0, 1]])
        err = np.concatenate([ep, er])
        if np.linalg.norm(err) < tol:
            break
        J = np.zeros((6, 7))
        eps = 1e-7
        for j in range(7):
            dq = q.copy()
            dq[j] += eps
            R2, p2 = hand_pose(dq, base)
            dR = R2 @ R.T
            J[:3, j] = (p2 - p) / eps
            J[3:, j] = np.array([dR[2, 1] - dR[1, 2], dR[0, 2] - dR[2, 0], dR[1, 0] - dR[0, 1]]) / (2 * eps)
        dq = J.T @ np.linalg.solve(J @ J.T + lam * np.eye(6), err)
        q[:7] = np.clip(q[:7] + dq, lo[:7], hi[:7])
    R, p = hand_pose(q, base)
    ok = np.linalg.norm(pt - p) < 1e-4
    return q, ok
