"""Offline proof that some self-collision pairs of the capsule model can never touch
while the joints stay inside the Franka limits (the MoveIt-SRDF idea of "never"
pairs, here proven instead of sampled).

For pair (I, J) the capsule distance depends only on the joints between link(I) and
link(J) (plus the finger slide for a finger capsule). On a grid over those joints the
exact float64 segment-segment distance d is evaluated; between grid points d changes
by at most sum_k L_k * h_k, where h_k is half the grid step of joint k and L_k a
Lipschitz bound of d in q_k: for a revolute joint the largest distance from its axis
origin to the moving capsule's endpoints (bounded by the sum of the chain offsets,
triangle inequality), for the finger slide 1. The pair is proven "never" when
    min_grid d - sum_k L_k h_k > r_I + r_J + 1e-4
(1e-4 m: margin for the float32 evaluation, ~1e-6 m, as the kernel's sphere test).

    python tools/prove_pairs.py [grid_scale]   -> JSON on stdout
"""
import json
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rbe550_final_project_amd import model  # noqa: E402

SRC = open(os.path.join(ROOT, "rbe550_final_project_amd", "csrc", "rp_model.h")).read()
G = np.array([[float(x.rstrip("f")) for x in r.split(",")]
              for r in re.findall(r"\{(-?[\d.]+f?(?:, -?[\d.]+f?){6})\},\s*// \w+", SRC)])
NAMES = ["link0", "link1", "link2", "link3", "link4", "link5a", "link5b", "link6", "link7", "hand", "lfinger",
         "rfinger"]
CAP_LINK = [0, 1, 2, 3, 4, 5, 5, 6, 7, 8, 9, 10]
# (translation, Rx degrees) of links 1..7 (as rp_math.h fk_walk)
CHAIN = [((0, 0, 0.333), 0.0), ((0, 0, 0), -90.0), ((0, -0.316, 0), 90.0), ((0.0825, 0, 0), 90.0),
         ((-0.0825, 0.384, 0), -90.0), ((0, 0, 0), 90.0), ((0.088, 0, 0), 90.0)]
HAND_Z, FINGER_Z = 0.107, 0.0584


def _rx(deg):
    a = np.deg2rad(deg)
    c, s = np.cos(a), np.sin(a)
    return np.array([[1, 0, 0], [0, c, -s], [0, s, c]])


def _rz(a):
    c, s = np.cos(a), np.sin(a)
    Z = np.zeros(a.shape + (3, 3))
    Z[..., 0, 0], Z[..., 0, 1], Z[..., 1, 0], Z[..., 1, 1], Z[..., 2, 2] = c, -s, s, c, 1
    return Z


def frames(q):
    N = len(q)
    R = np.broadcast_to(np.eye(3), (N, 3, 3)).copy()
    p = np.zeros((N, 3))
    out = [(R.copy(), p.copy())]
    for j, (t, a) in enumerate(CHAIN):
        p = p + R @ np.array(t, dtype=float)
        R = R @ _rx(a) @ _rz(q[:, j])
        out.append((R.copy(), p.copy()))
    p = p + R @ np.array([0, 0, HAND_Z])
    R = R @ _rz(np.full(N, -np.pi / 4))
    out.append((R.copy(), p.copy()))
    pf = p + R @ np.array([0, 0, FINGER_Z])
    out.append((R.copy(), pf + R[:, :, 1] * q[:, 7:8]))
    Rr = R @ _rz(np.full(N, np.pi))
    out.append((Rr, pf - R[:, :, 1] * q[:, 8:9]))
    return out


def endpoints(fr, c):
    R, p = fr[CAP_LINK[c]]
    return p + R @ G[c, :3], p + R @ G[c, 3:6]


def seg_seg(a1, b1, a2, b2):
    d1, d2, w = b1 - a1, b2 - a2, a1 - a2
    A = (d1 * d1).sum(1)
    E = (d2 * d2).sum(1)
    B = (d1 * d2).sum(1)
    C = (d1 * w).sum(1)
    F = (d2 * w).sum(1)
    den = A * E - B * B
    s = np.where(den > 1e-15, np.clip((B * F - C * E) / np.where(den > 1e-15, den, 1), 0, 1), 0.0)
    t = (B * s + F) / E
    s = np.where(t < 0, np.clip(-C / A, 0, 1), np.where(t > 1, np.clip((B - C) / A, 0, 1), s))
    t = np.clip(t, 0, 1)
    return np.linalg.norm((a1 + d1 * s[:, None]) - (a2 + d2 * t[:, None]), axis=1)


def lever_bound(J, k):
    """upper bound of |x - o_k| for the endpoints x of capsule J, o_k on joint k's
    axis (the origin of link k+1): the sum of the chain offsets from link k+1 on."""
    L = 0.0
    lj = CAP_LINK[J]
    for j in range(k + 1, min(lj, 7)):
        L += np.linalg.norm(CHAIN[j][0])
    if lj >= 8:
        L += HAND_Z
    if lj >= 9:
        L += FINGER_Z + 0.04
    return L + max(np.linalg.norm(G[J, :3]), np.linalg.norm(G[J, 3:6]))


def prove(I, J, n):
    li, lj = CAP_LINK[I], CAP_LINK[J]
    joints = [k for k in range(li, min(lj, 7))]      # q[k] turns link k+1
    if lj >= 8:
        joints = [k for k in range(li, 7)]
    fingers = [7] if J == 10 else [8] if J == 11 else []
    lo, hi = model.Q_LO.astype(np.float64), model.Q_HI.astype(np.float64)
    axes = [np.linspace(lo[k], hi[k], n) for k in joints] + [np.linspace(lo[k], hi[k], 9) for k in fingers]
    steps = [(hi[k] - lo[k]) / (n - 1) for k in joints] + [(hi[k] - lo[k]) / 8 for k in fingers]
    levers = [lever_bound(J, k) for k in joints] + [1.0 for _ in fingers]
    ks = joints + fingers
    mesh = np.stack(np.meshgrid(*axes, indexing="ij"), -1).reshape(-1, len(ks))
    dmin = np.inf
    for c0 in range(0, len(mesh), 250000):
        q = np.zeros((len(mesh[c0:c0 + 250000]), 9))
        q[:, ks] = mesh[c0:c0 + 250000]
        fr = frames(q)
        a1, b1 = endpoints(fr, I)
        a2, b2 = endpoints(fr, J)
        dmin = min(dmin, float(seg_seg(a1, b1, a2, b2).min()))
    slack = sum(L * h / 2 for L, h in zip(levers, steps))
    need = G[I, 6] + G[J, 6] + 1e-4
    return {"pair": [NAMES[I], NAMES[J]], "joints": ks, "grid_points": int(len(mesh)), "min_dist": dmin,
            "lipschitz_slack": slack, "radii_sum": need - 1e-4, "proven": bool(dmin - slack > need),
            "margin": dmin - slack - need}


CANDIDATES = [(2, 5), (3, 7), (3, 8), (4, 8), (4, 9), (4, 10), (4, 11), (6, 9), (6, 10), (6, 11)]


def grid_for(I, J):
    """points per revolute axis: finer for fewer axes (grid sizes ~2e6-3e7)"""
    li, lj = CAP_LINK[I], CAP_LINK[J]
    m = min(lj, 7) - li
    return {1: 4001, 2: 1001, 3: 161, 4: 71}.get(m, 41)


def main():
    scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
    out = [prove(I, J, max(11, int(grid_for(I, J) * scale))) for I, J in CANDIDATES]
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
