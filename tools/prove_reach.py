"""Offline bound of how far each capsule of the model can reach while the joints stay
inside the Franka limits: every point of capsule C lies within REACH[C] of a fixed
centre — the robot base for link0 (a fixed capsule), the shoulder S = base + (0, 0,
0.333) for the others (link1's origin, on joint 1's axis, so q0 does not change any
distance to it). k_validity skips a capsule's box tests in a wave whose states are
all inside the limits when every box's AABB is farther than REACH[C] + 1e-4 m from
the centre (rp_lib.hip env_far_mask): such a test can only say "no contact".

For capsules moved by at most MAX_GRID_JOINTS joints the bound is a grid maximum of
the exact float64 endpoint distance plus a Lipschitz slack (as tools/prove_pairs.py:
between grid points the distance changes by at most sum_k L_k h_k / 2, L_k the lever
of joint k); for the others the chain sum (triangle inequality). The capsule radius
is added. Output: JSON (tests/golden/reach_proof.json) and the C++ table.

    python tools/prove_reach.py [grid_scale] > tests/golden/reach_proof.json
"""
import json
import sys

import numpy as np

from prove_pairs import CAP_LINK, CHAIN, FINGER_Z, HAND_Z, NAMES, G, endpoints, frames, lever_bound, model

S = np.array([0.0, 0.0, 0.333])
MAX_GRID_JOINTS = 4
GRID = {0: 1, 1: 20001, 2: 2001, 3: 201, 4: 61}


def chain_bound(c):
    """sum of the chain offsets from S to capsule c's frame + its endpoint norm"""
    lc = CAP_LINK[c]
    L = sum(np.linalg.norm(CHAIN[j][0]) for j in range(1, min(lc, 7)))
    if lc >= 8:
        L += HAND_Z
    if lc >= 9:
        L += FINGER_Z + 0.04
    return L + max(np.linalg.norm(G[c, :3]), np.linalg.norm(G[c, 3:6]))


def reach(c, scale=1.0):
    r = float(G[c, 6])
    if c == 0:   # fixed to the base
        d = max(np.linalg.norm(G[0, :3]), np.linalg.norm(G[0, 3:6]))
        return {"capsule": NAMES[c], "centre": "base", "joints": [], "grid_max": d, "lipschitz_slack": 0.0,
                "radius": r, "reach": d + r}
    lc = CAP_LINK[c]
    joints = list(range(1, min(lc, 7)))          # q[k] turns link k + 1; q0 keeps |x - S|
    if lc >= 8:
        joints = list(range(1, 7))
    fingers = [7] if c == 10 else [8] if c == 11 else []
    if len(joints) > MAX_GRID_JOINTS:
        return {"capsule": NAMES[c], "centre": "shoulder", "joints": joints + fingers, "grid_max": None,
                "lipschitz_slack": None, "radius": r, "reach": chain_bound(c) + r, "method": "chain sum"}
    lo, hi = model.Q_LO.astype(np.float64), model.Q_HI.astype(np.float64)
    n = max(3, int(GRID[len(joints)] * scale))
    axes = [np.linspace(lo[k], hi[k], n) for k in joints]
    steps = [(hi[k] - lo[k]) / (n - 1) for k in joints]
    levers = [lever_bound(c, k) for k in joints]
    mesh = np.stack(np.meshgrid(*axes, indexing="ij"), -1).reshape(-1, len(joints)) if joints else np.zeros((1, 0))
    dmax = 0.0
    for c0 in range(0, len(mesh), 250000):
        q = np.zeros((len(mesh[c0:c0 + 250000]), 9))
        q[:, joints] = mesh[c0:c0 + 250000]
        fr = frames(q)
        a, b = endpoints(fr, c)
        dmax = max(dmax, float(np.linalg.norm(a - S, axis=1).max()), float(np.linalg.norm(b - S, axis=1).max()))
    slack = sum(L * h / 2 for L, h in zip(levers, steps))
    return {"capsule": NAMES[c], "centre": "shoulder", "joints": joints, "grid_points": int(len(mesh)),
            "grid_max": dmax, "lipschitz_slack": slack, "radius": r, "reach": dmax + slack + r,
            "method": "grid + Lipschitz"}


def main():
    scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
    out = [reach(c, scale) for c in range(12)]
    json.dump(out, sys.stdout, indent=1)
    print()
    print("// constexpr float REACH[NCAP] = {" + ", ".join(f"{np.nextafter(np.float32(o['reach']), np.float32(np.inf)):.6f}f"
                                                        for o in out) + "};", file=sys.stderr)


if __name__ == "__main__":
    main()
