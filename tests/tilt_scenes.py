"""Scenes with tilted boxes (test data): blocks that toppled or lean, as the
reference's towers leave them after a collapse ("Stack collapsed! ... TAMP will
re-plan", code/goal3_tallest.py:257; Report §XI "8th topples"). The collider
(Genesis, code/planning.py:211) sees every block at its simulated pose, so the
planner must test the capsules against the rotated boxes (rp_set_scene_rot)."""
import json
import math
import os

import numpy as np

from rbe550_final_project_amd import scenes

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def quat_axis_angle(axis, deg):
    """(w, x, y, z) of a rotation by `deg` degrees about `axis`."""
    a = np.asarray(axis, float)
    a = a / np.linalg.norm(a)
    h = math.radians(deg) / 2.0
    return (math.cos(h), *(math.sin(h) * a))


def quat_mul(p, q):
    w1, x1, y1, z1 = p
    w2, x2, y2, z2 = q
    return (w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
            w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2)


def rot_matrix(q):
    """World = R * box of a (w, x, y, z) quaternion (float64)."""
    w, x, y, z = np.asarray(q, float) / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def toppled_goal3():
    """goal3's 10 blocks (scenes.py:150-223) after a collapse: one rolled 90 deg about
    x (lying on a side face), one leaning 10 deg on an edge, one lying on an edge at
    45 deg and yawed, a block of a fallen tower resting tilted 25 deg about an oblique
    axis on another, and a plank (0.02 x 0.04 x 0.12 m) fallen flat across the table."""
    sc = scenes.goal3_tallest()
    h = scenes.HALF[0]
    sc.move("r2", sc.boxes[sc.index("r2")][0], quat=quat_axis_angle((1, 0, 0), 90.0))
    lean = math.radians(10.0)
    c = sc.boxes[sc.index("y2")][0]
    sc.move("y2", (c[0], c[1], h * (math.cos(lean) + math.sin(lean))), quat=quat_axis_angle((0, 1, 0), 10.0))
    c = sc.boxes[sc.index("g")][0]
    sc.move("g", (c[0], c[1], h * math.sqrt(2.0)),
            quat=quat_mul(quat_axis_angle((0, 0, 1), 30.0), quat_axis_angle((1, 0, 0), 45.0)))
    c = sc.boxes[sc.index("b")][0]
    sc.move("b2", (c[0] + 0.01, c[1] - 0.005, 0.062), quat=quat_axis_angle((1, 2, 0.5), 25.0))
    i = sc.index("o2")
    c = sc.boxes[i][0]
    sc.boxes[i] = ((c[0], c[1], 0.01), (0.01, 0.02, 0.06), quat_axis_angle((0, 1, 0), 90.0))
    return sc


def tilted_clutter64(seed=7):
    """The C5 clutter64 scene (axis-grid broad phase, > 16 boxes) with every third box
    given a random orientation (uniform random unit quaternion)."""
    q = json.load(open(os.path.join(GOLD, "workloads", "clutter64.json")))["queries"][0]
    sc = scenes.Scene.from_json(q["scene"])
    rng = np.random.default_rng(seed)
    for i in range(0, len(sc.boxes), 3):
        u = rng.standard_normal(4)
        u /= np.linalg.norm(u)
        c, hh, _ = sc.boxes[i]
        sc.boxes[i] = (c, hh, tuple(float(v) for v in u))
    return sc, q
