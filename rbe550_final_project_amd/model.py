"""Franka Panda planning model: joint bounds and the capsule collision model.

Bounds: the 9 qpos dims of the Genesis MJCF Panda (code/planning.py:139-150 reads
them from robot.q_limit). Genesis keeps q_limit in float32,
so the planner's bounds are the float32 values widened to float64 — which is why a
finger value of 0.04 is "out of bounds" in the reference (README.md:101-111).
"""
import json
import os

import numpy as np

from . import _abi

_HERE = os.path.dirname(os.path.abspath(__file__))
SPEC_PATH = os.path.join(os.path.dirname(_HERE), "spec", "franka_capsules.json")
if not os.path.exists(SPEC_PATH):  # installed copy
    SPEC_PATH = os.path.join(_HERE, "spec", "franka_capsules.json")

Q_LO_SPEC = np.array([-2.8973, -1.7628, -2.8973, -3.0718, -2.8973, -0.0175, -2.8973, 0.0, 0.0])
Q_HI_SPEC = np.array([2.8973, 1.7628, 2.8973, -0.0698, 2.8973, 3.7525, 2.8973, 0.04, 0.04])

# float32-stored limits, as Genesis hands them to planning.py:139-140
Q_LO = Q_LO_SPEC.astype(np.float32).astype(np.float64)
Q_HI = Q_HI_SPEC.astype(np.float32).astype(np.float64)

# poses used by the reference scripts
SAFE_HOME = np.array([0.0, -0.785, 0.0, -2.356, 0.0, 1.571, 0.785, 0.04, 0.04])   # goal1_scattered.py:43
SCENE_INIT = np.array([0.0, -0.5, -0.2, -1.0, 0.0, 1.00, 0.5, 0.02, 0.02])        # scenes.py:92
BASE_POS = (0.0, 0.0, 0.01)   # base raised 1 cm (scenes.py:29-34)


def max_extent(lo=Q_LO, hi=Q_HI):
    return float(np.sqrt(np.sum((np.asarray(hi) - np.asarray(lo)) ** 2)))


def load_spec(path=SPEC_PATH):
    with open(path) as f:
        return json.load(f)


def robot_desc(spec=None):
    """rp_robot_desc from spec/franka_capsules.json."""
    spec = spec or load_spec()
    links = {n: i for i, n in enumerate(spec["links"])}
    caps = spec["capsules"]
    names = {c["name"]: i for i, c in enumerate(caps)}
    d = _abi.RobotDesc()
    d.n_capsules = len(caps)
    for i, c in enumerate(caps):
        d.capsules[i].link = links[c["link"]]
        d.capsules[i].a[:] = c["a"]
        d.capsules[i].b[:] = c["b"]
        d.capsules[i].radius = c["radius"]
    d.n_self_pairs = len(spec["self_pairs"])
    for i, (a, b) in enumerate(spec["self_pairs"]):
        d.self_pairs[i][0] = names[a]
        d.self_pairs[i][1] = names[b]
    return d
