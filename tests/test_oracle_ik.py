"""CPU oracle of the batched hand-link IK (ro_ik, the algorithm of rp_ik /
rbe550_final_project_amd/csrc/rp_ik.h). Reference call site: Genesis
robot.inverse_kinematics(link=hand, pos, quat) in code/motion_primitives.py:131-134;
Genesis is absent here, so correctness is pinned by the pose error of the returned
configuration under an independent float64 numpy model of the chain
(tools/franka_np.py) rather than by reference outputs (parity unpinned against
Genesis itself)."""
import json
import os
import sys

import numpy as np

from rbe550_final_project_amd import _abi, model, scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import franka_np  # noqa: E402


HOME = model.SAFE_HOME.copy()
HOME[7:] = np.float32(0.04)   # open fingers inside the float32 bounds


def _targets(n=12):
    """hand poses of the goal configurations of the goal3 workload"""
    wl = json.load(open(os.path.join(ROOT, "tests", "golden", "workloads", "goal3_tallest_10box.json")))
    pos, quat = [], []
    for q in wl["queries"][:n]:
        R, p = franka_np.hand_pose(q["goal"])
        pos.append(p)
        quat.append(franka_np.mat_to_quat(R))
    return np.array(pos), np.array(quat)


def test_sincos64_accuracy(oracle_lib):
    x = np.concatenate([np.linspace(-7, 7, 2001), [0.0, np.pi / 4, np.pi / 2, -np.pi]])
    for v in x:
        s, c = oracle_lib.sincos64(v)
        assert abs(s - np.sin(v)) <= 4e-16 and abs(c - np.cos(v)) <= 4e-16


def test_hand_pose_matches_numpy_model(oracle_lib):
    o = oracle_lib.OracleScene()
    o.set_scene([], 0.0, (0.0, 0.0, 0.0))
    rng = np.random.default_rng(3)
    for _ in range(20):
        q = model.Q_LO + (model.Q_HI - model.Q_LO) * rng.random(9)
        R, p = o.hand_pose(q)
        R2, p2 = franka_np.hand_pose(q, base=(0.0, 0.0, 0.0))
        assert np.abs(R - R2).max() < 1e-12 and np.abs(p - p2).max() < 1e-12


def test_ik_reaches_workload_goals(oracle_lib):
    o = oracle_lib.OracleScene()
    sc = scenes.goal3_tallest()
    o.set_scene(sc.boxes, sc.plane_z, sc.base)
    pos, quat = _targets()
    init = np.tile(HOME, (len(pos), 1))
    p = _abi.make_ik_params(seed=7, n_seeds=32)
    q, st = o.ik(pos, quat, init, model.Q_LO, model.Q_HI, p)
    assert (st == _abi.IK_OK).all(), st
    for k in range(len(pos)):
        R, pp = franka_np.hand_pose(q[k], base=sc.base)
        assert np.linalg.norm(pp - pos[k]) <= 5e-4
        assert np.abs(R - franka_np.quat_to_mat(quat[k])).max() <= 1e-2
        assert np.all(q[k] >= model.Q_LO) and np.all(q[k] <= model.Q_HI)
        assert np.array_equal(q[k, 7:], HOME[7:])
        assert o.check_states(q[k:k + 1].astype(np.float32))[0] == 1


def test_ik_unreachable_and_deterministic(oracle_lib):
    o = oracle_lib.OracleScene()
    o.set_scene([], 0.0, (0.0, 0.0, 0.01))
    pos = np.array([[2.0, 0.0, 0.5], [0.5, 0.0, 0.3]])
    quat = np.array([[0.0, 1.0, 0.0, 0.0], [0.0, 1.0, 0.0, 0.0]])
    init = np.tile(HOME, (2, 1))
    p = _abi.make_ik_params(seed=1, n_seeds=16)
    q1, st1 = o.ik(pos, quat, init, model.Q_LO, model.Q_HI, p)
    q2, st2 = o.ik(pos, quat, init, model.Q_LO, model.Q_HI, p)
    assert st1[0] == _abi.IK_NOT_CONVERGED and st1[1] == _abi.IK_OK
    assert np.array_equal(q1, q2) and np.array_equal(st1, st2)
