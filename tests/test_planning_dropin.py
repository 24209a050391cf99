"""The drop-in planning.PlannerInterface (code/planning.py:24-242 contract) driven
through a Genesis-free mock robot/scene."""
import json
import sys
import os

import numpy as np
import pytest
import torch

from rbe550_final_project_amd import model, planning, scenes
from rbe550_final_project_amd.native import NativeError
import mock_genesis as M

GOLD = os.path.join(os.path.dirname(__file__), "golden")
REF = json.load(open(os.path.join(GOLD, "reference_fixtures.json")))


def _mk(boxes=()):
    sc = M.Scene(list(boxes))
    return planning.PlannerInterface(sc.robot, sc), sc


def test_bad_planner_raises_like_reference():
    pi, _ = _mk()
    with pytest.raises(planning.PlanningError) as e:
        pi.plan_path(model.SAFE_HOME, planner="Foo")
    assert str(e.value) == REF["errors"]["bad_planner"]


def test_bad_shape_raises_like_reference():
    pi, _ = _mk()
    with pytest.raises(planning.PlanningError) as e:
        pi.plan_path(model.SAFE_HOME[:7])
    assert str(e.value) == REF["errors"]["bad_shape"]


def test_batched_envs_and_free_joints_raise():
    sc = M.Scene([], n_envs=2)
    with pytest.raises(planning.PlanningError, match="batched envs"):
        planning.PlannerInterface(sc.robot, sc).plan_path(model.SAFE_HOME)
    sc = M.Scene([], n_dofs=7)
    with pytest.raises(planning.PlanningError, match="free joints"):
        planning.PlannerInterface(sc.robot, sc).plan_path(model.SAFE_HOME)


def test_genesis_scene_ingestion():
    boxes = [((0.65, 0.0, 0.02), (0.02, 0.02, 0.02), 0.0), ((0.5, 0.1, 0.02), (0.02, 0.02, 0.02), 0.7)]
    sc = M.Scene(boxes)
    s = scenes.from_genesis(sc, sc.robot)
    assert len(s.boxes) == 2 and s.entity_idx == [1, 2]
    assert np.allclose(s.boxes[1][0], (0.5, 0.1, 0.02)) and abs(s.boxes[1][2] - 0.7) < 1e-6
    assert np.allclose(s.boxes[0][1], (0.02, 0.02, 0.02))
    assert np.allclose(s.base, model.BASE_POS)


def test_no_silent_cpu_fallback():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    pi, _ = _mk()
    with pytest.raises(NativeError):
        pi.plan_path(model.SAFE_HOME)


@pytest.mark.gpu
def test_plan_path_contract_on_gpu():
    wl = json.load(open(os.path.join(GOLD, "workloads", "goal3_tallest_10box.json")))
    q = wl["queries"][0]
    s = scenes.Scene.from_json(q["scene"])
    sc = M.Scene(s.boxes)
    sc.robot.q = torch.tensor(q["start"], dtype=torch.float32)
    pi = planning.PlannerInterface(sc.robot, sc)
    planning.configure(seed=0)
    wps = pi.plan_path(qpos_goal=np.array(q["goal"]), num_waypoints=150, timeout=10.0)
    c = REF["return_contract"]
    assert len(wps) == c["n"] == 150
    assert all(isinstance(w, torch.Tensor) and w.dtype == torch.float32 and list(w.shape) == c["shape"]
               and w.device.type == "cpu" for w in wps)
    assert np.allclose(wps[0].numpy(), np.float32(q["start"]), atol=1e-6)
    assert np.allclose(wps[-1].numpy(), np.float32(q["goal"]), atol=1e-6)
    # consumer contract (motion_primitives.py:163-178): np.array(path[-1], dtype=float)
    # exactly as the caller writes it (torch's Tensor.__array__ predates NumPy 2's
    # copy keyword; the DeprecationWarning NumPy raises about it is torch's, not ours)
    import warnings
    with warnings.catch_warnings():
        warnings.filterwarnings("ignore", message=".*__array__.*copy.*", category=DeprecationWarning)
        arr = np.array(wps[-1], dtype=float)
    assert arr.shape == (9,)
    # the robot's qpos is restored at the end (planning.py:205)
    assert torch.equal(sc.robot.set_calls[-1], torch.tensor(q["start"], dtype=torch.float32))


@pytest.mark.gpu
def test_plan_path_attached_object_and_failure():
    wl = json.load(open(os.path.join(GOLD, "workloads", "goal3_tallest_10box.json")))
    q = [x for x in wl["queries"] if x["attached"] >= 0][0]
    s = scenes.Scene.from_json(q["scene"])
    sc = M.Scene(s.boxes)
    sc.robot.q = torch.tensor(q["start"], dtype=torch.float32)
    pi = planning.PlannerInterface(sc.robot, sc)
    held = sc.entities[1 + q["attached"]]
    wps = pi.plan_path(qpos_goal=np.array(q["goal"]), num_waypoints=150, attached_object=held, timeout=10.0)
    assert len(wps) == 150 and pi.attached_object is held
    # the held box must not be exempt for the arm links: without exemption the
    # start (fingers around the block) is invalid when the fingers are closed on it
    assert pi._is_ompl_state_valid(q["start"]) is True
    # float64 0.04 fingers are out of float32 bounds -> [] (README.md:101-111)
    bad = np.array(q["start"])
    bad[7:] = 0.04
    assert pi.plan_path(qpos_goal=np.array(q["goal"]), qpos_start=bad, num_waypoints=150) == []


@pytest.mark.gpu
def test_inverse_kinematics_then_plan():
    """_ik_for_pose replacement (motion_primitives.py:131-134): IK of a grasp pose
    from the current qpos, then plan_path to it."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import franka_np
    wl = json.load(open(os.path.join(GOLD, "workloads", "goal3_tallest_10box.json")))
    q = wl["queries"][1]
    s = scenes.Scene.from_json(q["scene"])
    sc = M.Scene(s.boxes)
    sc.robot.q = torch.tensor(q["start"], dtype=torch.float32)
    pi = planning.PlannerInterface(sc.robot, sc)
    R, p = franka_np.hand_pose(q["goal"])
    qg = pi.inverse_kinematics(p, franka_np.mat_to_quat(R))
    assert isinstance(qg, torch.Tensor) and qg.dtype == torch.float32 and tuple(qg.shape) == (9,)
    R2, p2 = franka_np.hand_pose(qg.double().numpy())
    assert np.linalg.norm(p2 - p) < 1e-3 and pi.last_ik_status == 0
    wps = pi.plan_path(qpos_goal=qg, num_waypoints=150, timeout=10.0)
    assert len(wps) == 150
    assert pi.inverse_kinematics([3.0, 0.0, 0.5], [0.0, 1.0, 0.0, 0.0]) is None


class _FakeContext:
    """Stands in for native.Context (CPU test of planning.py's host logic only)."""

    def __init__(self, *a, **k):
        self.scenes = []
        self.attached = []

    def set_scene(self, boxes, plane_z, base):
        self.scenes.append([tuple(map(tuple, b[:2])) + (b[2],) for b in boxes])

    def set_attached(self, idx):
        self.attached.append(idx)

    def check_states(self, q):
        return np.ones(len(np.asarray(q).reshape(-1, 9)), dtype=np.uint8)

    def plan_async(self, *a, **k):
        pass

    def plan_wait(self, out=None):
        raise NativeError("rp_plan failed (-5): path_cap too small")

    def stats(self):
        return {}


def test_native_error_in_plan_returns_empty_and_restores(monkeypatch):
    """A library error inside rp_plan (capacity, HIP) becomes the reference's
    failure contract: [] + a warning, qpos restored (planning.py:190-205)."""
    monkeypatch.setattr(planning, "Context", _FakeContext)
    pi, sc = _mk([((0.65, 0.0, 0.02), (0.02, 0.02, 0.02), 0.0)])
    q0 = sc.robot.q.clone()
    assert pi.plan_path(model.SAFE_HOME, num_waypoints=150) == []
    assert pi.last_status == 0 and pi.last_stats is None
    assert torch.equal(sc.robot.set_calls[-1], q0)


def test_state_validity_uses_live_scene(monkeypatch):
    """_is_ompl_state_valid checks against the scene as it is now (the reference
    runs detect_collision on the live simulation, planning.py:209-219): a box moved
    after the last plan_path is seen by the next check."""
    monkeypatch.setattr(planning, "Context", _FakeContext)
    pi, sc = _mk([((0.65, 0.0, 0.02), (0.02, 0.02, 0.02), 0.0)])
    assert pi._is_ompl_state_valid(model.SAFE_HOME) is True
    sc.entities[1].set_pos((0.40, 0.2, 0.02))
    assert pi._is_ompl_state_valid(model.SAFE_HOME) is True
    seen = pi._ctx.scenes
    assert len(seen) == 2 and abs(seen[0][0][0][0] - 0.65) < 1e-6 and abs(seen[1][0][0][0] - 0.40) < 1e-6
