"""Host side of the drop-in plan_path (code/planning.py:59-242) without a GPU: the
Genesis scene reader, the scene push only on change, the overlapped waypoint
tensors and the qpos restore, driven through a stand-in of native.Context that
follows rp_plan_async / rp_plan_wait's contract."""
import math

import numpy as np
import pytest
import torch

from rbe550_final_project_amd import _abi, model, planning, scenes
import mock_genesis as M

BOXES = [((0.65, 0.0, 0.02), (0.02, 0.02, 0.02), 0.0), ((0.5, 0.1, 0.02), (0.02, 0.03, 0.02), 0.7),
         ((0.3, -0.1, 0.2), (0.01, 0.02, 0.05), -2.5)]


class AsyncCtx:
    """rp_plan_async / rp_plan_wait stand-in: returns `path` (n, 9) float64."""

    def __init__(self, path):
        self.path = np.asarray(path, dtype=np.float64)
        self.scene_gen = 0
        self.scenes, self.attached, self.calls = [], [], []
        self.in_flight = False

    def set_scene_poses(self, poses, halves, plane_z, base, attached=-1):
        """rp_set_scene_poses' records: float32 of the centre, half extents and
        atan2 yaw (double)"""
        assert not self.in_flight and poses.dtype == np.float64 and halves.dtype == np.float32
        self.scene_gen += 1
        rec = np.empty((len(poses), 7), np.float32)
        for j, (x, y, z, w, qx, qy, qz) in enumerate(poses):
            rec[j, :3] = (x, y, z)
            rec[j, 3:6] = halves[j]
            rec[j, 6] = math.atan2(2.0 * (w * qz + qx * qy), 1.0 - 2.0 * (qy * qy + qz * qz))
        self.scenes.append((rec, plane_z, tuple(base)))
        self.attached.append(attached)

    def set_attached(self, idx):
        assert not self.in_flight
        self.scene_gen += 1
        self.attached.append(idx)

    def plan_async(self, start, goal, lo, hi, params, path_cap=4096):
        assert not self.in_flight
        self.in_flight = True
        self.calls.append((np.array(start), np.array(goal), params.n_waypoints, params.seed))

    def plan_wait(self, out=None):
        assert self.in_flight
        self.in_flight = False
        n = len(self.path)
        if out is not None and len(out) == n:
            np.copyto(out, self.path, casting="same_kind")
            return out, _abi.STATUS_EXACT
        return self.path.copy(), _abi.STATUS_EXACT

    def stats(self):
        return {"states_checked": 7}

    def check_states(self, q):
        return np.ones(len(np.asarray(q).reshape(-1, 9)), dtype=np.uint8)


def _path(n, seed=0):
    rng = np.random.default_rng(seed)
    return model.Q_LO + (model.Q_HI - model.Q_LO) * rng.random((n, 9))


@pytest.mark.parametrize("rigid_solver", [True, False])
def test_reader_matches_per_entity_scene(rigid_solver):
    """Batched link-pose reads and per-entity get_pos / get_quat give the same
    records, equal to the ctypes path's float32 rounding."""
    sc = M.Scene(BOXES, rigid_solver=rigid_solver)
    rd = scenes.GenesisReader(sc, sc.robot)
    assert (rd._links is not None) == rigid_solver
    poses, base = rd.poses()
    ctx = AsyncCtx(_path(2))
    ctx.set_scene_poses(np.array(poses, dtype=np.float64), rd.halves_f32, rd.plane_z, base)
    rec = ctx.scenes[-1][0]
    arr, n = _abi.make_boxes(rd.boxes(poses))
    assert n == 3 and np.array_equal(rec, np.frombuffer(arr, dtype=np.float32).reshape(-1, 7)[:n])
    assert np.allclose(rec[:, :3], [b[0] for b in BOXES]) and np.allclose(rec[:, 6], [b[2] for b in BOXES], atol=1e-6)
    assert np.allclose(base, model.BASE_POS)
    other = scenes.GenesisReader(M.Scene(BOXES, rigid_solver=not rigid_solver), sc.robot)
    assert np.array_equal(other.poses()[0], poses)


def test_scene_pushed_only_when_changed():
    sc = M.Scene(BOXES)
    pi = planning.PlannerInterface(sc.robot, sc)
    ctx = pi._ctx = AsyncCtx(_path(150))
    for _ in range(3):
        pi.plan_path(model.SAFE_HOME, num_waypoints=150)
    assert len(ctx.scenes) == 1 and ctx.attached == [-1]
    # attaching box 2 (entity 2): only the attachment is pushed
    pi.plan_path(model.SAFE_HOME, num_waypoints=150, attached_object=sc.entities[2])
    assert len(ctx.scenes) == 1 and ctx.attached == [-1, 1]
    # a block moved by the simulation: the scene is pushed again (with the attachment)
    sc.entities[1].set_pos((0.40, 0.2, 0.02))
    pi.plan_path(model.SAFE_HOME, num_waypoints=150, attached_object=sc.entities[2])
    assert len(ctx.scenes) == 2 and abs(float(ctx.scenes[-1][0][0, 0]) - 0.40) < 1e-6 and ctx.attached[-1] == 1
    # someone else set a scene on the context: pushed again although the poses are the same
    ctx.set_scene_poses(np.zeros((0, 7)), np.zeros((0, 3), np.float32), 0.0, (0, 0, 0))
    pi.plan_path(model.SAFE_HOME, num_waypoints=150, attached_object=sc.entities[2])
    assert len(ctx.scenes) == 4 and ctx.attached[-1] == 1


def test_waypoints_contract_and_restore():
    """150 float32 CPU tensors (9,) holding the planner's path rounded to float32;
    a later call never changes an earlier call's waypoints; qpos restored once."""
    sc = M.Scene(BOXES)
    q0 = sc.robot.q.clone()
    pi = planning.PlannerInterface(sc.robot, sc)
    p1 = _path(150, 1)
    ctx = pi._ctx = AsyncCtx(p1)
    w1 = pi.plan_path(model.SAFE_HOME, num_waypoints=150)
    assert isinstance(w1, list) and len(w1) == 150
    assert all(isinstance(w, torch.Tensor) and w.dtype == torch.float32 and tuple(w.shape) == (9,)
               and w.device.type == "cpu" for w in w1)
    assert np.array_equal(torch.stack(w1).numpy(), p1.astype(np.float32))
    assert len(sc.robot.set_calls) == 1 and torch.equal(sc.robot.set_calls[-1], q0)
    ctx.path = _path(150, 2)
    w2 = pi.plan_path(model.SAFE_HOME, num_waypoints=150)
    assert np.array_equal(torch.stack(w1).numpy(), p1.astype(np.float32))
    assert np.array_equal(torch.stack(w2).numpy(), ctx.path.astype(np.float32))
    # a path of another length than num_waypoints (e.g. a raw path longer than it)
    ctx.path = _path(203, 3)
    w3 = pi.plan_path(model.SAFE_HOME, num_waypoints=150)
    assert len(w3) == 203 and np.array_equal(torch.stack(w3).numpy(), ctx.path.astype(np.float32))
    assert pi.last_stats == {"states_checked": 7} and pi.last_timing["total_ms"] > 0
    # start = the current qpos (one get_qpos read), seeds advance per query
    starts = [c[0] for c in ctx.calls]
    assert all(np.array_equal(s, q0.numpy().astype(np.float64)) for s in starts)
    assert len({c[3] for c in ctx.calls}) == 3


def test_out_of_bounds_start_diagnosed_after_plan(caplog):
    """A start outside the float32 bounds: the plan reports INVALID_START (rp_plan
    applies OMPL's satisfiesBounds), then the reference's warnings follow."""
    sc = M.Scene(BOXES)
    pi = planning.PlannerInterface(sc.robot, sc)

    class Ctx(AsyncCtx):
        def plan_wait(self, out=None):
            self.in_flight = False
            return np.zeros((0, 9)), _abi.STATUS_INVALID_START

    pi._ctx = Ctx(_path(2))
    bad = np.array(model.SAFE_HOME, dtype=float)
    bad[7:] = 0.04
    with caplog.at_level("WARNING"):
        assert pi.plan_path(model.SAFE_HOME, qpos_start=bad, num_waypoints=150) == []
    text = caplog.text
    assert "OMPL start state out of bounds" in text and "State violates bounds on joints" in text
    assert "Path planning failed" in text
