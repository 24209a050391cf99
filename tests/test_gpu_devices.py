"""Multi-GPU planning through the reference's own API, in one process
(planning.configure(devices=[...]) / RBE_PLANNER_DEVICES): PlannerInterface opens one
context per device, rp_group_init_local makes them one rank group, and every
plan_path query runs on all of them from their planner threads (the reference drives
one planner from one process: code/motion_primitives.py:38, 144; batched envs are
rejected, code/planning.py:121-122). On the one-GPU box the contexts share device 0
(the in-process shared-segment transport); the returned path is rank 0's and must
equal the world-1 plan, the golden plan and the oracle's."""
import json
import os

import numpy as np
import pytest
import torch

from rbe550_final_project_amd import _abi, model, native, planning, scenes
import mock_genesis as M

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
FIX = np.load(os.path.join(GOLD, "plans_configured.npz"))
META = json.loads(str(FIX["meta"]))


def _plan_path(devices, m, q):
    """plan_path with the golden case's parameters through the Genesis mock."""
    sc = scenes.Scene.from_json(q["scene"])
    sim = M.Scene(sc.boxes)
    planning.configure(seed=m["seed"], batch=m["batch"], batch_min=m["batch"], straight_first=False,
                       tree_capacity=1 << 23, devices=devices)
    try:
        pl = planning.PlannerInterface(sim.robot, sim)
        held = sim.entities[1 + q["attached"]] if q["attached"] >= 0 else None
        wps = pl.plan_path(qpos_goal=np.array(q["goal"]), qpos_start=np.array(q["start"]), num_waypoints=150,
                           attached_object=held, timeout=600.0)
        stats = pl.last_stats
        ranks = [c.group_info() for c in pl._ctxs]
        ing = scenes.GenesisReader(sim, sim.robot).read()
        return (torch.stack(wps).numpy() if wps else None), pl.last_status, stats, ranks, ing, pl
    finally:
        planning.configure(seed=0, batch=4096, batch_min=0, straight_first=True, tree_capacity=0, devices=())


@pytest.mark.parametrize("name", ["C4_q10", "C5_well_s3", "C5_well_s4"])
@pytest.mark.parametrize("devices", [(0, 0), (0, 0, 0, 0)])
def test_plan_path_on_devices_equals_golden_and_oracle(oracle_lib, name, devices):
    """plan_path with 2 and 4 contexts on device 0 (one rank group, shared-segment
    transport; the configured 262,144- / 131,072-sample iterations are sharded): the
    same path, status and trees as the one-context planner, the oracle on the ingested
    scene, and the golden plan where the ingested scene is the golden scene (no yawed
    boxes: the mock's float32 quaternion moves a yaw in its last bits)."""
    m = META[name]
    q = json.load(open(os.path.join(GOLD, "workloads", m["workload"] + ".json")))["queries"][m["query"]]
    got, st, s, ranks, ing, pl = _plan_path(devices, m, q)
    assert [r["rank"] for r in ranks] == list(range(len(devices)))
    assert all(r["world"] == len(devices) and r["transport"] == "shm" for r in ranks), ranks
    assert st == m["status"] and got is not None and got.shape == (150, 9)
    assert s["iterations"] == m["iterations"]
    one, st1, s1, _, _, _ = _plan_path((0,), m, q)
    assert st1 == st and np.array_equal(one, got)
    assert (s1["start_tree_size"], s1["goal_tree_size"]) == (s["start_tree_size"], s["goal_tree_size"])
    if all(not _abi.is_quat(r) and r == 0.0 for _, _, r in ing.boxes):
        assert np.array_equal(got, FIX[name].astype(np.float32))
    o = oracle_lib.OracleScene()
    o.set_scene(ing.boxes, ing.plane_z, ing.base)
    o.set_attached(q["attached"])
    p = _abi.make_params(seed=m["seed"], batch=m["batch"], batch_min=m["batch"], n_waypoints=150, timeout_s=600.0,
                         straight_first=False, tree_capacity=1 << 23)
    lo, hi = pl._bounds()
    ref, st_ref, _ = o.plan(q["start"], q["goal"], lo, hi, p)
    assert st_ref == st and np.array_equal(got, ref.astype(np.float32))


def test_devices_from_env(monkeypatch):
    """RBE_PLANNER_DEVICES="0,0" makes the planner a 2-rank group with no code change
    in the caller (the goal scripts run unchanged)."""
    monkeypatch.setenv("RBE_PLANNER_DEVICES", "0,0")
    q = json.load(open(os.path.join(GOLD, "workloads", "goal3_tallest_10box.json")))["queries"][0]
    sc = scenes.Scene.from_json(q["scene"])
    sim = M.Scene(sc.boxes)
    sim.robot.q = torch.tensor(q["start"], dtype=torch.float32)
    pl = planning.PlannerInterface(sim.robot, sim)
    wps = pl.plan_path(qpos_goal=np.array(q["goal"]), num_waypoints=150, timeout=10.0)
    assert len(wps) == 150 and len(pl._ctxs) == 2
    assert pl._ctxs[1].group_info() == {"rank": 1, "world": 2, "transport": "shm"}


def test_group_init_local_rejects_rccl_on_one_device():
    """RCCL needs distinct GPUs (ncclCommInitAll); contexts sharing a device are an
    argument error for it, and fine for the shared segment."""
    a = native.Context(device=0, robot=model.robot_desc())
    b = native.Context(device=0, robot=model.robot_desc())
    try:
        with pytest.raises(native.NativeError):
            native.group_init_local([a, b], transport="rccl")
        native.group_init_local([a, b], transport="shm")
        assert b.group_info() == {"rank": 1, "world": 2, "transport": "shm"}
        native.group_init_local([a])   # world 1: back to single-rank planning
        assert a.group_info()["world"] == 1
    finally:
        b.close()
        a.close()


def test_failed_grouped_plan_reforms_the_group():
    """one failing rank must not disable the planner. Rank 1's next plan is
    made to fail (rp_debug_fail_next); rank 0 stops at its first exchange at once (the
    failed rank publishes a broken sequence word) instead of waiting out the watchdog;
    plan_path returns [] as the reference does on failure, re-forms the rank group, and
    the next plan_path returns the golden plan."""
    import time
    m = META["C5_well_s3"]
    q = json.load(open(os.path.join(GOLD, "workloads", m["workload"] + ".json")))["queries"][m["query"]]
    sc = scenes.Scene.from_json(q["scene"])
    sim = M.Scene(sc.boxes)
    planning.configure(seed=m["seed"], batch=m["batch"], batch_min=m["batch"], straight_first=False,
                       tree_capacity=1 << 23, devices=(0, 0))
    try:
        pl = planning.PlannerInterface(sim.robot, sim)
        kw = dict(qpos_goal=np.array(q["goal"]), qpos_start=np.array(q["start"]), num_waypoints=150, timeout=600.0)
        first = torch.stack(pl.plan_path(**kw)).numpy()   # (the golden seed: configure reset the count)
        assert pl.last_status == m["status"]
        assert native.load().rp_debug_fail_next(pl._ctxs[1]._h) == 0
        t0 = time.perf_counter()
        assert pl.plan_path(**kw) == []
        assert time.perf_counter() - t0 < 10.0   # (not the 120 s watchdog)
        planning.configure(seed=m["seed"])
        again = pl.plan_path(**kw)
        assert len(again) == 150 and np.array_equal(torch.stack(again).numpy(), first)
        assert [c.group_info()["world"] for c in pl._ctxs] == [2, 2]
    finally:
        planning.configure(seed=0, batch=4096, batch_min=0, straight_first=True, tree_capacity=0, devices=())


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs (the RCCL transport between devices)")
@pytest.mark.parametrize("name", ["C4_q10", "C5_well_s3"])
def test_plan_path_on_distinct_devices_rccl(oracle_lib, name):
    """the in-process RCCL group (rp_group_init_local over distinct GPUs,
    ncclCommInitAll; the default when devices differ): plans complete without deadlock
    and equal the one-context plan. Skipped on a one-GPU box."""
    m = META[name]
    q = json.load(open(os.path.join(GOLD, "workloads", m["workload"] + ".json")))["queries"][m["query"]]
    devs = tuple(range(min(torch.cuda.device_count(), 4)))
    got, st, s, ranks, ing, pl = _plan_path(devs, m, q)
    assert all(r["transport"] == "rccl" and r["world"] == len(devs) for r in ranks), ranks
    one, st1, s1, _, _, _ = _plan_path((0,), m, q)
    assert st == st1 == m["status"] and np.array_equal(one, got)
    assert (s1["start_tree_size"], s1["goal_tree_size"]) == (s["start_tree_size"], s["goal_tree_size"])
