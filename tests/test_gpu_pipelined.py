"""Pipelined queries (BASELINE config 3: goal3's ~21 RRT queries "pipelined"):
rp_plan_many (native.plan_pipelined) keeps the workload's queries in flight on several
contexts of one GPU (each its own stream and planner thread). Every path, status, iteration count
and tree size equals the CPU oracle's for that query alone — the queries share
nothing. Call sites replayed: code/goal3_tallest.py:63-283 through
code/motion_primitives.py:144."""
import json
import os

import numpy as np
import pytest

from rbe550_final_project_amd import _abi, build, model, native, scenes

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "workloads")


def _jobs(wl, straight_first, batch=4096):
    qs = json.load(open(os.path.join(GOLD, wl + ".json")))["queries"]
    return [{"scene": scenes.Scene.from_json(q["scene"]), "attached": q["attached"], "start": q["start"],
             "goal": q["goal"], "lo": model.Q_LO, "hi": model.Q_HI,
             "params": _abi.make_params(seed=i, batch=batch, n_waypoints=150, timeout_s=60,
                                        straight_first=straight_first)} for i, q in enumerate(qs)]


@pytest.fixture(scope="module")
def ctxs():
    build.build(verbose=False)
    cs = [native.Context(device=0, robot=model.robot_desc()) for _ in range(4)]
    for c in cs:
        c.reserve(4096, 0)
    yield cs
    for c in cs:
        c.close()


@pytest.mark.parametrize("wl", ["goal3_tallest_10box", "goal1_scattered_6box"])
@pytest.mark.parametrize("straight_first", [True, False])
@pytest.mark.parametrize("k", [2, 4])
def test_pipelined_plans_equal_the_oracle(ctxs, oracle_lib, wl, straight_first, k):
    jobs = _jobs(wl, straight_first)
    got = native.plan_pipelined(ctxs[:k], jobs)
    o = oracle_lib.OracleScene()
    for i, (job, (path, st, s)) in enumerate(zip(jobs, got)):
        sc = job["scene"]
        o.set_scene(sc.boxes, sc.plane_z, sc.base)
        o.set_attached(job["attached"])
        ref, st_ref, sref = o.plan(job["start"], job["goal"], model.Q_LO, model.Q_HI, job["params"])
        assert st == st_ref == _abi.STATUS_EXACT, (wl, i)
        assert path.shape == ref.shape == (150, 9) and np.array_equal(path, ref), (wl, i)
        if s is not None:   # (a context's stats are its last query's)
            assert s["iterations"] == sref["iterations"], (wl, i)
            if not straight_first:
                assert (s["start_tree_size"], s["goal_tree_size"]) == (sref["start_tree_size"],
                                                                       sref["goal_tree_size"])
    assert sum(s is not None for _, _, s in got) == k


def test_pipelined_reports_a_failed_query_and_finishes_the_rest(ctxs):
    """A query the library refuses (path capacity too small for its waypoints) raises
    after every other query in flight has been waited for; the contexts stay usable."""
    jobs = _jobs("goal3_tallest_10box", True)[:6]
    with pytest.raises(native.NativeError):
        native.plan_pipelined(ctxs[:3], jobs, path_cap=8)
    got = native.plan_pipelined(ctxs[:3], jobs)
    assert all(st == _abi.STATUS_EXACT for _, st, _ in got)


def test_pipelined_rejects_tilted_scenes_and_busy_contexts(ctxs):
    """rp_query carries upright boxes (rp_set_scene records): a tilted scene is refused
    before anything runs; so is a context already planning (RP_ERR_STATE)."""
    import tilt_scenes as T
    job = _jobs("goal3_tallest_10box", True)[0]
    with pytest.raises(ValueError):
        native.plan_pipelined(ctxs[:2], [dict(job, scene=T.toppled_goal3())])
    ctxs[0].plan_async(job["start"], job["goal"], model.Q_LO, model.Q_HI, job["params"])
    try:
        with pytest.raises(native.NativeError):
            native.plan_pipelined(ctxs[:2], [job, job])
    finally:
        ctxs[0].plan_wait()
