"""GPU test of the rank-group path of rp_plan (sharded speculative iterations, one
record all-gather each) on ONE GPU: world 2 / 4 contexts planned from host threads
with the host transport (the all-gather is a numpy concatenation between threads).
The plan must equal the world-1 plan and the CPU oracle (SURVEY.md §8(e)
acceptance: result independent of world size). Separate processes with
torch.distributed: tests/test_gpu_group_procs.py; RCCL: tests/test_gpu_configs.py
(world 1 on one GPU) and bench.py at N > 1."""
import json
import os
import threading

import numpy as np
import pytest
import torch

from rbe550_final_project_amd import _abi, model, scenes
from rbe550_final_project_amd.native import Context

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


class ThreadGroup:
    """world ranks in one process (host transport): each rank's callback gets numpy
    views of its pinned send / recv buffers; barrier, stage, barrier, gather."""

    def __init__(self, world):
        self.world = world
        self.stage = [None] * world
        self.bar = threading.Barrier(world, timeout=120)   # a failed rank breaks it, no hang
        self.calls = 0

    def fn(self, rank):
        def allgather(send, recv):
            self.stage[rank] = send.copy()
            self.bar.wait()
            if rank == 0:
                self.calls += 1
            recv[:] = np.concatenate(self.stage)
            self.bar.wait()
        return allgather


@pytest.mark.parametrize("wl,qi,batch", [("goal4_pentagon_10box", 2, 64), ("goal3_tallest_10box", 5, 256),
                                         ("clutter64", 0, 128)])
@pytest.mark.parametrize("packed,world,straight", [("", 2, False), ("1", 2, False), ("", 4, False), ("", 2, True)])
def test_two_rank_plan_equals_single(oracle_lib, wl, qi, batch, packed, world, straight, monkeypatch):
    """World 2 and 4 (ranks as threads on one GPU); packed "1": the ranks' connect
    launches are work-compacted (k_edges_packed); straight: the product default
    (straight edge first: every rank decides alone, no exchange when it is valid)."""
    if packed:
        monkeypatch.setenv("RBE_EDGE_PACKED", packed)
    q = json.load(open(os.path.join(GOLD, "workloads", wl + ".json")))["queries"][qi]
    sc = scenes.Scene.from_json(q["scene"])
    p = _abi.make_params(seed=13, batch=batch, n_waypoints=150, timeout_s=60, straight_first=straight)
    g = ThreadGroup(world)
    ctxs = []
    for r in range(world):
        c = Context(device=0, robot=model.robot_desc())
        c.set_scene(sc.boxes, sc.plane_z, sc.base)
        c.set_attached(q["attached"])
        c.group_init(r, world, g.fn(r))
        ctxs.append(c)
    out = [None] * world

    def run(r):
        out[r] = ctxs[r].plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    [t.start() for t in th]
    [t.join(timeout=300) for t in th]
    assert all(o is not None for o in out), "a rank did not finish"
    single = Context(device=0, robot=model.robot_desc())
    single.set_scene(sc.boxes, sc.plane_z, sc.base)
    single.set_attached(q["attached"])
    ref, st = single.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
    o = oracle_lib.OracleScene()
    o.set_scene(sc.boxes, sc.plane_z, sc.base)
    o.set_attached(q["attached"])
    ref_cpu, st_cpu, _ = o.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
    assert g.calls >= (0 if straight else 1)
    for path, status in out:
        assert status == st == st_cpu == _abi.STATUS_EXACT
        assert np.array_equal(path, ref) and np.array_equal(path, ref_cpu)
    for c in ctxs + [single]:
        c.close()
