"""Host-side cost of PlannerInterface.plan_path without a GPU (diagnostic tool): the
C3 queries through tests/mock_genesis.py as bench.py's C3_plan_path leg runs them,
on a stub context whose plan_async / plan_wait return a straight 150-waypoint path
at once. What is left is everything plan_path does on the host besides the GPU
query: scene ingestion, argument checks, parameter packing, the waypoint tensors.
python tools/plan_path_host.py [--profile]"""
import contextlib
import cProfile
import io
import json
import os
import pstats
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import mock_genesis as M  # noqa: E402
from rbe550_final_project_amd import _abi, planning, scenes  # noqa: E402


class StubCtx:
    scene_gen = 0

    def __init__(self):
        self._q = None

    def reserve(self, batch, cap):
        pass

    def set_scene_poses(self, P, halves, plane_z, base, idx):
        self.scene_gen += 1

    def set_attached(self, idx):
        pass

    def plan_async(self, start, goal, lo, hi, p, path_cap=0):
        self._q = (start, goal, p.n_waypoints)

    def plan_wait(self, out=None):
        s, g, n = self._q
        t = np.linspace(0.0, 1.0, n)[:, None]
        path = s[None, :] * (1 - t) + g[None, :] * t
        if out is not None:
            out[:] = path
            return out, _abi.STATUS_EXACT
        return path, _abi.STATUS_EXACT

    def stats(self):
        return {"states_checked": 0}


def main():
    wl = json.load(open(os.path.join(ROOT, "tests/golden/workloads/goal3_tallest_10box.json")))
    q0 = scenes.Scene.from_json(wl["queries"][0]["scene"])
    sim = M.Scene(q0.boxes)
    pi = planning.PlannerInterface(sim.robot, sim)
    pi._ctx = StubCtx()
    sink = io.StringIO()
    prepared = []
    for q in wl["queries"]:
        sc = scenes.Scene.from_json(q["scene"])
        prepared.append((sc, q))

    def one_pass(times):
        for sc, q in prepared:
            for ent, (c, h, yaw) in zip(sim.entities[1:], sc.boxes):
                ent.set_pos(c)
                ent._quat = np.array([np.cos(yaw / 2), 0.0, 0.0, np.sin(yaw / 2)])
            sim.robot.q = torch.tensor(q["start"], dtype=torch.float32)
            held = sim.entities[1 + q["attached"]] if q["attached"] >= 0 else None
            goal = np.array(q["goal"], dtype=float)
            with contextlib.redirect_stdout(sink):
                t0 = time.perf_counter()
                wps = pi.plan_path(qpos_goal=goal, num_waypoints=150, attached_object=held, timeout=10.0)
                times.append((1e3 * (time.perf_counter() - t0), pi.last_timing))
            sink.seek(0)
            sink.truncate()
            assert len(wps) == 150

    for _ in range(3):
        one_pass([])
    times = []
    for _ in range(20):
        one_pass(times)
    tot = np.median([t for t, _ in times])
    parts = {k: np.median([p[k] for _, p in times]) for k in ("scene_ms", "rp_plan_ms", "other_ms")}
    print(f"plan_path host-only median {tot:.4f} ms  " + "  ".join(f"{k} {v:.4f}" for k, v in parts.items()))
    if "--profile" in sys.argv:
        pr = cProfile.Profile()
        pr.enable()
        one_pass([])
        one_pass([])
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
