"""Host-side cost of PlannerInterface.plan_path without a GPU: the Context is a
stand-in whose plan() returns a canned 150-waypoint path at once, so what is timed
is everything plan_path does around rp_plan (scene ingestion, argument checks,
bounds, params, the waypoint tensors, restoring qpos). CPU only; dev tool.

    python tools/plan_path_host.py [--profile]
"""
import contextlib
import io
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import mock_genesis as M  # noqa: E402
from rbe550_final_project_amd import _abi, planning, scenes  # noqa: E402


class FakeCtx:
    def __init__(self):
        self.path = np.linspace(0, 1, 150 * 9).reshape(150, 9)
        self.scene_gen = 0
        self.uploads = 0

    def set_scene(self, boxes, plane_z=0.0, base=(0, 0, 0.01)):
        _abi.make_boxes(boxes)
        self.scene_gen += 1
        self.uploads += 1

    def set_attached(self, i, mask=_abi.ATTACH_EXEMPT_MASK):
        self.scene_gen += 1

    def plan_async(self, start, goal, lo, hi, params, path_cap=4096):
        np.asarray(start, dtype=np.float64)

    def plan_wait(self, out=None):
        if out is not None and len(out) == len(self.path):
            np.copyto(out, self.path, casting="same_kind")
            return out, _abi.STATUS_EXACT
        return self.path.copy(), _abi.STATUS_EXACT

    def stats(self):
        return {"states_checked": 1}


def main():
    wl = json.load(open(os.path.join(ROOT, "tests", "golden", "workloads", "goal3_tallest_10box.json")))
    q0 = scenes.Scene.from_json(wl["queries"][0]["scene"])
    sim = M.Scene(q0.boxes)
    pi = planning.PlannerInterface(sim.robot, sim)
    pi._ctx = FakeCtx()
    sink = io.StringIO()
    times = []
    parts = {"scene_ms": [], "rp_plan_ms": [], "other_ms": []}

    def run(n):
        for _ in range(n):
            for q in wl["queries"]:
                sc = scenes.Scene.from_json(q["scene"])
                for ent, (c, h, yaw) in zip(sim.entities[1:], sc.boxes):
                    ent.set_pos(c)
                    ent._quat = np.array([np.cos(yaw / 2), 0.0, 0.0, np.sin(yaw / 2)])
                sim.robot.q = torch.tensor(q["start"], dtype=torch.float32)
                held = sim.entities[1 + q["attached"]] if q["attached"] >= 0 else None
                goal = np.array(q["goal"], dtype=float)
                with contextlib.redirect_stdout(sink):
                    t0 = time.perf_counter()
                    pi.plan_path(qpos_goal=goal, num_waypoints=150, attached_object=held, timeout=10.0)
                    times.append(1e3 * (time.perf_counter() - t0))
                for k in parts:
                    parts[k].append(pi.last_timing[k])
                sink.seek(0)
                sink.truncate()

    run(5)
    times.clear()
    for k in parts:
        parts[k].clear()
    if "--profile" in sys.argv:
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        run(20)
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(25)
    else:
        run(20)
    print("uploads", pi._ctx.uploads, "plan_path host median %.4f ms" % np.median(times),
          {k: round(float(np.median(v)), 4) for k, v in parts.items()})


if __name__ == "__main__":
    main()
