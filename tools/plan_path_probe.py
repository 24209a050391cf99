"""Where PlannerInterface.plan_path's host time goes on the GPU box: each piece of
the call timed alone over the goal3 workload (mock Genesis scene), medians in us.

    python tools/plan_path_probe.py
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
from rbe550_final_project_amd import _abi, model, planning, scenes  # noqa: E402
from rbe550_final_project_amd.native import Context  # noqa: E402


def med(xs):
    return round(1e6 * float(np.median(xs)), 2)


def main():
    wl = json.load(open(os.path.join(ROOT, "tests", "golden", "workloads", "goal3_tallest_10box.json")))
    ctx = Context(0, model.robot_desc())
    q0 = scenes.Scene.from_json(wl["queries"][0]["scene"])
    sim = M.Scene(q0.boxes)
    pi = planning.PlannerInterface(sim.robot, sim)
    pi._ctx = ctx
    rd = scenes.GenesisReader(sim, pi.robot)
    T = {k: [] for k in ("poses", "set_scene_poses", "set_attached", "unbind150", "get_qpos",
                         "set_qpos", "plan_sync", "plan_async_wait", "plan_async_unbind_wait", "plan_path",
                         "plan_path_same_scene", "empty_call", "reference_tensor_list")}
    sink = io.StringIO()
    lo, hi = pi._bounds()
    for rep in range(12):
        for qi, q in enumerate(wl["queries"]):
            sc = scenes.Scene.from_json(q["scene"])
            for ent, (c, h, yaw) in zip(sim.entities[1:], sc.boxes):
                ent.set_pos(c)
                ent._quat = np.array([np.cos(yaw / 2), 0.0, 0.0, np.sin(yaw / 2)])
            sim.robot.q = torch.tensor(q["start"], dtype=torch.float32)
            t = time.perf_counter()
            poses, base = rd.poses()
            T["poses"].append(time.perf_counter() - t)
            t = time.perf_counter()
            ctx.set_scene_poses(np.array(poses, dtype=np.float64).reshape(-1, 7), rd.halves_f32, rd.plane_z,
                                np.array(base, dtype=np.float64), q["attached"])
            T["set_scene_poses"].append(time.perf_counter() - t)
            t = time.perf_counter()
            ctx.set_attached(q["attached"])
            T["set_attached"].append(time.perf_counter() - t)
            t = time.perf_counter()
            qc = sim.robot.get_qpos()
            T["get_qpos"].append(time.perf_counter() - t)
            t = time.perf_counter()
            sim.robot.set_qpos(qc)
            T["set_qpos"].append(time.perf_counter() - t)
            t = time.perf_counter()
            v = torch.empty((150, 9)).unbind(0)
            T["unbind150"].append(time.perf_counter() - t)
            p = _abi.make_params(seed=qi, batch=4096, n_waypoints=150, timeout_s=10.0, straight_first=False)
            start = np.asarray(q["start"], dtype=np.float64)
            goal = np.asarray(q["goal"], dtype=np.float64)
            t = time.perf_counter()
            ctx.plan(start, goal, lo, hi, p)
            T["plan_sync"].append(time.perf_counter() - t)
            t = time.perf_counter()
            ctx.plan_async(start, goal, lo, hi, p)
            ctx.plan_wait()
            T["plan_async_wait"].append(time.perf_counter() - t)
            out = np.empty((150, 9), np.float32)
            t = time.perf_counter()
            ctx.plan_async(start, goal, lo, hi, p)
            v = torch.empty((150, 9)).unbind(0)
            ctx.plan_wait(out)
            T["plan_async_unbind_wait"].append(time.perf_counter() - t)
            planning.configure(seed=qi, straight_first=False)
            held = sim.entities[1 + q["attached"]] if q["attached"] >= 0 else None
            with contextlib.redirect_stdout(sink):
                t = time.perf_counter()
                pi.plan_path(qpos_goal=goal, num_waypoints=150, attached_object=held, timeout=10.0)
                T["plan_path"].append(time.perf_counter() - t)
                t = time.perf_counter()
                pi.plan_path(qpos_goal=goal, num_waypoints=150, attached_object=held, timeout=10.0)
                T["plan_path_same_scene"].append(time.perf_counter() - t)
            t = time.perf_counter()
            len(v)
            T["empty_call"].append(time.perf_counter() - t)
            # the reference's own conversion of a 150-state path (code/planning.py:232-242:
            # one torch.tensor of a 9-float list per state), for scale
            path = np.linspace(0.0, 1.0, 150 * 9).reshape(150, 9)
            t = time.perf_counter()
            [torch.tensor([float(s[i]) for i in range(9)], dtype=torch.float32) for s in path]
            T["reference_tensor_list"].append(time.perf_counter() - t)
            sink.seek(0)
            sink.truncate()
    planning.configure(straight_first=True)
    print(json.dumps({k: med(v[21:]) for k, v in T.items()}, indent=1))


if __name__ == "__main__":
    main()
