"""Steady-state validity throughput (4M-state launches) per scene and state
distribution: uniform in the bounds, and near the workload's start configurations
(the region a plan's edges sweep)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rbe550_final_project_amd import model, scenes  # noqa: E402
from rbe550_final_project_amd.native import Context  # noqa: E402


def main():
    n = 1 << 22
    ctx = Context(0, model.robot_desc())
    s = torch.cuda.Stream()
    rng = np.random.default_rng(0)
    for wname in ("goal3_tallest_10box", "goal4_pentagon_10box", "clutter64"):
        wl = json.load(open(os.path.join(ROOT, "tests", "golden", "workloads", wname + ".json")))
        q0 = wl["queries"][min(14, len(wl["queries"]) - 1)]
        sc = scenes.Scene.from_json(q0["scene"])
        ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
        uni = model.Q_LO + (model.Q_HI - model.Q_LO) * rng.random((n, 9))
        near = np.clip(np.asarray(q0["start"])[None, :] + rng.normal(0, 0.5, (n, 9)), model.Q_LO, model.Q_HI)
        for name, arr in (("uniform", uni), ("near-start", near)):
            q = torch.from_numpy(arr.astype(np.float32)).cuda()
            f = torch.empty(n, dtype=torch.uint8, device="cuda")
            for _ in range(3):
                ctx.check_states_device(q.data_ptr(), n, f.data_ptr(), s.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(10):
                ctx.check_states_device(q.data_ptr(), n, f.data_ptr(), s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 10
            print(f"{wname:22s} {name:10s} {n / ms / 1e6:7.2f} G states/s  valid {f.float().mean().item():.3f}",
                  flush=True)


if __name__ == "__main__":
    main()
