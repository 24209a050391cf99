"""Plan wall time at the BASELINE configured iteration sizes (RRT-Connect forced,
batch_min = batch) for several first sub-batch sizes (RBE_PLAN_CHUNK, read by
rp_plan on every call): python tools/chunk_sweep.py [chunk ...]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rbe550_final_project_amd import _abi, model, native, scenes  # noqa: E402

CONFIGS = [("C2", "single_pick_place_5box", 65536, 10, 0), ("C4", "goal4_pentagon_10box", 262144, 1, 0),
           ("C5_clutter64", "clutter64", 131072, 1, 0), ("C5_well", "clutter64_well", 131072, 4, 8)]


def run(ctx, name, batch, reps, max_iters):
    wl = json.load(open(os.path.join(ROOT, "tests", "golden", "workloads", name + ".json")))
    t, samples = [], 0
    for rep in range(reps):
        for i, q in enumerate(wl["queries"]):
            sc = scenes.Scene.from_json(q["scene"])
            ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
            ctx.set_attached(q["attached"])
            p = _abi.make_params(seed=i + rep * (name == "clutter64_well"), batch=batch, batch_min=batch,
                                 n_waypoints=150, timeout_s=10.0, tree_capacity=1 << 23, straight_first=False,
                                 max_iters=max_iters)
            t0 = time.perf_counter()
            ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
            t.append(1e3 * (time.perf_counter() - t0))
            samples += ctx.stats()["samples"]
    return t, samples


def main():
    chunks = sys.argv[1:] or ["-1", "256", "1024", "4096"]
    ctx = native.Context(0, model.robot_desc())
    for key, name, batch, reps, mi in CONFIGS:   # warm-up
        run(ctx, name, batch, 1, mi)
    for ch in chunks:
        os.environ["RBE_PLAN_CHUNK"] = ch
        for key, name, batch, reps, mi in CONFIGS:
            t, samples = run(ctx, name, batch, reps, mi)
            print(f"chunk {ch:>6} {key:13s} batch {batch}: median {np.median(t):.3f} ms  total {sum(t):.2f} ms "
                  f"(n={len(t)}, samples processed {samples})", flush=True)


if __name__ == "__main__":
    main()
