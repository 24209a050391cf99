"""Plan wall time of a workload with a given library build (A/B of variants):
python tools/plan_bench.py [LIB.so] [workload] [batch] [full] [sf]   (sf: straight edge first)"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rbe550_final_project_amd import _abi, model, native, scenes  # noqa: E402


def main():
    if len(sys.argv) > 1 and sys.argv[1].endswith(".so"):
        native.LIB_PATH = os.path.abspath(sys.argv.pop(1))
    name = sys.argv[1] if len(sys.argv) > 1 else "goal4_pentagon_10box"
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 262144
    batch_min = batch if "full" in sys.argv[3:] else 0
    sf = "sf" in sys.argv[3:]   # product default: straight edge first
    wl = json.load(open(os.path.join(ROOT, "tests", "golden", "workloads", name + ".json")))
    ctx = native.Context(0, model.robot_desc())
    for rep in range(3):
        t, tw = [], []
        for i, q in enumerate(wl["queries"]):
            sc = scenes.Scene.from_json(q["scene"])
            tw0 = time.perf_counter()
            ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
            ctx.set_attached(q["attached"])
            p = _abi.make_params(seed=i, batch=batch, batch_min=batch_min, n_waypoints=150, timeout_s=10.0,
                                 tree_capacity=1 << 24, straight_first=sf)
            t0 = time.perf_counter()
            ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
            t.append(1e3 * (time.perf_counter() - t0))
            tw.append(1e3 * (time.perf_counter() - tw0))
        print(f"{os.path.basename(native.LIB_PATH)} {'sf' if sf else 'rrt'} {name} batch {batch}: "
              f"total {sum(t):.2f} ms median {np.median(t):.3f} ms; with set_scene + set_attached: "
              f"median {np.median(tw):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
