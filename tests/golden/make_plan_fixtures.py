"""Golden plans at the BASELINE configs' own batch sizes, from the CPU oracle.

    python tests/golden/make_plan_fixtures.py   -> tests/golden/plans_configured.npz

The GPU planner must reproduce these bit for bit (tests/test_gpu_configs.py);
they are generated once here because the oracle needs minutes for them (the
covered-well C5 query grows trees of 10^5 nodes whose brute-force NN dominates).
Cases (RRT-Connect forced, batch_min = batch, 150 waypoints, simplify level 1):

  C2  single_pick_place_5box, both queries, 65,536-sample iterations, seeds 0-2
  C4  goal4_pentagon_10box, every 5th query, 262,144-sample iterations
  C4  goal4_pentagon_ring (the completed pentagon, deep grasps between placed
      blocks: no straight edge), queries 0 / 3 / 5 / 8, 262,144-sample iterations
  C5  clutter64, 131,072-sample iterations
  C5  clutter64_well (goal inside a covered well), 131,072-sample iterations,
      max 8 iterations (= the 2^20-sample budget): seeds 2, 3, 4 solve in 6, 7
      and 3 iterations, seed 0 exhausts the budget (APPROXIMATE)

Each case stores the oracle's status, 150 x 9 float64 waypoints, iteration count
and final tree sizes. The oracle is test infrastructure (oracle/); this script
is how its outputs become committed vectors.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle.oracle import OracleScene  # noqa: E402
from rbe550_final_project_amd import _abi, model, scenes  # noqa: E402

GOLD = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(GOLD, "plans_configured.npz")


def cases():
    """(name, workload, query index, seed, batch, max_iters)"""
    out = []
    for qi in (0, 1):
        for seed in (0, 1, 2):
            out.append((f"C2_q{qi}_s{seed}", "single_pick_place_5box", qi, seed, 65536, 0))
    for qi in range(0, 25, 5):
        out.append((f"C4_q{qi}", "goal4_pentagon_10box", qi, qi, 262144, 0))
    for qi in (0, 3, 5, 8):   # the completed ring: no valid straight edge (make_workloads.py)
        out.append((f"C4_ring_q{qi}", "goal4_pentagon_ring", qi, qi, 262144, 0))
    out.append(("C5_clutter64", "clutter64", 0, 0, 131072, 0))
    for seed in (2, 3, 4, 0):
        out.append((f"C5_well_s{seed}", "clutter64_well", 0, seed, 131072, 8))
    return out


def params(seed, batch, max_iters):
    return _abi.make_params(seed=seed, batch=batch, batch_min=batch, n_waypoints=150, timeout_s=3600.0,
                            straight_first=False, tree_capacity=1 << 23, max_iters=max_iters)


def main():
    only = set(sys.argv[1:])
    data = dict(np.load(OUT)) if os.path.exists(OUT) else {}
    meta = json.loads(str(data.pop("meta"))) if "meta" in data else {}
    for name, wl, qi, seed, batch, max_iters in cases():
        if only and name not in only:
            continue
        q = json.load(open(os.path.join(GOLD, "workloads", wl + ".json")))["queries"][qi]
        sc = scenes.Scene.from_json(q["scene"])
        o = OracleScene()
        o.set_scene(sc.boxes, sc.plane_z, sc.base)
        o.set_attached(q["attached"])
        t0 = time.time()
        path, st, stats = o.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, params(seed, batch, max_iters))
        data[name] = path
        meta[name] = {"workload": wl, "query": qi, "seed": seed, "batch": batch, "max_iters": max_iters,
                      "status": st, "iterations": stats["iterations"], "start_tree": stats["start_tree_size"],
                      "goal_tree": stats["goal_tree_size"], "oracle_s": round(time.time() - t0, 1)}
        print(name, meta[name], flush=True)
    np.savez_compressed(OUT, meta=np.array(json.dumps(meta)), **data)


if __name__ == "__main__":
    main()
