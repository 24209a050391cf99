"""C5 covered-well plans (131,072-sample iterations) under execution knobs set per
plan (rp_plan reads them on every call): RBE_NN_MFMA (matrix-core / packed-f32
nearest node), RBE_PLAN_CHUNK (first sub-batch; -1 = whole iteration). Prints
wall time and the kernel-class profile per configuration (median of the seeds).
python tools/well_ab.py [NAME=ENV1:V,ENV2:V ...]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rbe550_final_project_amd import _abi, model, scenes  # noqa: E402
from rbe550_final_project_amd.native import Context  # noqa: E402

CONFIGS = {
    "part_whole": {"RBE_NN_MFMA": "0", "RBE_PLAN_CHUNK": "-1"},
    "mfma4_w4_whole": {"RBE_NN_MFMA": "4", "RBE_PLAN_CHUNK": "-1"},
    "mfma4_w1_whole": {"RBE_NN_MFMA": "4", "RBE_NN_WAVES": "1", "RBE_PLAN_CHUNK": "-1"},
    "mfma8_w4_whole": {"RBE_NN_MFMA": "8", "RBE_PLAN_CHUNK": "-1"},
    "mfma4_w4_r1": {"RBE_NN_MFMA": "4", "RBE_PLAN_CHUNK": "-1", "RBE_NN_RANGES": "1"},
    "mfma4_w4_r8": {"RBE_NN_MFMA": "4", "RBE_PLAN_CHUNK": "-1", "RBE_NN_RANGES": "8"},
    "default": {},
}


def main():
    cfgs = CONFIGS
    if len(sys.argv) > 1:
        cfgs = {}
        for a in sys.argv[1:]:
            name, kv = a.split("=", 1)
            cfgs[name] = dict(x.split(":") for x in kv.split(","))
    q = json.load(open(os.path.join(ROOT, "tests/golden/workloads/clutter64_well.json")))["queries"][0]
    sc = scenes.Scene.from_json(q["scene"])
    ctx = Context(0)
    ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
    ctx.set_attached(q["attached"])
    # WELL_AB_PROF=0: profiling off (its events sit between the launches), wall times only
    ctx.set_profiling(os.environ.get("WELL_AB_PROF", "1") != "0")
    keys = ("RBE_NN_MFMA", "RBE_PLAN_CHUNK", "RBE_CHUNK_TREE", "RBE_NN_WAVES", "RBE_NN_RANGES", "RBE_EDGE_PACKED",
            "RBE_NN_BLOCKS", "RBE_NN_DEVGEOM", "RBE_NN_PILOT", "RBE_NN_GEOM_FIT",
            "RBE_EDGE_COARSE", "RBE_EDGE_COARSE_MIN", "RBE_EDGE_UNITS", "RBE_EARLY_STATUS", "RBE_ACCEPT_LB", "RBE_WAIT_SPIN_US", "RBE_WAIT_SLEEP_FRAC",
            "RBE_PLAN_PIPELINE", "RBE_PLAN_SPECULATE", "RBE_SCENE_LDS", "RBE_NN_SHARE")
    for rep in range(2):   # rep 0: warm-up
        for name, env in cfgs.items():
            for k in keys:
                os.environ.pop(k, None)
            os.environ.update(env)
            rows = []
            for seed in (2, 3, 4, 0):
                p = _abi.make_params(seed=seed, batch=131072, batch_min=131072, n_waypoints=150, timeout_s=60.0,
                                     straight_first=False, tree_capacity=1 << 23, max_iters=8)
                path, st = ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
                s, pr = ctx.stats(), ctx.profile()
                rows.append((s["total_ms"], pr["nn_ms"], pr["nn_launches"], pr["nn_pairs"], pr["edge_ms"],
                             pr["edge_launches"], s["iterations"], s["samples"], float(path.sum()), pr["edge_states"]))
            if rep == 0:
                continue
            r = np.array(rows)
            print(f"{name:14s} total med {np.median(r[:, 0]):8.2f} ms (sum {r[:, 0].sum():8.2f}) | NN {r[:, 1].sum():8.2f} ms "
                  f"{int(r[:, 2].sum())} launches {r[:, 3].sum():.3g} pairs -> {r[:, 3].sum() / (r[:, 1].sum() * 1e-3):.3g} pairs/s"
                  f" | edges {r[:, 4].sum():7.2f} ms {int(r[:, 5].sum())} launches "
                  f"{r[:, 9].sum() / (r[:, 4].sum() * 1e-3) / 1e9:.2f} G states/s | iters {r[:, 6].astype(int).tolist()} "
                  f"samples {int(r[:, 7].sum())} pathsum {r[:, 8].sum():.9g}", flush=True)


if __name__ == "__main__":
    main()
