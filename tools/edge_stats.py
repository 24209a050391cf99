"""How much of the edge launches' work an early exit could skip (diagnostic): the C5
covered-well plans (131,072-sample iterations, seeds 2, 3, 4, 0) with RBE_EDGE_STATS
set, so the library sums after every wave-compacted edge launch (k_edge_stats) the
slots of all edges, of the edges that failed, and of the edges past their connect
chain's first failure (rp_debug_edges).

    python tools/edge_stats.py"""
import ctypes as C
import json
import os
import sys

os.environ["RBE_EDGE_STATS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rbe550_final_project_amd import _abi, model, native, scenes  # noqa: E402

q = json.load(open(os.path.join(ROOT, "tests/golden/workloads/clutter64_well.json")))["queries"][0]
sc = scenes.Scene.from_json(q["scene"])
ctx = native.Context(0)
ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
ctx.set_attached(q["attached"])


def stats():
    out = (C.c_double * 5)()
    native.load().rp_debug_edges(ctx._h, out, 5)
    return list(out)


stats()
tot = [0.0] * 5
for seed in (2, 3, 4, 0):
    p = _abi.make_params(seed=seed, batch=131072, batch_min=131072, n_waypoints=150, timeout_s=60.0,
                         straight_first=False, tree_capacity=1 << 23, max_iters=8)
    ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
    s = ctx.stats()
    v = stats()
    tot = [a + b for a, b in zip(tot, v)]
    print(f"seed {seed}: states_checked {s['states_checked']} | slots {v[0]:.0f}, of failed edges {v[1]:.0f} "
          f"({v[1] / max(v[0], 1):.3f}), past a chain's first failure {v[4]:.0f} ({v[4] / max(v[0], 1):.3f}) | "
          f"edges {v[2]:.0f}, failed {v[3]:.0f} ({v[3] / max(v[2], 1):.3f})", flush=True)
print(f"all: slots {tot[0]:.0f}, of failed edges {tot[1] / tot[0]:.3f}, past a chain's first failure "
      f"{tot[4] / tot[0]:.3f}, failed edges {tot[3] / max(tot[2], 1):.3f}")
