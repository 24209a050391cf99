"""Debug: plan sequences on one context (which sequence hangs?). Each plan is
bounded by the context's own timeout; faulthandler dumps the stack on a hang."""
import faulthandler
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from rbe550_final_project_amd import _abi, model, scenes  # noqa: E402
from rbe550_final_project_amd.native import Context  # noqa: E402

faulthandler.dump_traceback_later(40, exit=True)
if os.environ.get("DBG_TORCH"):
    import torch  # noqa: F401  (torch's bundled HIP runtime / RCCL get loaded first)
W = {n: json.load(open(os.path.join(ROOT, "tests/golden/workloads", n + ".json")))["queries"]
     for n in ("goal3_tallest_10box", "goal4_pentagon_10box")}


def plan(ctx, wl, qi, seed, batch, bmin=0):
    q = W[wl][qi]
    sc = scenes.Scene.from_json(q["scene"])
    ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
    ctx.set_attached(q["attached"])
    p = _abi.make_params(seed=seed, batch=batch, batch_min=bmin, n_waypoints=150, timeout_s=20.0,
                         straight_first=False, tree_capacity=1 << 23)
    t = time.time()
    path, st = ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
    s = ctx.stats()
    print(f"  {wl}[{qi}] batch {batch}: status {st} it {s['iterations']} trees {s['start_tree_size']} "
          f"{s['goal_tree_size']} {1e3 * (time.time() - t):.1f} ms", flush=True)


which = sys.argv[1]
if which == "small_then_large":
    c = Context(0)
    plan(c, "goal3_tallest_10box", 5, 13, 256)
    plan(c, "goal4_pentagon_10box", 0, 0, 262144, 262144)
elif which == "group_then_single":
    class TG:
        def __init__(self):
            self.stage = [None, None]
            self.bar = threading.Barrier(2, timeout=30)

        def fn(self, r):
            def ag(send, recv):
                self.stage[r] = send.copy()
                self.bar.wait()
                recv[:] = np.concatenate(self.stage)
                self.bar.wait()
            return ag
    g = TG()
    cs = [Context(0), Context(0)]
    for r in range(2):
        cs[r].group_init(r, 2, g.fn(r))
    for (wl, qi, seed, b, bm) in (("goal3_tallest_10box", 5, 13, 256, 0), ("goal4_pentagon_10box", 0, 0, 262144, 262144)):
        th = [threading.Thread(target=plan, args=(cs[r], wl, qi, seed, b, bm)) for r in range(2)]
        [t.start() for t in th]
        [t.join() for t in th]
    cs[0].group_leave()
    plan(cs[0], "goal3_tallest_10box", 5, 13, 256)
    plan(cs[0], "goal4_pentagon_10box", 0, 0, 262144, 262144)
print("done", which, flush=True)
