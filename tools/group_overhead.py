"""Where a rank-group plan's time goes, in ONE process (no GPU sharing): C3
RRT-forced medians for the single-rank iteration, the group iteration at world 1
without a transport (RBE_PLAN_GROUPED=1), and with the shared-memory transport at
world 1 (gloo process group of one)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import torch.distributed as dist  # noqa: E402

from rbe550_final_project_amd import _abi, model, scenes  # noqa: E402
from rbe550_final_project_amd.distributed import Group  # noqa: E402
from rbe550_final_project_amd.native import Context  # noqa: E402

qs = json.load(open(os.path.join(ROOT, "tests/golden/workloads/goal3_tallest_10box.json")))["queries"]


def med(ctx, reps=3):
    out = []
    for r in range(reps):
        for i, q in enumerate(qs):
            sc = scenes.Scene.from_json(q["scene"])
            ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
            ctx.set_attached(q["attached"])
            p = _abi.make_params(seed=i, batch=4096, n_waypoints=150, timeout_s=10.0, straight_first=False)
            t0 = time.perf_counter()
            ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
            if r:
                out.append(1e3 * (time.perf_counter() - t0))
    return float(np.median(out))


os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29555")
dist.init_process_group("gloo", rank=0, world_size=1)
ctx = Context(0)
print(f"single-rank iteration      {med(ctx):.4f} ms", flush=True)
os.environ["RBE_PLAN_GROUPED"] = "1"
print(f"group iteration, world 1   {med(ctx):.4f} ms", flush=True)
del os.environ["RBE_PLAN_GROUPED"]
g = Group(ctx, transport="shm")
print(f"shm transport, world 1     {med(ctx):.4f} ms", flush=True)
g.leave()
g = Group(ctx, transport="host")
print(f"host transport, world 1    {med(ctx):.4f} ms", flush=True)
g.leave()
dist.destroy_process_group()
