"""Control for the one-GPU N=2 rehearsal: two processes on the SAME GPU planning
independently (single-rank, no group, barrier-aligned per query). Their C3
RRT-forced median vs one process alone is the cost of sharing the GPU, which the
group rehearsal pays on top of its exchange. Run under torch.distributed.run."""
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

dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
if os.environ.get("PROBE_TORCH_GPU"):   # initialise torch's GPU context as bench.py does
    torch.cuda.set_device(0)
    _t = torch.ones(1 << 20, device="cuda") * 2
    torch.cuda.synchronize()
qs = json.load(open(os.path.join(ROOT, "tests/golden/workloads/goal3_tallest_10box.json")))["queries"]
ctx = Context(0)
if os.environ.get("PROBE_VALIDITY"):   # bench.py's validity launches on a torch stream first
    torch.cuda.set_device(0)
    n = 1 << 22
    qd = torch.rand((n, 9), device="cuda")
    fl = torch.empty(n, dtype=torch.uint8, device="cuda")
    st = torch.cuda.Stream()
    sc0 = scenes.Scene.from_json(qs[0]["scene"])
    ctx.set_scene(sc0.boxes, sc0.plane_z, sc0.base)
    for _ in range(15):
        ctx.check_states_device(qd.data_ptr(), n, fl.data_ptr(),
                                None if os.environ.get("PROBE_CTX_STREAM") else st.cuda_stream)
    torch.cuda.synchronize()


def med(reps=3):
    out = []
    for r in range(reps):
        for i, q in enumerate(qs):
            sc = scenes.Scene.from_json(q["scene"])
            ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
            ctx.set_attached(q["attached"])
            p = _abi.make_params(seed=i, batch=4096, n_waypoints=150, timeout_s=10.0, straight_first=False)
            dist.barrier()
            t0 = time.perf_counter()
            ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
            if r:
                out.append(1e3 * (time.perf_counter() - t0))
    return float(np.median(out))


m_ind = med()
g = Group(ctx, transport="shm")
m_grp = med()
if os.environ.get("PROBE_BIG_FIRST"):   # a 65,536-sample C2 plan first, as bench.py runs them
    q = json.load(open(os.path.join(ROOT, "tests/golden/workloads/single_pick_place_5box.json")))["queries"][0]
    sc = scenes.Scene.from_json(q["scene"])
    ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
    ctx.set_attached(q["attached"])
    p = _abi.make_params(seed=0, batch=65536, batch_min=65536, n_waypoints=150, timeout_s=10.0, straight_first=False)
    dist.barrier()
    ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
    m_big = med()
    if rank == 0:
        print(f"after a 65,536-sample plan: rank group (shm) {m_big:.4f} ms", flush=True)
g.leave()
if rank == 0:
    print(f"world {world} on one GPU: independent single-rank plans {m_ind:.4f} ms, "
          f"rank group (shm) {m_grp:.4f} ms", flush=True)
dist.destroy_process_group()
