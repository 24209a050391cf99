"""Plan latency with each lane count of the low-latency kernels (RBE_ML_LANES):
C1 / C3 product default and RRT-forced medians, and k_validity(_ml) time at 64k
states, on one context."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (first: the process then uses torch's HIP runtime for both)

from rbe550_final_project_amd import _abi, model, scenes  # noqa: E402
from rbe550_final_project_amd.native import Context  # noqa: E402


def wl(name):
    return json.load(open(os.path.join(ROOT, "tests/golden/workloads", name + ".json")))["queries"]


def plans(ctx, qs, straight, reps=3):
    out = []
    for r in range(reps):
        for i, q in enumerate(qs):
            sc = scenes.Scene.from_json(q["scene"])
            ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
            ctx.set_attached(q["attached"])
            p = _abi.make_params(seed=i, batch=4096, n_waypoints=150, timeout_s=10.0, straight_first=straight)
            t0 = time.perf_counter()
            ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
            if r > 0:
                out.append(1e3 * (time.perf_counter() - t0))
    return np.median(out), np.sum(out) / (reps - 1)


ctx = Context(0)
g3, g1 = wl("goal3_tallest_10box"), wl("goal1_scattered_6box")
rng = np.random.default_rng(0)
qs = (model.Q_LO + (model.Q_HI - model.Q_LO) * rng.random((65536, 9))).astype(np.float32)
for lanes in (sys.argv[1:] or ["1", "8", "16", "32", "64", ""]) if os.environ.get("TUNE_PLANS", "1") == "1" else []:
    os.environ["RBE_ML_LANES"] = lanes
    plans(ctx, g3[:3], True, 2)   # warm
    m3, t3 = plans(ctx, g3, True)
    m3r, t3r = plans(ctx, g3, False)
    m1, t1 = plans(ctx, g1, True)
    m1r, t1r = plans(ctx, g1, False)
    sc = scenes.Scene.from_json(g3[0]["scene"])
    ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
    ctx.set_attached(-1)
    for n in (2, 64, 4096, 65536):
        ctx.check_states(qs[:n])
    ts = {}
    for n in (2, 64, 4096, 65536):
        t0 = time.perf_counter()
        for _ in range(20):
            ctx.check_states(qs[:n])
        ts[n] = 1e3 * (time.perf_counter() - t0) / 20
    print(f"lanes={lanes or 'auto':>4}: C3 {m3:.4f}/{t3:.3f} ms  C3rrt {m3r:.4f}/{t3r:.3f}  C1 {m1:.4f}/{t1:.3f}  "
          f"C1rrt {m1r:.4f}/{t1r:.3f}  | check_states ms: " + " ".join(f"{n}:{ts[n]:.4f}" for n in ts), flush=True)

# kernel time of the validity launch on device buffers (HIP events), per lane count
dev = torch.device("cuda", 0)
qd = torch.tensor(qs, device=dev)
fl = torch.empty(65536, dtype=torch.uint8, device=dev)
st = torch.cuda.Stream(dev)
for lanes in ["1", "8", "16", "32", "64"]:
    os.environ["RBE_ML_LANES"] = lanes
    line = f"lanes={lanes:>3} kernel us:"
    for n in (64, 1024, 4096, 16384, 65536):
        for _ in range(3):
            ctx.check_states_device(qd.data_ptr(), n, fl.data_ptr(), st.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(20):
            ctx.check_states_device(qd.data_ptr(), n, fl.data_ptr(), st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        us = 1e3 * e0.elapsed_time(e1) / 20
        line += f" {n}:{us:.1f} ({n / us / 1e3:.2f} G/s)"
    print(line, flush=True)
