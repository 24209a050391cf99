"""Edge-kernel diagnostic: rp_check_edges_device (the dense, wave-compacted k_edges
launch for >= 2,049 edges) against k_validity on the materialised interpolated
states; prints the edges whose verdicts differ with their group position, slot
count and first colliding slot.

    python tools/edge_diag.py [--n 8192] [--scene goal3|clutter64]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rbe550_final_project_amd import model, native, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--scene", default="goal3")
    ap.add_argument("--scale", type=float, default=1.0)
    a = ap.parse_args()
    if a.scene == "goal3":
        sc = scenes.goal3_tallest()
    else:
        sc = scenes.Scene.from_json(json.load(open(os.path.join(ROOT, "tests", "golden", "workloads",
                                                               a.scene + ".json")))["queries"][0]["scene"])
    rng = np.random.default_rng(7)
    lo, hi = model.Q_LO, model.Q_HI
    ext = model.max_extent()
    qa = lo + (hi - lo) * rng.random((a.n, 9))
    d = rng.standard_normal((a.n, 9))
    d *= (a.scale * 0.2 * ext * rng.random((a.n, 1))) / np.linalg.norm(d, axis=1, keepdims=True)
    qb = np.clip(qa + d, lo, hi)
    res = 0.01 * ext
    ctx = native.Context(0, model.robot_desc())
    ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
    dev = torch.device("cuda", 0)
    ta = torch.from_numpy(qa).to(dev)
    tb = torch.from_numpy(qb).to(dev)
    fe = torch.empty(a.n, dtype=torch.uint8, device=dev)
    L = native.load()
    ctx._check(L.rp_check_edges_device(ctx._h, ta.data_ptr(), tb.data_ptr(), a.n, float(res), fe.data_ptr(), None),
               "rp_check_edges_device")
    torch.cuda.synchronize()
    ok_e = fe.cpu().numpy().astype(bool)
    # reference verdicts: the interpolated states through rp_check_states (k_validity)
    nd = np.array([max(1, int(np.ceil(np.sqrt(((qb[i] - qa[i]) ** 2).sum()) / res))) for i in range(a.n)])
    states, owner, slots = [], [], []
    for i in range(a.n):
        for k in range(nd[i]):
            states.append(qb[i] if k == 0 else qa[i] + (qb[i] - qa[i]) * (k / nd[i]))
            owner.append(i)
            slots.append(k)
    st = np.asarray(states).astype(np.float32)
    fs = ctx.check_states(st).astype(bool)
    owner = np.asarray(owner)
    ref = np.ones(a.n, bool)
    np.logical_and.at(ref, owner, fs)
    bad = np.nonzero(ref != ok_e)[0]
    print(f"{a.scene} n {a.n}: {len(bad)} of {a.n} edge verdicts differ (gpu valid {ok_e.mean():.3f}, "
          f"ref valid {ref.mean():.3f}); slots max {nd.max()} mean {nd.mean():.1f}", flush=True)
    slots = np.asarray(slots)
    for i in bad[:25]:
        m = owner == i
        first = slots[m][~fs[m]]
        gsum = nd[(i // 64) * 64:i].sum()
        print(f"  edge {i} (group {i // 64} lane {i % 64}, items before it in the group {gsum}) nd {nd[i]} "
              f"gpu {ok_e[i]} ref {ref[i]} colliding slots {first.tolist()[:8]}", flush=True)


if __name__ == "__main__":
    main()
