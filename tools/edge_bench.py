"""Edge-check kernel vs the validity kernel on the same states (diagnostic for the
edge launches' roofline): n random edges of about one RRT step (OMPL range =
0.2 maxExtent, ~20 slots at resolution 0.01 maxExtent) checked by
rp_check_edges_device, and the same interpolated states (materialised once) checked
by rp_check_states_device. Run under rocprofv3 --kernel-trace --stats for the
kernel times; prints wall-clock rates of both.

    python tools/edge_bench.py [LIB.so] [--n 262144] [--scene clutter64|goal3] [--reps 10] [--host]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rbe550_final_project_amd import model, native, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?")
    ap.add_argument("--n", type=int, default=262144)
    ap.add_argument("--scene", default="clutter64")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--host", action="store_true",
                    help="edges through rp_check_edges (host buffers; the loop-free k_edges with the read-back slot "
                         "bound; RBE_EDGE_KMAX_PAD adds waves per group past it)")
    a = ap.parse_args()
    if a.lib:
        native.LIB_PATH = os.path.abspath(a.lib)
    if a.scene == "goal3":
        sc = scenes.goal3_tallest()
    else:
        sc = scenes.Scene.from_json(json.load(open(os.path.join(ROOT, "tests", "golden", "workloads",
                                                               a.scene + ".json")))["queries"][0]["scene"])
    rng = np.random.default_rng(5)
    lo, hi = model.Q_LO, model.Q_HI
    ext = model.max_extent()
    qa = lo + (hi - lo) * rng.random((a.n, 9))
    d = rng.standard_normal((a.n, 9))
    d *= (0.2 * ext) / np.linalg.norm(d, axis=1, keepdims=True)
    qb = np.clip(qa + d, lo, hi)
    res = 0.01 * ext
    # the states the edge kernel checks (checkMotion mode 0: slots 1..nd-1 interpolated,
    # slot 0 = the far endpoint b), interpolated in f64 and rounded to f32
    nd = np.ceil(np.sqrt(((qb - qa) ** 2).sum(1)) / res).astype(np.int64)
    nd = np.maximum(nd, 1)
    tot = int(nd.sum())
    st = np.empty((tot, 9))
    o = 0
    for k in range(int(nd.max()) + 1):
        m = nd > k
        if not m.any():
            break
        cnt = int(m.sum())
        st[o:o + cnt] = np.where(k == 0, qb[m], qa[m] + (qb[m] - qa[m]) * (k / nd[m])[:, None])
        o += cnt
    st32 = st[:o].astype(np.float32)
    ctx = native.Context(0, model.robot_desc())
    ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
    dev = torch.device("cuda", 0)
    ta = torch.from_numpy(qa).to(dev)
    tb = torch.from_numpy(qb).to(dev)
    ts = torch.from_numpy(st32).to(dev)
    fe = torch.empty(a.n, dtype=torch.uint8, device=dev)
    fs = torch.empty(len(st32), dtype=torch.uint8, device=dev)
    L = native.load()
    h = ctx._h

    def edges():
        if a.host:
            fe.copy_(torch.from_numpy(ctx.check_edges(qa, qb, float(res)).astype(np.uint8)))
            return
        ctx._check(L.rp_check_edges_device(h, ta.data_ptr(), tb.data_ptr(), a.n, float(res), fe.data_ptr(), None),
                   "rp_check_edges_device")

    def states():
        ctx.check_states_device(ts.data_ptr(), len(st32), fs.data_ptr(), None)

    out = {}
    for name, f, count in (("edges", edges, o), ("states", states, len(st32))):
        f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            f()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.reps
        out[name] = count / dt
        print(f"{os.path.basename(native.LIB_PATH)} {a.scene} {name}: {count} states in {1e3 * dt:.3f} ms = "
              f"{count / dt / 1e9:.2f} G states/s", flush=True)
    # the same verdicts: an edge is valid iff all its states are
    ok_e = fe.cpu().numpy().astype(bool)
    ok_s = fs.cpu().numpy().astype(bool)
    edge_of = np.concatenate([np.nonzero(nd > k)[0] for k in range(int(nd.max()) + 1) if (nd > k).any()])
    agg = np.ones(a.n, bool)
    np.logical_and.at(agg, edge_of, ok_s)
    print(f"edge verdicts equal to the states' AND: {bool(np.array_equal(agg, ok_e))}; valid edges "
          f"{ok_e.mean():.3f}, valid states {ok_s.mean():.3f}; edges/states rate {out['edges'] / out['states']:.3f}",
          flush=True)


if __name__ == "__main__":
    main()
