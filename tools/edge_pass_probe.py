"""Coarse-first edge passes on a controlled set (diagnostic): n random edges of about
one RRT step (tests/test_gpu_edges.py's generator) in a scene, checked through
rp_check_edges with RBE_EDGE_COARSE = each given stride (0 = one pass), reps times
each, interleaved. Prints per stride the states checked (pass 0's count follows from
the slot counts; pass 1's is the rest) and the wall time per call; run it under
rocprofv3 --kernel-trace for the per-pass kernel times (tools/edge_pass_probe.py
--trace DIR splits them: k_edges before / after k_edge_rest).

    python tools/edge_pass_probe.py [--scene clutter64] [--n 262144] [--reps 5] [--strides 0,4,8]
    python tools/edge_pass_probe.py --trace gpurun_out/epp/kt_kernel_trace.csv"""
import argparse
import csv
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def trace(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    out = []   # (pass-0 us, rest us, pass-1 us) per coarse launch; one-pass launches alone
    i = 0
    while i < len(rows):
        n = rows[i]["Kernel_Name"]
        us = (int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])) / 1e3
        if "k_edges<" in n:
            if i + 2 < len(rows) and "k_edge_rest" in rows[i + 1]["Kernel_Name"]:
                r = rows[i + 1]
                p = rows[i + 2]
                out.append(("coarse", us, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
                            (int(p["End_Timestamp"]) - int(p["Start_Timestamp"])) / 1e3))
                i += 3
                continue
            out.append(("one", us, 0.0, 0.0))
        i += 1
    for kind, a, b, c in out:
        print(f"{kind:6s} pass0/one {a:8.1f} us  rest {b:6.1f} us  pass1 {c:8.1f} us")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="clutter64")
    ap.add_argument("--n", type=int, default=262144)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--strides", default="0,4,8")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--trace")
    a = ap.parse_args()
    if a.trace:
        trace(a.trace)
        return
    from rbe550_final_project_amd import model, scenes
    from rbe550_final_project_amd.native import Context
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_gpu_edges import _edges
    if a.scene == "goal3":
        sc = scenes.goal3_tallest()
    else:
        sc = scenes.Scene.from_json(json.load(open(os.path.join(ROOT, "tests", "golden", "workloads",
                                                               a.scene + ".json")))["queries"][0]["scene"])
    ctx = Context(0, model.robot_desc())
    ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
    ctx.set_attached(-1)
    os.environ["RBE_ML_LANES"] = "1"
    qa, qb, res = _edges(a.n, 3, a.scale)
    d = np.sqrt(((qb - qa) ** 2).sum(axis=1))
    cnt = np.maximum(np.ceil(d / res).astype(np.int64), 1)
    strides = [int(x) for x in a.strides.split(",")]
    ref = None
    for rep in range(a.reps + 1):
        for pk in strides:
            os.environ["RBE_EDGE_COARSE"] = str(pk)
            os.environ["RBE_EDGE_COARSE_MIN"] = "0"
            t0 = time.perf_counter()
            flags = ctx.check_edges(qa, qb, res)
            dt = time.perf_counter() - t0
            st = ctx.stats()["states_checked"]
            if ref is None:
                ref = flags
            assert np.array_equal(flags, ref)
            if rep == 0:
                continue
            p0 = int((1 + (cnt - 1) // pk).sum()) if pk > 1 else int(cnt.sum())
            print(f"stride {pk:2d}: states {st:9d} (pass 0 {p0:9d}, pass 1 {st - p0:9d}) of {int(cnt.sum())} "
                  f"slots; edges valid {float(flags.mean()):.3f}; call {dt * 1e3:7.3f} ms", flush=True)


if __name__ == "__main__":
    main()
