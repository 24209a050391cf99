"""Validity launches of mid sizes on the BASELINE scenes: time per launch (HIP
events around 50 back-to-back launches on one stream) and a hash of the flags, for
one library / RBE_SPLIT_MAX setting per process (the split kernel's bound is read
once). Compare the printed flag hashes across runs: they must agree.

    [RBE_SPLIT_MAX=0] python tools/split_ab.py [LIB.so] [--tag NAME]
"""
import argparse
import hashlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rbe550_final_project_amd import model, native, scenes  # noqa: E402

SIZES = (8192, 16384, 32768, 65536, 131072, 262144)
REPS = 50


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?")
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    if a.lib:
        native.LIB_PATH = os.path.abspath(a.lib)
    dev = torch.device("cuda", 0)
    ctx = native.Context(0, model.robot_desc())
    wl = lambda n: json.load(open(os.path.join(ROOT, "tests", "golden", "workloads", n + ".json")))  # noqa: E731
    sc_list = {"C2_goal1_5box": scenes.Scene(boxes=scenes.goal1_scattered(0).boxes[:5]),
               "C3_goal3": scenes.goal3_tallest(),
               "C5_clutter64": scenes.Scene.from_json(wl("clutter64")["queries"][0]["scene"])}
    rng = np.random.default_rng(0)
    qs = (model.Q_LO + (model.Q_HI - model.Q_LO) * rng.random((max(SIZES), 9))).astype(np.float32)
    qd = torch.tensor(qs, device=dev)
    fl = torch.empty(qs.shape[0], dtype=torch.uint8, device=dev)
    st = torch.cuda.Stream(dev)
    tag = a.tag or os.path.basename(native.LIB_PATH) + " split_max=" + os.environ.get("RBE_SPLIT_MAX", "default")
    for name, sc in sc_list.items():
        ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
        ctx.set_attached(-1)
        parts = []
        h = hashlib.sha1()
        for n in SIZES:
            for _ in range(3):
                ctx.check_states_device(qd.data_ptr(), n, fl.data_ptr(), st.cuda_stream)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(REPS):
                ctx.check_states_device(qd.data_ptr(), n, fl.data_ptr(), st.cuda_stream)
            e1.record(st)
            torch.cuda.synchronize()
            us = 1e3 * e0.elapsed_time(e1) / REPS
            h.update(fl[:n].cpu().numpy().tobytes())
            parts.append(f"{n}:{us:.2f}us={n / us * 1e-3:.2f}G/s")
        print(f"{tag:34s} {name:14s} " + " ".join(parts) + f" flags {h.hexdigest()[:12]}", flush=True)


if __name__ == "__main__":
    main()
