"""A/B timing of librbe_mi355x.so build variants, interleaved in one process
(cdna_hip_programming.md §5.4 rule 24). Each variant must give the same flags as
the first. Usage: python tools/variant_bench.py lib1.so lib2.so ... [--states N]"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rbe550_final_project_amd import _abi, model, scenes  # noqa: E402


def bind(path):
    L = C.CDLL(os.path.abspath(path))
    L.rp_create.argtypes = [C.POINTER(C.c_void_p), C.c_int, C.c_void_p]
    L.rp_set_scene.argtypes = [C.c_void_p, C.POINTER(_abi.Box), C.c_int32, C.c_float, C.POINTER(C.c_float)]
    L.rp_check_states_device.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]
    L.rp_destroy.argtypes = [C.c_void_p]
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--states", type=int, default=1 << 22)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--scene", default="goal3")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    sc = {"goal3": scenes.goal3_tallest(), "empty": scenes.Scene(),
          "goal1_5box": scenes.Scene(boxes=scenes.goal1_scattered(0).boxes[:5]),
          "clutter64": scenes.Scene.from_json(json.load(open(os.path.join(
              ROOT, "tests/golden/workloads/clutter64.json")))["queries"][0]["scene"])}[a.scene]
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    lo = torch.tensor(model.Q_LO, dtype=torch.float32, device=dev)
    hi = torch.tensor(model.Q_HI, dtype=torch.float32, device=dev)
    q = (lo + (hi - lo) * torch.rand((a.states, 9), generator=g, device=dev)).contiguous()
    stream = torch.cuda.Stream(dev)
    ctxs, flags = [], []
    arr, nb = _abi.make_boxes(sc.boxes)
    # "lib.so@ENV=V": that variant runs with ENV=V set (the library reads it per launch)
    envs = {p: dict(kv.split("=", 1) for kv in p.split("@")[1:]) for p in a.libs}
    for p in a.libs:
        L = bind(p.split("@")[0])
        h = C.c_void_p()
        assert L.rp_create(C.byref(h), 0, None) == 0, p
        assert L.rp_set_scene(h, arr, nb, 0.0, (C.c_float * 3)(*sc.base)) == 0
        f = torch.empty(a.states, dtype=torch.uint8, device=dev)
        ctxs.append((L, h))
        flags.append(f)
    torch.cuda.synchronize()
    times = {p: [] for p in a.libs}
    for r in range(a.rounds):
        for (L, h), f, p in zip(ctxs, flags, a.libs):
            for k in set().union(*envs.values()):
                os.environ.pop(k, None)
            os.environ.update(envs[p])
            for _ in range(2):
                L.rp_check_states_device(h, q.data_ptr(), a.states, f.data_ptr(), stream.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.iters):
                L.rp_check_states_device(h, q.data_ptr(), a.states, f.data_ptr(), stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize()
            times[p].append(e0.elapsed_time(e1) / a.iters)
    ref = flags[0].cpu()
    for p, f in zip(a.libs, flags):
        same = bool(torch.equal(f.cpu(), ref))
        t = np.array(times[p])
        print(f"{os.path.basename(p):40s} median {np.median(t):.4f} ms  min {t.min():.4f}  "
              f"{a.states / np.median(t) / 1e6:.2f} Gstates/s  flags_equal={same}")


if __name__ == "__main__":
    main()
