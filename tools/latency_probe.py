"""Validity-kernel latency vs launch size (run under rocprofv3 --kernel-trace):
small launches are what a plan iteration issues, so their per-wave latency (not
the bulk throughput) bounds plan wall time. Prints host-side timings; the kernel
durations come from the trace (tools/latency_probe.py --summarize <csv>)."""
import csv
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SIZES = [64, 64 * 8, 64 * 89, 64 * 256, 64 * 1024, 64 * 4096, 64 * 16384]


def run():
    import torch
    from rbe550_final_project_amd import model, scenes
    from rbe550_final_project_amd.native import Context
    ctx = Context(0, model.robot_desc())
    sc = scenes.goal3_tallest()
    ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
    rng = np.random.default_rng(0)
    near = np.clip(model.SAFE_HOME[None, :] + rng.normal(0, 0.2, (max(SIZES), 9)), model.Q_LO, model.Q_HI)
    uni = model.Q_LO + (model.Q_HI - model.Q_LO) * rng.random((max(SIZES), 9))
    flags = torch.empty(max(SIZES), dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    # edges like a plan's extension step: 256 edges of length `range` from near home
    res = 0.01 * model.max_extent()
    qa = near[:256].astype(np.float64)
    d = rng.normal(0, 1, qa.shape)
    qb = np.clip(qa + 0.2 * model.max_extent() * d / np.linalg.norm(d, axis=1, keepdims=True), model.Q_LO, model.Q_HI)
    for _ in range(30):
        ok = ctx.check_edges(qa, qb, res)
    print(f"edges 256 x range: valid {ok.mean():.3f}", flush=True)
    for name, arr in (("near", near), ("uniform", uni)):
        q = torch.from_numpy(arr.astype(np.float32)).cuda()
        print(name, flush=True)
        run_sizes(ctx, q, flags, s, torch)


def run_sizes(ctx, q, flags, s, torch):
    for n in SIZES:
        for _ in range(30):
            ctx.check_states_device(q.data_ptr(), n, flags.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(30):
            ctx.check_states_device(q.data_ptr(), n, flags.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 30 * 1e6
        print(f"n={n:8d} host-side {dt:8.1f} us/launch  valid {flags[:n].float().mean().item():.3f}", flush=True)


def summarize(path):
    """median duration of each run of consecutive launches of one kernel / grid"""
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    runs = []
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:32]
        if "rp::" not in name:
            continue
        key = (name, int(r["Grid_Size_X"]))
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if runs and runs[-1][0] == key:
            runs[-1][1].append(dur)
        else:
            runs.append((key, [dur]))
    for (name, g), d in runs:
        if len(d) >= 5:
            d = np.array(d)
            print(f"{name:34s} grid {g:8d}  n {len(d):3d}  median {np.median(d):8.2f} us  min {d.min():8.2f}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summarize":
        summarize(sys.argv[2])
    else:
        run()
