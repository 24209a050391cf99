"""Per-launch k_validity times over a long back-to-back run (bench.py's workload).

Shows how the kernel time moves from the first launch of a fresh process to the
steady state (clock / power ramp), to size bench.py's settle phase. One HIP event
pair per launch on the context's stream.

    python tools/clock_probe.py [--seconds 3] [--states 16777216] [--idle 0]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rbe550_final_project_amd import model, scenes  # noqa: E402
from rbe550_final_project_amd.native import Context  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--states", type=int, default=1 << 24)
    ap.add_argument("--idle", type=float, default=0.0, help="host sleep before the run (s)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    scene = scenes.goal3_tallest()
    ctx = Context(device=0, robot=model.robot_desc())
    ctx.set_scene(scene.boxes, scene.plane_z, scene.base)
    n = args.states
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    lo = torch.tensor(model.Q_LO, dtype=torch.float32, device=dev)
    hi = torch.tensor(model.Q_HI, dtype=torch.float32, device=dev)
    q = (lo + (hi - lo) * torch.rand((n, 9), generator=g, device=dev, dtype=torch.float32)).contiguous()
    flags = torch.empty(n, dtype=torch.uint8, device=dev)
    stream = torch.cuda.ExternalStream(ctx.stream_handle(), device=dev)
    torch.cuda.synchronize(dev)
    if args.idle > 0:
        time.sleep(args.idle)
    evs = []
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < args.seconds:
        batch = []
        for _ in range(20):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            ctx.check_states_device(q.data_ptr(), n, flags.data_ptr(), None)
            b.record(stream)
            batch.append((a, b))
        evs.extend(batch)
        batch[-1][1].synchronize()
    torch.cuda.synchronize(dev)
    us = [1e3 * a.elapsed_time(b) for a, b in evs]
    out = {"launches": len(us), "first_40_us": [round(x, 1) for x in us[:40]]}
    win = []
    for s in range(0, len(us), 100):
        w = us[s:s + 100]
        win.append(round(sum(w) / len(w), 1))
    out["avg_per_100_us"] = win
    tail = sorted(us[len(us) // 2:])
    out["second_half_median_us"] = round(tail[len(tail) // 2], 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
