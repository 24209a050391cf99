"""A/B of the two box broad phases (cluster AABBs vs axis grid, rp_model.h) on
several scenes, interleaved in one process: states/s of each and flag equality."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rbe550_final_project_amd import model, scenes  # noqa: E402
from rbe550_final_project_amd.native import Context  # noqa: E402


def wl_scene(name, i=0):
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "workloads", name + ".json")))
    return scenes.Scene.from_json(d["queries"][i]["scene"])


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 22
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    lo = torch.tensor(model.Q_LO, dtype=torch.float32, device=dev)
    hi = torch.tensor(model.Q_HI, dtype=torch.float32, device=dev)
    q = (lo + (hi - lo) * torch.rand((n, 9), generator=g, device=dev)).contiguous()
    stream = torch.cuda.Stream(dev)
    cases = {"goal1": scenes.goal1_scattered(0), "goal3": scenes.goal3_tallest(),
             "goal4": wl_scene("goal4_pentagon_10box", 14), "clutter64": wl_scene("clutter64")}
    for name, sc in cases.items():
        ctxs = []
        for mode in ("0", "1"):
            os.environ["RBE_SCENE_GRID"] = mode
            c = Context(0, model.robot_desc())
            c.set_scene(sc.boxes, sc.plane_z, sc.base)
            ctxs.append((mode, c, torch.empty(n, dtype=torch.uint8, device=dev)))
        os.environ.pop("RBE_SCENE_GRID")
        times = {m: [] for m, _, _ in ctxs}
        for _ in range(5):
            for mode, c, f in ctxs:
                c.check_states_device(q.data_ptr(), n, f.data_ptr(), stream.cuda_stream)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(10):
                    c.check_states_device(q.data_ptr(), n, f.data_ptr(), stream.cuda_stream)
                torch.cuda.synchronize()
                times[mode].append((time.perf_counter() - t0) / 10)
        same = bool(torch.equal(ctxs[0][2], ctxs[1][2]))
        rate = {m: n / np.median(t) / 1e9 for m, t in times.items()}
        print(f"{name:10s} boxes {len(sc.boxes):3d}  clusters {rate['0']:7.2f} G/s  grid {rate['1']:7.2f} G/s  "
              f"valid {ctxs[0][2].float().mean().item():.3f}  flags_equal {same}", flush=True)
        for _, c, _ in ctxs:
            c.close()


if __name__ == "__main__":
    main()
