"""A/B of the validity launch kinds at C2's size (BASELINE configs[1]: a 65,536-state
launch on the goal1 5-box scene): the three-role split kernel (the
product's choice for 4k-64k states) against the lane-group kernel k_validity_ml with
GL = 8 / 16 / 32 / 64 lanes per state (RBE_ML_LANES forces it), interleaved rounds,
HIP events on the context stream. Also 16,384 and 131,072 states.
python tools/c2_lanes_ab.py [out.json]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rbe550_final_project_amd import model, scenes  # noqa: E402
from rbe550_final_project_amd.native import Context  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    ctx = Context(0, model.robot_desc())
    sc = scenes.Scene(boxes=scenes.goal1_scattered(0).boxes[:5])
    ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
    stream = torch.cuda.ExternalStream(ctx.stream_handle(), device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    lo = torch.tensor(model.Q_LO, dtype=torch.float32, device=dev)
    hi = torch.tensor(model.Q_HI, dtype=torch.float32, device=dev)
    nmax = 131072
    q = (lo + (hi - lo) * torch.rand((nmax, 9), generator=g, device=dev)).contiguous()
    flags = torch.empty(nmax, dtype=torch.uint8, device=dev)
    ref = {}
    res = {}
    for rnd in range(3):
        for n in (16384, 65536, 131072):
            for gl in ("1", "8", "16", "32", "64"):
                os.environ["RBE_ML_LANES"] = gl
                for _ in range(5):
                    ctx.check_states_device(q.data_ptr(), n, flags.data_ptr(), None)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(100):
                    ctx.check_states_device(q.data_ptr(), n, flags.data_ptr(), None)
                e1.record(stream)
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / 100
                f = flags[:n].cpu().numpy()
                if n not in ref:
                    ref[n] = f
                assert np.array_equal(f, ref[n]), (n, gl)   # every launch kind: the same flags
                res.setdefault(f"{n}/{gl}", []).append(ms)
    os.environ.pop("RBE_ML_LANES", None)
    out = {}
    for k, v in res.items():
        n, gl = k.split("/")
        us = 1e3 * float(np.median(v))
        out[k] = {"states": int(n), "lanes_per_state": int(gl), "kernel": "k_validity_split<3 roles>" if gl == "1"
                  else f"k_validity_ml<{gl}>", "us_median": round(us, 3), "g_states_per_s": round(int(n) / us / 1e3, 3)}
        print(f"{int(n):7d} states, {gl:>2s} lanes/state: {us:8.2f} us  {int(n) / us / 1e3:6.2f} G states/s", flush=True)
    if len(sys.argv) > 1:
        json.dump(out, open(sys.argv[1], "w"), indent=1)
    ctx.close()


if __name__ == "__main__":
    main()
