"""Small validity launches: where the time per launch goes.

For each batch size (C2's 5-box scene) and lane count (RBE_ML_LANES), three
numbers per launch: back-to-back calls from Python (HIP events on the launch
stream: includes any host submission gap), the same launches replayed from a
captured hipGraph (dispatch only), and, under rocprofv3 --kernel-trace, the
kernel's own duration (read from the trace afterwards).
python tools/small_launch.py [lanes ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rbe550_final_project_amd import model, scenes  # noqa: E402
from rbe550_final_project_amd.native import Context  # noqa: E402

REPS = 50


def main():
    dev = torch.device("cuda", 0)
    ctx = Context(0)
    sc = scenes.Scene(boxes=scenes.goal1_scattered(0).boxes[:5])   # bench.py's C2 scene
    ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
    rng = np.random.default_rng(0)
    qs = (model.Q_LO + (model.Q_HI - model.Q_LO) * rng.random((1 << 18, 9))).astype(np.float32)
    qd = torch.tensor(qs, device=dev)
    fl = torch.empty(qs.shape[0], dtype=torch.uint8, device=dev)
    st = torch.cuda.Stream(dev)
    sizes = (64, 4096, 16384, 65536, 262144)
    for lanes in (sys.argv[1:] or ["", "1", "8", "16"]):
        os.environ["RBE_ML_LANES"] = lanes
        line = f"lanes={lanes or 'auto':>4}"
        for n in sizes:
            def call(s):
                ctx.check_states_device(qd.data_ptr(), n, fl.data_ptr(), s)
            for _ in range(3):
                call(st.cuda_stream)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(REPS):
                call(st.cuda_stream)
            e1.record(st)
            torch.cuda.synchronize()
            us_py = 1e3 * e0.elapsed_time(e1) / REPS
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                for _ in range(REPS):
                    call(st.cuda_stream)
            g.replay()
            torch.cuda.synchronize()
            e0.record(st)
            with torch.cuda.stream(st):
                g.replay()
            e1.record(st)
            torch.cuda.synchronize()
            us_g = 1e3 * e0.elapsed_time(e1) / REPS
            line += f" | {n}: py {us_py:6.1f} us ({n / us_py / 1e3:5.2f} G/s) graph {us_g:6.1f} us ({n / us_g / 1e3:5.2f} G/s)"
        print(line, flush=True)


if __name__ == "__main__":
    main()
