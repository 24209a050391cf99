"""Mid-size validity launches for counter collection (diagnostic): 65,536 uniform
states on bench.py's C2 5-box scene, 30 launches through rp_check_states_device —
the three-role k_validity_split (rp_kernels.h). Run under
rocprofv3 --pmc (tools/gpu_job.sh splitpmc).

    python tools/split_profile.py [states]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from rbe550_final_project_amd import model, scenes  # noqa: E402
from rbe550_final_project_amd.native import Context  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    dev = torch.device("cuda", 0)
    ctx = Context(0)
    sc = scenes.Scene(boxes=scenes.goal1_scattered(0).boxes[:5])
    ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
    rng = np.random.default_rng(0)
    q = torch.tensor((model.Q_LO + (model.Q_HI - model.Q_LO) * rng.random((n, 9))).astype(np.float32), device=dev)
    fl = torch.empty(n, dtype=torch.uint8, device=dev)
    for _ in range(30):
        ctx.check_states_device(q.data_ptr(), n, fl.data_ptr(), None)
    torch.cuda.synchronize()
    print(f"{n} states x 30 launches, valid fraction {fl.float().mean().item():.4f}")
    ctx.close()


if __name__ == "__main__":
    main()
