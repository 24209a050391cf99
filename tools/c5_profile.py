"""Kernel-class profile (rp_set_profiling) of C5 plans that grow large trees: the
covered-well query (tests/golden/workloads/clutter64_well.json) at 131,072-sample
iterations. Prints NN (query x node pairs, 27 FP64 FLOP each) and edge-launch
rates per plan."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rbe550_final_project_amd import _abi, model, scenes  # noqa: E402
from rbe550_final_project_amd.native import Context  # noqa: E402

q = json.load(open(os.path.join(ROOT, "tests/golden/workloads/clutter64_well.json")))["queries"][0]
sc = scenes.Scene.from_json(q["scene"])
ctx = Context(0)
ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
ctx.set_attached(q["attached"])
if "noprof" in sys.argv[1:]:
    ctx.reserve(131072, 1 << 23)   # as bench.py: no first-use hipMalloc inside the traced plans
grouped = "grouped" in sys.argv[1:]
if grouped:
    os.environ["RBE_PLAN_GROUPED"] = "1"
pmc = "pmc" in sys.argv[1:]   # counter passes: two plans, profiling off
noprof = "noprof" in sys.argv[1:]   # kernel traces: the four plans, profiling off
for prof in ((False,) if pmc or noprof else (False, True)):
    ctx.set_profiling(prof)
    for seed in ((2, 4) if pmc else (2, 3, 4, 0)):
        p = _abi.make_params(seed=seed, batch=131072, batch_min=131072, n_waypoints=150, timeout_s=60.0,
                             straight_first=False, tree_capacity=1 << 23, max_iters=8)
        path, st = ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
        s = ctx.stats()
        line = (f"prof={int(prof)} seed {seed}: status {st} it {s['iterations']} trees {s['start_tree_size']} "
                f"{s['goal_tree_size']} total {s['total_ms']:.2f} ms states {s['states_checked']}")
        if prof:
            pr = ctx.profile()
            nn_tf = pr["nn_pairs"] * 27 / (pr["nn_ms"] * 1e-3) / 1e12 if pr["nn_ms"] else 0
            ed = pr["edge_states"] / (pr["edge_ms"] * 1e-3) / 1e9 if pr["edge_ms"] else 0
            line += (f" | NN {pr['nn_launches']} launches {pr['nn_ms']:.2f} ms {pr['nn_pairs']:.3g} pairs "
                     f"{nn_tf:.2f} TF64 | edges {pr['edge_launches']} launches {pr['edge_ms']:.2f} ms {ed:.2f} G states/s")
        print(line, flush=True)
        if noprof:
            time.sleep(0.005)   # (plans apart in a kernel trace: tools/gap_summary.py)
