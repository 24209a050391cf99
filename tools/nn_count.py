"""Exact-path statistics of the matrix-core nearest-node search (diagnostic build
-DRP_NN_COUNT, abvariants/lib_nncount.so) on C5 covered-well plans:
python tools/nn_count.py abvariants/lib_nncount.so [RB ...]"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rbe550_final_project_amd import _abi, model, native, scenes  # noqa: E402

native.LIB_PATH = os.path.abspath(sys.argv[1])
from rbe550_final_project_amd.native import Context  # noqa: E402

L = native.load()
L.rp_debug_nncount.argtypes = [C.c_void_p]
q = json.load(open(os.path.join(ROOT, "tests/golden/workloads/clutter64_well.json")))["queries"][0]
sc = scenes.Scene.from_json(q["scene"])
ctx = Context(0)
ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
ctx.set_attached(q["attached"])
os.environ["RBE_PLAN_CHUNK"] = "-1"
buf = (C.c_ulonglong * 4)()
for rb in (sys.argv[2:] or ["4", "8"]):
    os.environ["RBE_NN_MFMA"] = rb
    L.rp_debug_nncount(buf)
    for seed in (2, 4):
        p = _abi.make_params(seed=seed, batch=131072, batch_min=131072, n_waypoints=150, timeout_s=60.0,
                             straight_first=False, tree_capacity=1 << 23, max_iters=8)
        ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
        L.rp_debug_nncount(buf)
        t, e, r, el = list(buf)
        print(f"RB {rb} seed {seed}: wave-tiles {t} exact-path tiles {e} ({e / max(t, 1):.3f}) rounds {r} "
              f"({r / max(e, 1):.2f} per exact tile) passing elements {el} ({el / max(t, 1):.3f} per tile)", flush=True)
