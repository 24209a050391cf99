import os, sys, json, numpy as np, torch
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from rbe550_final_project_amd import model, scenes
from rbe550_final_project_amd.native import Context
from oracle import oracle as O
import test_gpu_edges as T
sc = T._scene("clutter64")
o = O.OracleScene(); o.set_scene(sc.boxes, sc.plane_z, sc.base); o.set_attached(-1)
ctx = Context(0); ctx.set_scene(sc.boxes, sc.plane_z, sc.base); ctx.set_attached(-1)
n, scale = 20000, 10.0
qa, qb, res = T._edges(n, 7 + n, scale)
e = 494
d = float(np.sqrt(np.sum((qa[e] - qb[e]) ** 2))); nd = int(np.ceil(d / res))
s = qa[e] + (qb[e] - qa[e]) * (3 / nd)
s32 = s.astype(np.float32)
print("state f32", s32.tolist())
print("state f32 hex", [v.view(np.uint32).item() for v in s32])
print("oracle valid", o.check_states(s32[None])[0], "gpu valid", ctx.check_states(s32[None])[0])
s64 = s32.astype(np.float64)
print("gpu contacts", ctx.contacts(s64))
print("oracle contacts", o.contacts(s64))
caps = o.fk_capsules(s32)
print("oracle capsules", caps.tolist())
json.dump({"state": s32.tolist(), "scene": "clutter64"}, open("gpurun_out/edge_diff_state.json", "w"))
