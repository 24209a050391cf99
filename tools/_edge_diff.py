import os, sys, json, numpy as np, torch
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from rbe550_final_project_amd import model, scenes
from rbe550_final_project_amd.native import Context
from oracle import oracle as O
import test_gpu_edges as T
sc = T._scene("clutter64")
o = O.OracleScene(); o.set_scene(sc.boxes, sc.plane_z, sc.base); o.set_attached(-1)
ctx = Context(0); ctx.set_scene(sc.boxes, sc.plane_z, sc.base); ctx.set_attached(-1)
for vw, pk in [("1","0"),("4","0"),("1","8"),("4","8")]:
    os.environ["RBE_EDGE_VW"]=vw; os.environ["RBE_EDGE_COARSE"]=pk; os.environ["RBE_EDGE_COARSE_MIN"]="0"; os.environ["RBE_ML_LANES"]="1"
    for seed_off in (7, 11, 3):
        n, scale = 20000, 10.0
        qa, qb, res = T._edges(n, seed_off + n, scale)
        ref = o.check_edges(qa, qb, res)
        got = ctx.check_edges(qa, qb, res)
        dev = torch.device("cuda", 0)
        ta, tb = torch.from_numpy(qa).to(dev), torch.from_numpy(qb).to(dev)
        out = torch.empty(n, dtype=torch.uint8, device=dev)
        ctx.check_edges_device(ta.data_ptr(), tb.data_ptr(), n, res, out.data_ptr()); torch.cuda.synchronize()
        gd = out.cpu().numpy()
        bad = np.nonzero(got != ref)[0]; badd = np.nonzero(gd != ref)[0]
        print(vw, pk, seed_off, "host-path diffs", bad[:5].tolist(), "device-path diffs", badd[:5].tolist(), flush=True)
        for e in list(bad[:2]) + list(badd[:1]):
            d = float(np.sqrt(np.sum((qa[e] - qb[e]) ** 2)))
            nd = int(np.ceil(d / res))
            st = [qb[e]] + [qa[e] + (qb[e] - qa[e]) * (m / nd) for m in range(1, nd)]
            st32 = np.array(st).astype(np.float32)
            fo = o.check_states(st32); fg = ctx.check_states(st32)
            print("  edge", int(e), "ref", int(ref[e]), "host", int(got[e]), "dev", int(gd[e]), "nd", nd,
                  "oracle states invalid", np.nonzero(fo == 0)[0][:8].tolist(), "gpu states invalid", np.nonzero(fg == 0)[0][:8].tolist(),
                  "state flag diffs", np.nonzero(fo != fg)[0][:8].tolist(), flush=True)
