"""Broad-phase statistics of k_validity's self-pair and capsule-box stages on uniform
states (CPU oracle FK): per self pair, the fraction of states whose bounding-sphere
test passes, whose AABB test passes and whose narrow phase hits, and the fraction
of 64-state waves where ANY state passes (the SIMT cost driver). Diagnostic only.
    python tools/pair_stats.py [--states 16384]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle  # noqa: E402
from rbe550_final_project_amd import model, scenes  # noqa: E402

PAIRS = [(0, 6), (0, 7), (0, 8), (0, 9), (0, 10), (0, 11), (1, 5), (1, 6), (1, 7), (1, 8), (1, 9), (1, 10), (1, 11),
         (2, 5), (2, 6), (2, 7), (2, 8), (2, 9), (2, 10), (2, 11), (3, 7), (3, 8), (3, 9), (3, 10), (3, 11),
         (4, 8), (4, 9), (4, 10), (4, 11), (5, 9), (5, 10), (5, 11), (6, 9), (6, 10), (6, 11)]
NEVER = {(2, 5), (3, 7), (3, 8), (4, 8), (4, 9), (4, 10), (4, 11), (6, 9), (6, 10), (6, 11)}


def seg_seg_d2(a1, b1, a2, b2):
    return oracle.seg_seg_d2(a1, b1, a2, b2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--states", type=int, default=8192)
    a = ap.parse_args()
    spec = json.load(open(os.path.join(ROOT, "spec/franka_capsules.json")))
    rad = np.array([c["radius"] for c in spec["capsules"]], dtype=np.float64)
    geo = [np.array(c["a"] + c["b"], dtype=np.float64) for c in spec["capsules"]]
    half = np.array([0.5 * np.linalg.norm(g[3:] - g[:3]) for g in geo])
    srad = rad + half + 1e-4
    o = oracle.OracleScene()
    sc = scenes.goal3_tallest()
    o.set_scene(sc.boxes, base=sc.base)
    rng = np.random.default_rng(5)
    lo, hi = np.array(model.Q_LO, np.float32), np.array(model.Q_HI, np.float32)
    q = (lo + (hi - lo) * rng.random((a.states, 9), dtype=np.float32)).astype(np.float32)
    caps = np.stack([o.fk_capsules(x) for x in q])          # (n, 12, 2, 3)
    A, B = caps[:, :, 0].astype(np.float64), caps[:, :, 1].astype(np.float64)
    cen = 0.5 * (A + B)
    alo = np.minimum(A, B) - rad[None, :, None]
    ahi = np.maximum(A, B) + rad[None, :, None]
    nw = a.states // 64
    print(f"{'pair':10s} {'sphere':>7s} {'aabb':>7s} {'hit':>7s} | {'wave sph':>8s} {'wave aabb':>9s}")
    tot = np.zeros(3)
    for (i, j) in PAIRS:
        if (i, j) in NEVER:
            continue
        sph = np.linalg.norm(cen[:, i] - cen[:, j], axis=1) <= srad[i] + srad[j]
        ab = sph & ~np.any((alo[:, i] > ahi[:, j]) | (alo[:, j] > ahi[:, i]), axis=1)
        hit = np.zeros(a.states, bool)
        for s in np.nonzero(ab)[0]:
            hit[s] = seg_seg_d2(caps[s, i, 0], caps[s, i, 1], caps[s, j, 0], caps[s, j, 1]) <= (rad[i] + rad[j]) ** 2
        ws = sph[:nw * 64].reshape(nw, 64).any(1).mean()
        wa = ab[:nw * 64].reshape(nw, 64).any(1).mean()
        tot += [sph.mean(), ab.mean(), hit.mean()]
        print(f"{i:2d}-{j:2d}      {sph.mean():7.4f} {ab.mean():7.4f} {hit.mean():7.4f} | {ws:8.3f} {wa:9.3f}")
    print(f"per state: sphere passes {tot[0]:.3f}, aabb passes {tot[1]:.3f}, hits {tot[2]:.3f}")
    # capsule vs boxes (goal3)
    boxes = sc.boxes
    bext = []
    for (c, h, y) in boxes:
        cs, sn = abs(np.cos(y)), abs(np.sin(y))
        bext.append([cs * h[0] + sn * h[1], sn * h[0] + cs * h[1], h[2]])
    bc = np.array([b[0] for b in boxes])
    blo, bhi = bc - np.array(bext), bc + np.array(bext)
    print("boxes:", len(boxes))
    cnt = 0.0
    for c in range(12):
        ov = ~((alo[:, c, None, :] > bhi[None]) | (ahi[:, c, None, :] < blo[None])).any(2)
        cnt += ov.sum(1).mean()
        print(f"capsule {c:2d}: box AABB candidates per state {ov.sum(1).mean():.3f}, waves with any {ov[:nw * 64].reshape(nw, 64, -1).any(1).any(1).mean():.3f}")
    print(f"box candidates per state {cnt:.3f}")


if __name__ == "__main__":
    main()
