"""Nearest-node kernel micro-benchmark (rp_selftest_nn): n uniform queries against a
tree of T nodes (uniform, or clustered along random-walk branches like an RRT tree),
timed per call; run under rocprofv3 for the k_nn_mfma kernel time and counters.

    python tools/nn_bench.py [LIB.so] [--n 131072] [--T 300000] [--mode 8] [--reps 5] [--tree walk|uniform]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rbe550_final_project_amd import model, native  # noqa: E402


def walk_tree(rng, T, step=0.2):
    """RRT-like node cloud: branches of short steps from random earlier nodes."""
    lo, hi = model.Q_LO, model.Q_HI
    pts = np.empty((T, 9))
    pts[0] = lo + (hi - lo) * rng.random(9)
    for i in range(1, T, 4096):
        m = min(4096, T - i)
        par = rng.integers(0, i, m)
        d = rng.standard_normal((m, 9))
        d *= (step * (hi - lo).max() / 6.0) / np.linalg.norm(d, axis=1, keepdims=True)
        pts[i:i + m] = np.clip(pts[par] + d, lo, hi)
    return pts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?")
    ap.add_argument("--n", type=int, default=131072)
    ap.add_argument("--T", type=int, default=300000)
    ap.add_argument("--mode", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--tree", default="walk")
    ap.add_argument("--check", action="store_true", help="compare with mode 0 (k_nn_part)")
    a = ap.parse_args()
    if a.lib:
        native.LIB_PATH = os.path.abspath(a.lib)
    rng = np.random.default_rng(7)
    lo, hi = model.Q_LO, model.Q_HI
    q = lo + (hi - lo) * rng.random((a.n, 9))
    tree = walk_tree(rng, a.T) if a.tree == "walk" else lo + (hi - lo) * rng.random((a.T, 9))
    ctx = native.Context(0, model.robot_desc())
    out = ctx.selftest_nn(q, tree, lo, hi, a.mode)
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        out = ctx.selftest_nn(q, tree, lo, hi, a.mode)
        ts.append(time.perf_counter() - t0)
    msg = (f"{os.path.basename(native.LIB_PATH)} mode {a.mode} tree {a.tree} n {a.n} T {a.T}: "
           f"call median {1e3 * np.median(ts):.2f} ms (incl. copies)")
    if a.check:
        ref = ctx.selftest_nn(q, tree, lo, hi, 0)
        msg += f"; equal to k_nn_part: {bool(np.array_equal(out, ref))}"
    print(msg, flush=True)


if __name__ == "__main__":
    main()
