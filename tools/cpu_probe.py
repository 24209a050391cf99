"""Host CPU of a long query, per thread (diagnostic): the sealed well (no path
exists; tests/test_gpu_async.py _sealed_well) planned for `--timeout` seconds
through rp_plan_async / rp_plan_wait, with each thread's utime + stime from
/proc/self/task before and after. Run once per wait setting (RBE_WAIT_SPIN_US,
RBE_WAIT_SLEEP_FRAC, RBE_PLAN_WAIT_SPIN_US are read once per process).

    python tools/cpu_probe.py [--timeout 2] [--batch 4096]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def threads():
    out = {}
    tck = os.sysconf("SC_CLK_TCK")
    for tid in os.listdir("/proc/self/task"):
        try:
            st = open(f"/proc/self/task/{tid}/stat").read()
            comm = st[st.index("(") + 1:st.rindex(")")]
            f = st[st.rindex(")") + 2:].split()
            out[tid] = (comm, (int(f[11]) + int(f[12])) / tck)
        except (OSError, ValueError):
            pass
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--timeout", type=float, default=2.0)
    ap.add_argument("--batch", type=int, default=4096)
    a = ap.parse_args()
    from rbe550_final_project_amd import _abi, model
    from rbe550_final_project_amd.native import Context
    import test_gpu_async as T
    q, sc = T._sealed_well()
    ctx = Context(device=0, robot=model.robot_desc())
    ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
    ctx.set_attached(q["attached"])
    ctx.reserve(a.batch, 1 << 23)
    p = _abi.make_params(seed=0, batch=a.batch, n_waypoints=150, timeout_s=a.timeout, straight_first=False,
                         tree_capacity=1 << 23)
    ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI,
             _abi.make_params(seed=1, batch=64, n_waypoints=150, timeout_s=0.05, straight_first=False))
    import ctypes as C
    from rbe550_final_project_amd import native

    def waits():
        out = (C.c_double * 5)()
        native.load().rp_debug_waits(ctx._h, out, 5)
        return list(out)

    wt0 = waits()
    th0, t0, w0 = threads(), os.times(), time.perf_counter()
    ctx.plan_async(q["start"], q["goal"], model.Q_LO, model.Q_HI, p, path_cap=256)
    path, st = ctx.plan_wait()
    th1, t1, wall = threads(), os.times(), time.perf_counter() - w0
    wt = [b - a for a, b in zip(wt0, waits())]
    s = ctx.stats()
    per = {}
    for tid, (comm, cpu) in th1.items():
        d = cpu - th0.get(tid, (comm, 0.0))[1]
        if d > 0.005:
            per[f"{comm}:{tid}" + (":main" if int(tid) == os.getpid() else "")] = round(d, 3)
    print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith("RBE_")}, "wall_s": round(wall, 3),
                      "cpu_s": round((t1.user - t0.user) + (t1.system - t0.system), 3), "per_thread_s": per,
                      "status": _abi.STATUS_NAMES[st], "iterations": s["iterations"], "samples": s["samples"],
                      "trees": [s["start_tree_size"], s["goal_tree_size"]],
                      "waits": {"wait_seq": int(wt[0]), "stream_wait": int(wt[1]), "spin_s": round(wt[2], 3),
                                "sleep_loop_s": round(wt[3], 3), "sleeps": int(wt[4])}}))
    ctx.close()


if __name__ == "__main__":
    main()
