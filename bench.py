"""Benchmark of the MI355X planner hot path (BASELINE.json metric:
"states-checked/sec + plan wall-time, 7-DOF arm/10 blocks, 1/2/4/8 GPU").

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Step = one launch of the state-validity kernel (Franka FK + capsule vs plane / box /
self collision) over a batch of synthetic 9-D states resident in HBM, on the
goal3_tallest 10-box scene (code/scenes.py:150-223; BASELINE config C3). Per-GPU
batch is fixed (weak scaling); no collective is on this path. After the timed
steps every rank also runs the C3 plan workload (21 RRT-Connect queries replaying
goal3_tallest's pick/stack call sites) with the rank group sharding each iteration
(RCCL all-gather), and rank 0 times the CPU oracle beside it (N=1 only).
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from rbe550_final_project_amd import _abi, model, scenes  # noqa: E402
from rbe550_final_project_amd.native import Context  # noqa: E402

METRIC = "states-checked/sec + plan wall-time, 7-DOF arm/10 blocks, 1/2/4/8 GPU"
ROOF = json.load(open(os.path.join(ROOT, "bench", "roofline.json")))   # frozen constants
VALU_PEAK_TFLOPS = ROOF["peaks"]["fp32_vector_tflops"]
FP64_PEAK_TFLOPS = ROOF["peaks"]["fp64_vector_tflops"]
HBM_PEAK_GBPS = ROOF["peaks"]["hbm_gbps"]
BYTES_PER_STATE = ROOF["state_check"]["bytes"]     # 9 x fp32 in, 1 B flag out
BYTES_PER_EDGE = ROOF["edge_check"]["bytes"]
NN_FLOP_PER_PAIR = ROOF["nearest_node"]["flop"]
NN_MFMA_FLOP_PER_PAIR = ROOF["nearest_node"]["mfma_flop"]
F16_MFMA_PEAK_TFLOPS = ROOF["peaks"]["f16_mfma_dense_tflops"]
C2_BATCH = 65536             # BASELINE C2: 64k-sample batch
C4_BATCH = 262144            # BASELINE C4: 256k-sample iterations
C5_BATCH = 131072            # BASELINE C5: 131,072-sample iterations (2^20 budget)


def flops_per_state(n_boxes):
    """Algorithmic FP32 work of one full (collision-free) state check, from
    bench/roofline.json (counted from rp_math.h)."""
    f = ROOF["state_check"]["flop"]
    return f["fk"] + f["capsule_aabb_and_plane"] + f["box_broad_phase_per_box"] * n_boxes + f["self_broad_phase"]


def host_info():
    """The host the CPU baseline ran on: the threads it may use and the machine."""
    model_name = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model_name = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count()
    return {"nproc": os.cpu_count(), "affinity": affinity, "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "cpu_model": model_name}


def load_workload(name):
    with open(os.path.join(ROOT, "tests", "golden", "workloads", name + ".json")) as f:
        return json.load(f)


def pmc_traffic(n_states):
    """HBM bytes per validity launch from the committed rocprofv3 --pmc summary
    (profiles/), corrected per MI355X_MICROARCH.md §HBM; None if absent."""
    path = os.path.join(ROOT, "profiles", "pmc_validity.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        if int(d.get("states_per_launch", -1)) != int(n_states):
            return None
        from rbe550_final_project_amd.build import validity_source_hash
        if d.get("source_hash") != validity_source_hash():
            return None   # measured on another build of k_validity: stale
        return float(d["hbm_bytes_per_launch"])
    except Exception:
        return None


def run_plans(ctx, wl, batch, seed, group, batch_min=0, tree_capacity=0, stats_out=None, straight_first=True,
              max_iters=0):
    """Wall time of every query of a workload (ms), plus aggregate states checked.
    straight_first=False forces RRT-Connect on every query (the product default
    first checks the straight edge start -> goal)."""
    times, states, statuses = [], 0, []
    # the workspace for this batch / tree size, allocated before the timed queries
    # (rp_reserve; the product's PlannerInterface does the same when it opens a context)
    ctx.reserve(batch, tree_capacity)
    for i, q in enumerate(wl["queries"]):
        sc = scenes.Scene.from_json(q["scene"])
        ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
        ctx.set_attached(q["attached"])
        p = _abi.make_params(seed=seed + i, batch=batch, batch_min=batch_min, n_waypoints=150, timeout_s=10.0,
                             tree_capacity=tree_capacity, straight_first=straight_first, max_iters=max_iters)
        if group is not None:
            dist.barrier()
        t0 = time.perf_counter()
        path, st = ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
        times.append(1e3 * (time.perf_counter() - t0))
        s = ctx.stats()
        states += s["states_checked"]
        statuses.append(st)
        if stats_out is not None:
            for k in ("exchange_ms", "iterations", "samples"):
                stats_out[k] = stats_out.get(k, 0) + s[k]
    return times, states, statuses


def run_plan_path(ctx, wl, seed, straight_first=True):
    """End-to-end wall time of the reference's own call, per query (ms):
    `PlannerInterface.plan_path(qpos_goal=goal, num_waypoints=150,
    attached_object=held, timeout=10.0)` (code/motion_primitives.py:144), through the
    Genesis stand-in of the CPU tests (tests/mock_genesis.py: box entities with
    get_pos / get_quat torch tensors, a robot with get_qpos / set_qpos / q_limit).
    One PlannerInterface per workload, on the bench's context (one context per
    process, as motion_primitives.py:38 keeps one planner); before each query the
    blocks are moved to the query's poses and the robot to its start (the
    simulation's state when the caller plans). Timed: the whole plan_path call —
    scene ingestion, rp_plan, the 150 waypoint tensors, restoring qpos."""
    import contextlib
    import io
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import mock_genesis as M
    from rbe550_final_project_amd import planning
    q0 = scenes.Scene.from_json(wl["queries"][0]["scene"])
    sim = M.Scene(q0.boxes)
    pi = planning.PlannerInterface(sim.robot, sim)
    pi._ctx = ctx
    planning.configure(seed=seed, batch=4096, straight_first=straight_first)
    times, parts, statuses, states = [], {"scene_ms": [], "rp_plan_ms": [], "other_ms": []}, [], 0
    sink = io.StringIO()   # plan_path prints "Number of waypoints in path" (planning.py:200)
    try:
        for q in wl["queries"]:
            sc = scenes.Scene.from_json(q["scene"])
            for ent, (c, h, yaw) in zip(sim.entities[1:], sc.boxes):
                ent.set_pos(c)
                ent._quat = np.array([np.cos(yaw / 2), 0.0, 0.0, np.sin(yaw / 2)])
            sim.robot.q = torch.tensor(q["start"], dtype=torch.float32)
            held = sim.entities[1 + q["attached"]] if q["attached"] >= 0 else None
            goal = np.array(q["goal"], dtype=float)
            with contextlib.redirect_stdout(sink):
                t0 = time.perf_counter()
                wps = pi.plan_path(qpos_goal=goal, num_waypoints=150, attached_object=held, timeout=10.0)
                times.append(1e3 * (time.perf_counter() - t0))
            sink.seek(0)
            sink.truncate()
            statuses.append(pi.last_status)
            states += int(pi.last_stats["states_checked"])
            for k in parts:
                parts[k].append(pi.last_timing[k])
            assert len(wps) == 150, (q["label"], len(wps))
    finally:
        planning.configure(straight_first=True)
    return times, states, statuses, {k: round(float(np.median(v)), 4) for k, v in parts.items()}


def run_plan_path_devices(devices, seeds=(1, 2, 3, 4)):
    """The C5 covered-well queries (131,072-sample iterations) through
    PlannerInterface.plan_path with planning.configure(devices=devices): one process,
    one context per device, one rank group (rp_group_init_local: RCCL between distinct
    GPUs, the in-process shared segment when a device repeats). Per query wall time
    (ms) of the whole call; one untimed warm-up query first."""
    import contextlib
    import io
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import mock_genesis as M
    from rbe550_final_project_amd import planning
    q = load_workload("clutter64_well")["queries"][0]
    sc = scenes.Scene.from_json(q["scene"])
    sim = M.Scene(sc.boxes)
    times, statuses, states, info = [], [], 0, None
    sink = io.StringIO()
    try:
        planning.configure(seed=seeds[0], batch=C5_BATCH, batch_min=C5_BATCH, straight_first=False,
                           tree_capacity=1 << 23, devices=devices)
        pi = planning.PlannerInterface(sim.robot, sim)
        for k in range(len(seeds) + 1):
            if k == 1:
                planning.configure(seed=seeds[0])   # the timed queries: seeds[0], seeds[0] + 1, ...
            with contextlib.redirect_stdout(sink):
                t0 = time.perf_counter()
                wps = pi.plan_path(qpos_goal=np.array(q["goal"]), qpos_start=np.array(q["start"]),
                                   num_waypoints=150, timeout=10.0)
                dt = 1e3 * (time.perf_counter() - t0)
            sink.seek(0)
            sink.truncate()
            assert len(wps) == 150
            if k > 0:
                times.append(dt)
                statuses.append(pi.last_status)
                states += int(pi.last_stats["states_checked"])
        info = [c.group_info() for c in pi._ctxs]
        for c in pi._ctxs:
            c.close()
    finally:
        planning.configure(seed=0, batch=4096, batch_min=0, straight_first=True, tree_capacity=0, devices=())
    return times, states, statuses, info


def run_plans_pipelined(device, wl, batch, straight_first, serial_total_ms, ks=(2, 4, 8), reps=5):
    """C3 pipelined: the workload's queries in flight on K contexts of one GPU
    (rp_plan_many: each context its own stream and planner thread, the host side of a
    query in C++; a context waits only for its own previous query). Wall time of the
    whole workload (one rp_plan_many call), best
    K, median of `reps` passes after a warm-up pass; the same seeds as the serial legs
    (query i: seed i), so every path is the one the serial leg returns
    (tests/test_gpu_pipelined.py checks them against the oracle)."""
    from rbe550_final_project_amd import native
    jobs = [{"scene": scenes.Scene.from_json(q["scene"]), "attached": q["attached"], "start": q["start"],
             "goal": q["goal"], "lo": model.Q_LO, "hi": model.Q_HI,
             "params": _abi.make_params(seed=i, batch=batch, n_waypoints=150, timeout_s=10.0,
                                        straight_first=straight_first)} for i, q in enumerate(wl["queries"])]
    ctxs = [Context(device=device, robot=model.robot_desc()) for _ in range(max(ks))]
    per_k = {}
    try:
        for c in ctxs:
            c.reserve(batch, 0)
        qs, keep = native.make_queries(jobs)   # (the records, made once: the serial legs' scenes are set
        n = len(jobs)                           # outside their timed calls too)
        for k in ks:
            native.plan_many(ctxs[:k], qs, n, model.Q_LO, model.Q_HI)   # warm-up pass
            walls = []
            for _ in range(reps):
                t0 = time.perf_counter()
                res = native.plan_many(ctxs[:k], qs, n, model.Q_LO, model.Q_HI)
                walls.append(1e3 * (time.perf_counter() - t0))
            solved = sum(st in (_abi.STATUS_EXACT, _abi.STATUS_APPROXIMATE) for _, st, _ in res)
            per_k[k] = {"total_ms": round(float(np.median(walls)), 4), "min_ms": round(min(walls), 4),
                        "solved": int(solved)}
        del keep
    finally:
        for c in ctxs:
            c.close()
    best = min(per_k, key=lambda k: per_k[k]["total_ms"])
    rec = dict(per_k[best])
    rec.update({"queries": len(jobs), "batch": batch, "contexts": best, "per_contexts": per_k,
                "serial_total_ms": serial_total_ms,
                "speedup_vs_serial": round(serial_total_ms / rec["total_ms"], 3) if rec["total_ms"] else None,
                "mode": ("product default: straight edge first, then RRT-Connect" if straight_first
                         else "RRT-Connect forced (straight_first off)")
                + "; all queries in flight on K contexts of one GPU (rp_plan_many), median of "
                  f"{reps} passes of the whole workload"})
    return rec


SCALING_XGMI_LAT_MS = 0.025     # assumed per all-gather latency of a small RCCL message over xGMI
SCALING_XGMI_GBPS = 153.0       # one xGMI link (MI355X_MICROARCH.md), the ring's per-step bound


def kernel_slices(ctx, scene, q, flags, stream, sizes, tree_nodes=200_000):
    """ms per launch of the three hot kernel classes at each size n (states / edges /
    queries): k_validity (n uniform states), the planner's edge launch (n random
    range-length edges, coarse-first passes + pass-1 work list), the matrix-core
    nearest-node search (n queries against a tree of `tree_nodes` uniform nodes; the
    pilot, k_nn_mfma and the reduce). HIP events on the context stream
    (rp_last_kernel_ms with profiling on)."""
    ctx.set_scene(scene.boxes, scene.plane_z, scene.base)
    ctx.set_attached(-1)
    rng = np.random.default_rng(5)
    nmax = max(sizes)
    lo, hi = model.Q_LO, model.Q_HI
    qa = lo + (hi - lo) * rng.random((nmax, 9))
    d = rng.standard_normal((nmax, 9))
    rng_len = 0.2 * float(np.linalg.norm(hi - lo))
    qb = np.clip(qa + d / np.linalg.norm(d, axis=1, keepdims=True) * rng_len, lo, hi)
    res = 0.01 * float(np.linalg.norm(hi - lo))
    tree = lo + (hi - lo) * rng.random((tree_nodes, 9))
    out = {"validity": {}, "edges": {}, "nearest_node": {}}
    ctx.set_profiling(True)
    try:
        for n in sizes:
            _, ms, _ = rate_on_scene(ctx, scene, q, n, flags, stream, 10)
            out["validity"][n] = round(ms, 5)
            v = []
            for _ in range(4):
                ctx.check_edges(qa[:n], qb[:n], res)
                v.append(ctx.last_kernel_ms())
            out["edges"][n] = round(float(np.median(v[1:])), 5)
            v = []
            for _ in range(3):
                ctx.selftest_nn(qa[:n], tree, lo, hi, 8)
                v.append(ctx.last_kernel_ms())
            out["nearest_node"][n] = round(float(np.median(v[1:])), 5)
    finally:
        ctx.set_profiling(False)
    return out


def scaling_model(ctx, q, flags, stream, ranks=(2, 4, 8), thresholds=(4096, 16384, 65536, 1 << 40)):
    """Multi-GPU readiness at N = 1: for the C5 covered-well and the
    C4 configured-batch plans, the host wall time of every sub-batch (rp_debug_subbatches)
    split by the rank-group rule (<= group_repl samples: replicated on every rank, no
    exchange; larger: sharded over the ranks + one record all-gather),
    the three hot kernels measured at the per-rank slice sizes, and a projection of the
    plan time at N ranks: replicated sub-batches and the rest of the plan unchanged; a
    sharded sub-batch of C samples scaled by the measured kernel-time ratio
    (t(C / N) / t(C), summed over the three kernel classes) plus one all-gather of
    12 C + 4 N bytes (assumed latency SCALING_XGMI_LAT_MS + ring transfer at one link's
    bandwidth). A model, not a measurement: no N > 1 run on distinct GPUs exists."""
    res = {"assumptions": {"allgather_latency_ms": SCALING_XGMI_LAT_MS, "xgmi_link_gbps": SCALING_XGMI_GBPS,
                           "model": "T_N = T_other + sum_repl t_sb + sum_shard (t_sb * rho(C, N) + X(C, N)); "
                                    "rho = sum_k t_k(C / N) / sum_k t_k(C) over k_validity, edges, nearest node "
                                    "(log-interpolated between the measured sizes); group_repl threshold thr: "
                                    "sub-batches of C <= thr replicated"}}
    well = load_workload("clutter64_well")
    c4 = load_workload("goal4_pentagon_10box")
    cases = (("C5_well", {"queries": well["queries"] * 4}, C5_BATCH, 1, 8,
              scenes.Scene.from_json(well["queries"][0]["scene"])),
             ("C4_configured", c4, C4_BATCH, 0, 0, scenes.Scene.from_json(c4["queries"][14]["scene"])))
    for key, wl, batch, seed0, max_iters, scene in cases:
        plans = []
        ctx.reserve(batch, 1 << 23)
        for i, qq in enumerate(wl["queries"]):
            sc = scenes.Scene.from_json(qq["scene"])
            ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
            ctx.set_attached(qq["attached"])
            p = _abi.make_params(seed=seed0 + i, batch=batch, batch_min=batch, n_waypoints=150, timeout_s=10.0,
                                 tree_capacity=1 << 23, straight_first=False, max_iters=max_iters)
            t0 = time.perf_counter()
            ctx.plan(qq["start"], qq["goal"], model.Q_LO, model.Q_HI, p)
            plans.append((1e3 * (time.perf_counter() - t0), ctx.sub_batches()))
        sizes = sorted({1 << k for k in range(12, 19)} | {batch // n for n in (1,) + tuple(ranks)})
        sizes = [n for n in sizes if n <= max(batch, 4096)]
        ks = kernel_slices(ctx, scene, q, flags, stream, sizes)
        xs = np.log(np.array(sizes, dtype=float))

        def t_all(n):   # summed kernel-class time at n (log-log interpolation)
            tot = 0.0
            for cls in ks.values():
                ys = np.log(np.array([cls[s] for s in sizes]))
                tot += float(np.exp(np.interp(np.log(max(n, 1)), xs, ys)))
            return tot

        def project(thr, N):
            total = 0.0
            for wall, sbs in plans:
                t = wall
                for C, ms in sbs:
                    if C > thr and N > 1:
                        x = SCALING_XGMI_LAT_MS + (N - 1) / N * (12 * C + 4 * N) / (SCALING_XGMI_GBPS * 1e6)
                        t += ms * (t_all(C / N) / t_all(C) - 1.0) + x
                total += t
            return total / len(plans)

        walls = [w for w, _ in plans]
        all_sb = [sb for _, sbs in plans for sb in sbs]
        repl_ms = sum(ms for C, ms in all_sb if C <= 4096) / len(plans)
        shard_ms = sum(ms for C, ms in all_sb if C > 4096) / len(plans)
        proj = {}
        for thr in thresholds:
            name = "none" if thr >= 1 << 40 else str(thr)
            proj[name] = {str(N): round(project(thr, N), 4) for N in (1,) + tuple(ranks)}
        best = {str(N): min(proj, key=lambda k: proj[k][str(N)]) for N in ranks}
        res[key] = {"plans": len(plans), "batch": batch, "mean_plan_ms": round(float(np.mean(walls)), 4),
                    "median_plan_ms": round(float(np.median(walls)), 4),
                    "per_plan_ms": {"replicated_sub_batches": round(repl_ms, 4),
                                    "sharded_sub_batches": round(shard_ms, 4),
                                    "outside_sub_batches": round(float(np.mean(walls)) - repl_ms - shard_ms, 4),
                                    "exchange_at_N1": 0.0},
                    "sub_batch_sizes": sorted({C for C, _ in all_sb}),
                    "kernel_slices_ms": {k: {str(n): v for n, v in d.items()} for k, d in ks.items()},
                    "projected_mean_plan_ms": proj, "best_group_repl": best,
                    "projected_speedup_default_repl": {str(N): round(proj["4096"]["1"] / proj["4096"][str(N)], 3)
                                                       for N in ranks}}
    return res


def max_over_ranks(x, dev, distributed):
    """max of a float over the ranks (device tensor on RCCL, host tensor on gloo)"""
    if not distributed:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def plan_record(times, states, statuses, batch, dev, distributed, extra=None):
    """Summary of a plan workload; total = max over ranks of the summed wall time."""
    total = max_over_ranks(sum(times), dev, distributed)
    rec = {"queries": len(times), "batch": batch, "total_ms": round(total, 3),
           "median_ms": round(float(np.median(times)), 3), "max_ms": round(float(np.max(times)), 3),
           "solved": int(sum(s in (_abi.STATUS_EXACT, _abi.STATUS_APPROXIMATE) for s in statuses)),
           "states_checked": int(states), "states_per_sec_in_plan": round(states / (sum(times) / 1e3), 1)}
    rec.update(extra or {})
    return rec


def config_scenes():
    """BASELINE.md configs other than the headline C3: (name, scene, states per launch)."""
    c4 = load_workload("goal4_pentagon_10box")["queries"][14]["scene"]
    c5 = load_workload("clutter64")["queries"][0]["scene"]
    return [("C3_goal3_10box_4M", scenes.goal3_tallest(), 1 << 22),   # (the round 1-3 headline batch)
            ("C2_goal1_5box_64k", scenes.Scene(boxes=scenes.goal1_scattered(0).boxes[:5]), 1 << 16),
            ("C4_goal4_pentagon_256k", scenes.Scene.from_json(c4), 1 << 18),
            ("C5_clutter64_1M", scenes.Scene.from_json(c5), 1 << 20)]


def rate_on_scene(ctx, scene, q, n, flags, stream, steps):
    """states/s of the validity kernel on one scene (this rank; events on the
    kernel's stream)."""
    ctx.set_scene(scene.boxes, scene.plane_z, scene.base)
    for _ in range(3):
        ctx.check_states_device(q.data_ptr(), n, flags.data_ptr(), None)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        ctx.check_states_device(q.data_ptr(), n, flags.data_ptr(), None)
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    return n / (ms * 1e-3), ms, float(flags[:n].float().mean().item())


def cpu_baseline(scene, n_states, threads, chunk=1 << 24):
    """CPU oracle (test infrastructure, the cpu_baseline leg only): OpenMP validity
    over `threads` host cores on a bounded sample of the same workload (uniform
    states, generated in chunks outside the timed calls)."""
    from oracle.oracle import OracleScene
    o = OracleScene()
    o.set_scene(scene.boxes, scene.plane_z, scene.base)
    rng = np.random.default_rng(123)
    lo32, span32 = model.Q_LO.astype(np.float32), (model.Q_HI - model.Q_LO).astype(np.float32)
    o.check_states((lo32 + span32 * rng.random((4096, 9), dtype=np.float32)), threads=threads)
    dt, done = 0.0, 0
    while done < n_states:
        m = min(chunk, n_states - done)
        q = lo32 + span32 * rng.random((m, 9), dtype=np.float32)
        t0 = time.perf_counter()
        o.check_states(q, threads=threads)
        dt += time.perf_counter() - t0
        done += m
    return n_states / dt, dt


def cpu_plan_baseline(wl, seed, straight_first=True, timeout_s=10.0, batch=1):
    """The reference's CPU planner class: RRT-Connect one sample at a time (OMPL's
    loop, batch 1) in the CPU oracle on one core, per query, with the reference's
    per-query budget (motion_primitives.py:144: timeout=10.0)."""
    from oracle.oracle import OracleScene
    o = OracleScene()
    times, statuses = [], []
    for i, q in enumerate(wl["queries"]):
        sc = scenes.Scene.from_json(q["scene"])
        o.set_scene(sc.boxes, sc.plane_z, sc.base)
        o.set_attached(q["attached"])
        p = _abi.make_params(seed=seed + i, batch=batch, n_waypoints=150, timeout_s=timeout_s,
                             straight_first=straight_first)
        t0 = time.perf_counter()
        _, st, _ = o.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
        times.append(1e3 * (time.perf_counter() - t0))
        statuses.append(st)
    return times, statuses


def cpu_plan_record(times, statuses, sample):
    return {"queries": len(times), "total_ms": round(sum(times), 3), "median_ms": round(float(np.median(times)), 3),
            "max_ms": round(float(np.max(times)), 3),
            "exact": int(sum(s == _abi.STATUS_EXACT for s in statuses)),
            "approximate": int(sum(s == _abi.STATUS_APPROXIMATE for s in statuses)), "sample": sample}


def well_profile(ctx, seeds=(2, 3, 4, 0)):
    """C5 covered-well plans (131,072-sample iterations, up to the 2^20 budget) with
    the kernel-class profile on: the nearest-node and edge-launch rooflines on trees
    of 10^5 - 3 x 10^5 nodes (rp_get_profile: HIP events on the planner stream)."""
    wl = load_workload("clutter64_well")
    q = wl["queries"][0]
    sc = scenes.Scene.from_json(q["scene"])
    ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
    ctx.set_attached(q["attached"])
    ctx.set_profiling(True)
    tot = {"nn_ms": 0.0, "nn_pairs": 0.0, "edge_ms": 0.0, "edge_states": 0, "nn_launches": 0, "edge_launches": 0}
    try:
        for seed in seeds:
            p = _abi.make_params(seed=seed, batch=C5_BATCH, batch_min=C5_BATCH, n_waypoints=150, timeout_s=60.0,
                                 straight_first=False, tree_capacity=1 << 23, max_iters=8)
            ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
            pr = ctx.profile()
            for k in tot:
                tot[k] += pr[k]
    finally:
        ctx.set_profiling(False)
    pairs_per_s = tot["nn_pairs"] / (tot["nn_ms"] * 1e-3)
    nn_mfma_tf = pairs_per_s * NN_MFMA_FLOP_PER_PAIR / 1e12   # the matrix cores' executed work
    nn_alg_tf = pairs_per_s * NN_FLOP_PER_PAIR / 1e12        # the squared distance's algorithmic FLOP
    fps = flops_per_state(len(sc.boxes))
    ed_tf = tot["edge_states"] * fps / (tot["edge_ms"] * 1e-3) / 1e12
    plans = f"C5 covered-well plans, seeds {list(seeds)}, 131,072-sample iterations (trees up to 3.3e5 nodes); "
    sample = plans + ("every nearest-node search of the plans (large trees: the pilot + k_nn_mfma + k_nn_reduce_g; "
                      "small: the fused LDS-tile kernels); pairs = queries x tree nodes of each search")
    edge_sample = plans + ("every edge launch of the plans (both coarse-first passes and k_edge_rest of the large "
                           "ones); states = the states actually checked (a pass-0 failure skips the rest of its edge)")
    return ({"bound": "mfma", "achieved": round(nn_mfma_tf, 3), "peak": F16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
             "frac": round(nn_mfma_tf / F16_MFMA_PEAK_TFLOPS, 4),
             "kernel": "k_nn_mfma (+ k_ext_conn_nn / k_ext_nn / k_conn_nn on small trees)",
             "launches": tot["nn_launches"], "kernel_ms": round(tot["nn_ms"], 3), "pairs": tot["nn_pairs"],
             "pairs_per_sec": round(pairs_per_s, 1), "mfma_flop_per_pair": NN_MFMA_FLOP_PER_PAIR,
             "algorithmic": {"flop_per_pair": NN_FLOP_PER_PAIR, "achieved": round(nn_alg_tf, 3),
                             "fp32_vector_peak": VALU_PEAK_TFLOPS,
                             "frac_of_fp32_vector_peak": round(nn_alg_tf / VALU_PEAK_TFLOPS, 4)},
             "sample": sample},
            {"bound": "valu", "achieved": round(ed_tf, 3), "peak": VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
             "frac": round(ed_tf / VALU_PEAK_TFLOPS, 4), "kernel": "k_edges/k_edges_packed",
             "launches": tot["edge_launches"], "kernel_ms": round(tot["edge_ms"], 3),
             "states": int(tot["edge_states"]),
             "states_per_sec": round(tot["edge_states"] / (tot["edge_ms"] * 1e-3), 1),
             "flop_per_state": fps, "sample": edge_sample})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--settle-ms", type=float, default=250.0,
                    help="back-to-back untimed launches before the warmup steps (clock ramp)")
    # 2^24 states (604 MB of HBM) per GPU and step: at 4M the launch's last partial
    # round of waves and the launch gap cost ~5 % (34.2 vs 35.9 G states/s, same box,
    # profiles/r04/validity_batch_size.txt); the 4M rate is kept in per_config
    ap.add_argument("--states", type=int, default=1 << 24, help="states per GPU per step")
    ap.add_argument("--plan-batch", type=int, default=4096, help="RRT-Connect samples per iteration (global)")
    ap.add_argument("--no-plan", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-configs", action="store_true", help="skip the C2/C4/C5 scene rates (profiling runs)")
    ap.add_argument("--backend", default="nccl",
                    help="torch.distributed backend: nccl (= RCCL, the product path) or gloo (rehearsal of N > 1 "
                         "with several ranks on one GPU; records exchanged through a shared-memory segment)")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "0") or 0))
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    if args.backend == "gloo":   # rehearsal: ranks may share a GPU
        local = local % max(1, torch.cuda.device_count())
    if distributed:
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.backend)
    dev = torch.device("cuda", local)

    wl = load_workload("goal3_tallest_10box")
    scene = scenes.goal3_tallest()           # 10 boxes, initial layout
    ctx = Context(device=local, robot=model.robot_desc())
    ctx.set_scene(scene.boxes, scene.plane_z, scene.base)

    # synthetic states in HBM (per-rank stream of uniform samples, float32 bounds)
    n = args.states
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    lo = torch.tensor(model.Q_LO, dtype=torch.float32, device=dev)
    hi = torch.tensor(model.Q_HI, dtype=torch.float32, device=dev)
    q = lo + (hi - lo) * torch.rand((n, 9), generator=g, device=dev, dtype=torch.float32)
    q = q.contiguous()
    flags = torch.empty(n, dtype=torch.uint8, device=dev)
    # the kernel runs on the context's own stream and the HIP events are recorded on
    # it (torch.cuda.ExternalStream over rp_get_stream): no extra hardware queue per
    # rank (an extra torch stream per process slowed later plans 2x when ranks share
    # a GPU, tools/share_probe.py)
    stream = torch.cuda.ExternalStream(ctx.stream_handle(), device=dev)
    torch.cuda.synchronize(dev)

    def step():
        ctx.check_states_device(q.data_ptr(), n, flags.data_ptr(), None)

    # clock settle: a fresh process's first ~100 launches run while the GPU's clocks
    # ramp (tools/clock_probe.py, profiles/r05/clock_ramp.json: 500-530 us per launch
    # over launches 2-15, 415 us from launch ~100 on, flat for 9,500 launches), so
    # back-to-back launches for --settle-ms of wall time come before the W warmup
    # steps; the timed region is still exactly K steps. 0 disables it.
    settle_n, ts = 0, time.perf_counter()
    while (time.perf_counter() - ts) * 1e3 < args.settle_ms:
        for _ in range(10):
            step()
        settle_n += 10
        torch.cuda.synchronize(dev)
    settle_ms = (time.perf_counter() - ts) * 1e3
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    kernel_ms = e0.elapsed_time(e1) / args.steps      # only the validity kernel is on this stream
    wall_max = max_over_ranks(wall, dev, distributed)
    valid_frac = float(flags.float().mean().item())

    total_states = n * world * args.steps
    value = total_states / wall_max
    ms_per_step = 1e3 * wall_max / args.steps

    # ---- the other BASELINE configs' scenes (validity throughput per GPU, no collective)
    per_config = {}
    for name, sc_c, n_c in ([] if args.no_configs else config_scenes()):
        n_c = min(n_c, n)
        rate, ms, vf = rate_on_scene(ctx, sc_c, q, n_c, flags, stream, 10)
        per_config[name] = {"boxes": len(sc_c.boxes), "states_per_launch": n_c,
                            "states_per_sec_per_gpu": round(rate, 1), "kernel_ms": round(ms, 5),
                            "valid_fraction": round(vf, 4)}
    ctx.set_scene(scene.boxes, scene.plane_z, scene.base)

    # ---- plan wall-time: C3 (headline), C4 (262,144-sample iterations) and C5
    # (131,072-sample iterations); every iteration is sharded over the ranks when
    # N > 1 (RCCL all-gather per phase)
    plan = None
    rank_group = None
    if not args.no_plan:
        # the rank group: at N > 1 a plan number without the group would be a
        # single-rank number, so if any rank fails to join it every rank skips the plan
        # workloads (the ranks agree on that first) and the line reports the error;
        # the validity metric above stands on its own
        group = None
        group_err = None
        if distributed:
            # a rank group whose exchange never completes (RCCL at N > 1 runs only on
            # the driver's node) must not hold the line: each plan wait gives up after
            # 30 s instead of 120 (the longest legitimate wait here is milliseconds),
            # and after a failed workload the rest are skipped (a stuck stream would
            # fail them all, one watchdog period each)
            os.environ.setdefault("RBE_WAIT_WATCHDOG_S", "30")
            from rbe550_final_project_amd.distributed import Group
            try:
                group = Group(ctx, transport="shm" if args.backend == "gloo" else "rccl")
            except Exception as ex:
                group_err = f"rank {rank}: {ex!r}"[:300]
            errs = [None] * world
            dist.all_gather_object(errs, group_err)
            if any(errs):
                if group is not None:
                    group.leave()
                group = None
                rank_group = {"error": [e for e in errs if e]}
            else:
                # what the transport itself reports on every rank (RCCL: ncclCommUserRank /
                # ncclCommCount of the library's communicator)
                views = [None] * world
                dist.all_gather_object(views, ctx.group_info())
                rank_group = {"transport": views[0]["transport"], "ranks": views,
                              "consistent": all(v["world"] == world and v["rank"] == r for r, v in enumerate(views))}
        try:
            if distributed and group is None:
                raise RuntimeError(f"no rank group: {rank_group['error']}")
            # warm-up: one untimed pass over the whole C3 workload in both modes (a
            # 2-query warm-up left the first timed workload at 2x its median on one box)
            run_plans(ctx, wl, args.plan_batch, 100, group)
            run_plans(ctx, wl, args.plan_batch, 100, group, straight_first=False)
            times, pstates, st = run_plans(ctx, wl, args.plan_batch, 0, group)
            plan = plan_record(times, pstates, st, args.plan_batch, dev, distributed,
                               {"mode": "product default: straight edge first, then RRT-Connect"})
            # C1: goal1_scattered's 12 queries (BASELINE configs[0]; the reference runs
            # it on the CPU), product default and RRT-forced
            wl1 = load_workload("goal1_scattered_6box")
            t1, s1, st1 = run_plans(ctx, wl1, args.plan_batch, 0, group)
            plan["C1_goal1"] = plan_record(t1, s1, st1, args.plan_batch, dev, distributed,
                                           {"mode": "product default: straight edge first, then RRT-Connect"})
            t1, s1, st1 = run_plans(ctx, wl1, args.plan_batch, 0, group, straight_first=False)
            plan["C1_goal1_rrt"] = plan_record(t1, s1, st1, args.plan_batch, dev, distributed,
                                               {"mode": "RRT-Connect forced (straight_first off)"})
            # C2: the single pick -> place segment (2 queries, 5 boxes) with 65,536-sample
            # iterations over 10 seeds (BASELINE configs[1]: median of 20 plans)
            wl2 = load_workload("single_pick_place_5box")
            wl2x = {"queries": wl2["queries"] * 10}
            t2, s2, st2 = run_plans(ctx, wl2x, C2_BATCH, 0, group)
            plan["C2_single_64k"] = plan_record(t2, s2, st2, C2_BATCH, dev, distributed,
                                                {"mode": "product default: straight edge first, then RRT-Connect"})
            t2, s2, st2 = run_plans(ctx, wl2x, C2_BATCH, 0, group, batch_min=C2_BATCH, straight_first=False)
            plan["C2_single_64k_rrt"] = plan_record(t2, s2, st2, C2_BATCH, dev, distributed,
                                                    {"mode": "RRT-Connect forced, 65,536-sample iterations",
                                                     "batch_min": C2_BATCH})
            # the same queries with RRT-Connect forced (straight_first off)
            t3, s3, st3 = run_plans(ctx, wl, args.plan_batch, 0, group, straight_first=False)
            plan["C3_rrt"] = plan_record(t3, s3, st3, args.plan_batch, dev, distributed,
                                         {"mode": "RRT-Connect forced (straight_first off)"})
            # the same queries through the reference's API end to end:
            # PlannerInterface.plan_path with the call site's arguments (run_plan_path)
            for key, wname, sf in (("C3_plan_path", "goal3_tallest_10box", True),
                                   ("C3_plan_path_rrt", "goal3_tallest_10box", False),
                                   ("C1_plan_path", "goal1_scattered_6box", True),
                                   ("C1_plan_path_rrt", "goal1_scattered_6box", False)):
                w = wl if wname == "goal3_tallest_10box" else wl1
                run_plan_path(ctx, w, 100, sf)   # warm-up pass (untimed)
                tp, sp, stp, parts = run_plan_path(ctx, w, 0, sf)
                plan[key] = plan_record(tp, sp, stp, args.plan_batch, dev, distributed,
                                        {"mode": "PlannerInterface.plan_path(qpos_goal, num_waypoints=150, "
                                                 "attached_object, timeout=10.0) through tests/mock_genesis.py"
                                                 + ("" if sf else "; RRT-Connect forced"),
                                         "median_parts_ms": parts})
            # C3 "pipelined" (BASELINE configs[2]: ~20 RRT queries pipelined): the 21
            # queries kept in flight on K contexts of this GPU (native.plan_pipelined),
            # the wall time of the whole workload next to the serial legs above
            if not distributed:
                for key, sf in (("C3_pipelined", True), ("C3_pipelined_rrt", False)):
                    serial = plan["total_ms"] if sf else plan["C3_rrt"]["total_ms"]
                    plan[key] = run_plans_pipelined(local, wl, args.plan_batch, sf, serial)
        except Exception as ex:  # report, keep the primary metric
            plan = {"error": repr(ex)[:300]}
        plan_failed = plan is None or "error" in plan
        # configured-batch workloads: C4 (262,144-sample iterations) and C5
        # (131,072-sample iterations: clutter64, and the covered well, whose trees
        # grow to 10^5 - 3 x 10^5 nodes over up to 8 iterations = the 2^20 budget);
        # "_sched": the product's batch schedule (64 samples first, doubling to the
        # configured batch) on the same queries
        well = load_workload("clutter64_well")
        wellx = {"queries": well["queries"] * 4}
        for key, wl_c, batch, bmin, seeds_from, max_iters in ([] if (distributed and (group is None or plan_failed))
                                                               else (
                ("C4_pentagon", load_workload("goal4_pentagon_10box"), C4_BATCH, C4_BATCH, 0, 0),
                ("C4_pentagon_sched", load_workload("goal4_pentagon_10box"), C4_BATCH, 0, 0, 0),
                # the completed pentagon: deep grasps between placed blocks, no valid
                # straight edge on any query (tests/golden/make_workloads.py)
                ("C4_ring", load_workload("goal4_pentagon_ring"), C4_BATCH, C4_BATCH, 0, 0),
                ("C4_ring_sched", load_workload("goal4_pentagon_ring"), C4_BATCH, 0, 0, 0),
                ("C5_clutter64", load_workload("clutter64"), C5_BATCH, C5_BATCH, 0, 0),
                ("C5_well", wellx, C5_BATCH, C5_BATCH, 1, 8),
                ("C5_well_sched", wellx, C5_BATCH, 0, 1, 8))):
            try:
                extra = {}
                tq, sq, stq = run_plans(ctx, wl_c, batch, seeds_from, group, batch_min=bmin, tree_capacity=1 << 23,
                                        stats_out=extra, straight_first=False, max_iters=max_iters)
                it = max(1, int(extra.get("iterations", 0)))
                extra = {"mode": "RRT-Connect forced (straight_first off)", "batch_min": bmin or 64,
                         "exchange_ms": round(extra.get("exchange_ms", 0.0), 3),
                         "exchange_ms_per_iteration": round(extra.get("exchange_ms", 0.0) / it, 4),
                         "iterations": int(extra.get("iterations", 0)), "samples": int(extra.get("samples", 0)),
                         "max_iters": max_iters or None}
                plan[key] = plan_record(tq, sq, stq, batch, dev, distributed, extra)
            except Exception as ex:
                plan[key] = {"error": repr(ex)[:300]}
                if distributed:
                    break
        # multi-GPU through the reference's own API in ONE process (the drop-in with
        # planning.configure(devices=...)): every visible GPU, or two contexts on the
        # one GPU of a single-GPU box (a rehearsal of the group: both share the chip)
        if not distributed:
            ndev = torch.cuda.device_count()
            devs = tuple(range(ndev)) if ndev > 1 else (0, 0)
            for key, dv in (("C5_well_plan_path", (local,)), ("C5_well_plan_path_devices", devs)):
                try:
                    tq, sq, stq, info = run_plan_path_devices(dv)
                    plan[key] = plan_record(tq, sq, stq, C5_BATCH, dev, distributed, {
                        "mode": "PlannerInterface.plan_path(qpos_goal, qpos_start, num_waypoints=150, timeout=10.0) "
                                "through tests/mock_genesis.py, covered-well query, seeds 1-4, 131,072-sample "
                                "iterations, planning.configure(devices=...)",
                        "devices": list(dv), "ranks": info,
                        "shares_gpu": len(set(dv)) < len(dv)})
                except Exception as ex:
                    plan[key] = {"error": repr(ex)[:300]}
        if group is not None:   # every rank done with the group's segment / communicator
            dist.barrier()
            group.leave()

    # ---- nearest-node and edge-launch rooflines on large trees (this rank, no group)
    rooflines_plan = None
    if not args.no_plan and rank == 0 and not distributed:
        try:
            nn_roof, edge_roof = well_profile(ctx)
            rooflines_plan = {"nearest_node": nn_roof, "edges": edge_roof}
        except Exception as ex:
            rooflines_plan = {"error": repr(ex)[:300]}
    # ---- multi-GPU readiness without the hardware: sub-batch accounting, the kernels
    # at per-rank slice sizes, projected N = 2 / 4 / 8 plan times (a model)
    scaling = None
    if not args.no_plan and rank == 0 and not distributed:
        try:
            scaling = scaling_model(ctx, q, flags, stream)
        except Exception as ex:
            scaling = {"error": repr(ex)[:300]}
    ctx.set_scene(scene.boxes, scene.plane_z, scene.base)
    ctx.set_attached(-1)

    flop = flops_per_state(len(scene.boxes))
    achieved_tflops = n * flop / (kernel_ms * 1e-3) / 1e12
    traffic = pmc_traffic(n)
    roofline = {"bound": "valu", "achieved": round(achieved_tflops, 3), "peak": VALU_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": round(achieved_tflops / VALU_PEAK_TFLOPS, 4), "traffic": traffic,
                "kernel": "k_validity", "kernel_ms": round(kernel_ms, 5), "flop_per_state": flop,
                "hbm": {"achieved": round(n * BYTES_PER_STATE / (kernel_ms * 1e-3) / 1e9, 2),
                        "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                        "frac": round(n * BYTES_PER_STATE / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 5),
                        "bytes_per_state": BYTES_PER_STATE}}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        try:
            hi = host_info()
            # the box's CPU share for one GPU is OMP_NUM_THREADS (16 on the GPU pool);
            # the whole machine's count is recorded beside it (host.nproc)
            threads = args.cpu_threads or int(hi["omp_num_threads"] or 0) or (hi["affinity"] or 1)
            sample = 1 << 27   # ~8-10 s of oracle work on 16 cores
            rate, dt = cpu_baseline(scene, sample, threads)
            rate1, dt1 = cpu_baseline(scene, 1 << 22, 1)      # one core: the per-core rate
            cpu = {"value": round(rate, 1), "unit": "states/s", "cores": threads, "kind": "port",
                   "sample": f"{sample} uniform states, goal3 10-box scene, OpenMP CPU oracle ({dt:.1f} s)",
                   "per_core": round(rate1, 1), "per_core_sample": f"{1 << 22} states on 1 thread ({dt1:.1f} s)",
                   "host": hi,
                   # the whole host, extrapolated: this job's CPU share is OMP_NUM_THREADS
                   # threads (the pool's rule for one GPU), so the affinity count is not
                   # run; measured per-thread rate at `threads` x the affinity count
                   "full_host_extrapolated": {
                       "value": round(rate / threads * (hi["affinity"] or threads), 1), "threads": hi["affinity"],
                       "basis": f"{threads}-thread rate / {threads} x {hi['affinity']} threads (linear scaling, "
                                "an upper bound: SMT threads share cores)"}}
            # plan wall-time of the reference's CPU planner class (sequential
            # RRT-Connect, batch 1, one core, 10 s budget per query)
            plans = {}
            for key, wname, sf, reps in (("C1_goal1", "goal1_scattered_6box", True, 1),
                                         ("C1_goal1_rrt", "goal1_scattered_6box", False, 1),
                                         ("C3", "goal3_tallest_10box", True, 1),
                                         ("C3_rrt", "goal3_tallest_10box", False, 1),
                                         ("C2_rrt", "single_pick_place_5box", False, 10),
                                         ("C4_rrt", "goal4_pentagon_10box", False, 1),
                                         ("C4_ring", "goal4_pentagon_ring", True, 1),
                                         ("C5_clutter64_rrt", "clutter64", False, 1),
                                         ("C5_well_rrt", "clutter64_well", False, 1)):
                w = load_workload(wname)
                w = {"queries": w["queries"] * reps}
                t, stc = cpu_plan_baseline(w, 0, straight_first=sf)
                plans[key] = cpu_plan_record(t, stc, f"{wname}: {'straight edge first, then ' if sf else ''}"
                                                     "sequential RRT-Connect (batch 1, OMPL's loop) with an exact "
                                                     "kd-tree nearest-node index (OMPL: GNAT), CPU oracle, 1 core, "
                                                     "10 s budget per query")
            cpu["plans"] = plans
            # legacy keys (round 1 records)
            cpu["plan_total_ms"], cpu["plan_median_ms"] = plans["C3"]["total_ms"], plans["C3"]["median_ms"]
            cpu["plan_rrt_total_ms"], cpu["plan_rrt_median_ms"] = plans["C3_rrt"]["total_ms"], plans["C3_rrt"]["median_ms"]
        except Exception as ex:
            cpu = {"error": repr(ex)[:300]}

    if rank == 0:
        out = {"metric": METRIC, "value": round(value, 1), "unit": "states/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 5),
               "settle": {"ms": round(settle_ms, 1), "launches": settle_n,
                          "why": "untimed back-to-back launches before the warmup steps: GPU clock ramp "
                                 "(tools/clock_probe.py)"},
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
               "data": "synthetic: uniform 9-D Franka states in the float32 joint bounds (HBM resident); "
                       "goal3 10-box scene; plan queries from tests/golden/workloads",
               "config": {"workload": "C3 goal3_tallest 10-block scene: validity batch per GPU + 21-query plan",
                          "states_per_gpu": n, "global_batch": n * world, "parallelism": f"dp{world}",
                          "valid_fraction": round(valid_frac, 4)},
               "rank_group": rank_group,
               "plan_wall": plan, "per_config": per_config, "roofline": roofline,
               "rooflines_plan": rooflines_plan, "scaling_model": scaling, "cpu_baseline": cpu}
        print(json.dumps(out), flush=True)
    ctx.close()
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
