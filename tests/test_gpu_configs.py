"""GPU plans at the BASELINE configs' own batch sizes, bit for bit against the
oracle's golden plans (tests/golden/plans_configured.npz, made by
tests/golden/make_plan_fixtures.py):

  C2  65,536-sample iterations (single pick -> place, 5 boxes)
  C4  262,144-sample iterations (pentagon, yawed boxes)
  C5  131,072-sample iterations: clutter64, and the covered-well query whose
      trees reach 10^5 - 3 x 10^5 nodes over 3 - 8 iterations (nearest-node
      search over large trees; seed 0 spends the whole 2^20-sample budget and
      returns the APPROXIMATE path)

each through the single-rank iteration (ordered sub-batches: speculative first,
two-phase when large; or the whole iteration at once), the one-exchange group
iteration at world 1 (RBE_PLAN_GROUPED=1), and the RCCL transport at world 1
(ncclAllGather on the planner stream). Tolerance in the
tests: 1e-5 rad (north_star); the measured difference is 0."""
import json
import os

import numpy as np
import pytest

from rbe550_final_project_amd import _abi, model, native, scenes
from rbe550_final_project_amd.native import Context

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
FIX = np.load(os.path.join(GOLD, "plans_configured.npz"))
META = json.loads(str(FIX["meta"]))
TOL = 1e-5


def _case(name):
    m = META[name]
    q = json.load(open(os.path.join(GOLD, "workloads", m["workload"] + ".json")))["queries"][m["query"]]
    p = _abi.make_params(seed=m["seed"], batch=m["batch"], batch_min=m["batch"], n_waypoints=150, timeout_s=3600.0,
                         straight_first=False, tree_capacity=1 << 23, max_iters=m["max_iters"])
    return m, q, p


def _check(ctx, name):
    m, q, p = _case(name)
    sc = scenes.Scene.from_json(q["scene"])
    ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
    ctx.set_attached(q["attached"])
    path, st = ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
    s = ctx.stats()
    ref = FIX[name]
    assert st == m["status"], (name, st, m["status"])
    assert s["iterations"] == m["iterations"], (name, s["iterations"], m)
    assert (s["start_tree_size"], s["goal_tree_size"]) == (m["start_tree"], m["goal_tree"]), (name, s, m)
    assert path.shape == ref.shape == (150, 9)
    assert np.max(np.abs(path - ref)) <= TOL
    assert np.array_equal(path, ref)
    return s


@pytest.mark.parametrize("name", sorted(META))
def test_configured_batch_plan_equals_oracle(gpu_ctx, name):
    """Default execution: each configured iteration runs as ordered sub-batches
    (64 samples, then x4 but at least a quarter of what is left; at least a quarter
    of the iteration first on trees of >= 4,096 nodes) and ends after the one holding
    the first REACHED sample."""
    s = _check(gpu_ctx, name)
    assert s["samples"] <= META[name]["iterations"] * META[name]["batch"]
    if META[name]["status"] == _abi.STATUS_APPROXIMATE:   # every iteration ran whole
        assert s["samples"] == META[name]["iterations"] * META[name]["batch"]


@pytest.mark.parametrize("name", ["C2_q0_s0", "C2_q1_s2", "C4_q10", "C5_clutter64", "C5_well_s3", "C5_well_s0"])
@pytest.mark.parametrize("chunk", ["-1", "16384"])
def test_configured_batch_sub_batching(gpu_ctx, name, chunk, monkeypatch):
    """The same plans with the iteration in one piece ("-1": every sample of the
    iteration checked, the appends cut at the winning sample) and with 16,384-sample
    first sub-batches: sub-batching changes the work, not the trees."""
    monkeypatch.setenv("RBE_PLAN_CHUNK", chunk)
    s = _check(gpu_ctx, name)
    if chunk == "-1":
        assert s["samples"] == META[name]["iterations"] * META[name]["batch"]


@pytest.mark.parametrize("name", ["C2_q0_s0", "C4_q0", "C5_clutter64", "C5_well_s4", "C5_well_s0"])
def test_configured_batch_group_iteration_world1(gpu_ctx, name, monkeypatch):
    """The rank-group iteration (speculative front + record exchange + multi-block
    accept) at world 1 without a transport: same plans."""
    monkeypatch.setenv("RBE_PLAN_GROUPED", "1")
    _check(gpu_ctx, name)


@pytest.mark.parametrize("name", ["C2_q1_s1", "C5_well_s4"])
@pytest.mark.parametrize("repl", ["0", ""])
def test_rccl_transport_world1(name, repl, monkeypatch):
    """The RCCL transport end to end on one GPU (a 1-rank communicator: the
    records go through ncclAllGather on the planner stream). RBE_GROUP_REPL=0 shards
    every sub-batch (every one exchanges); the default replicates sub-batches of up to
    4,096 samples (the 64-sample first one of these plans: no exchange)."""
    monkeypatch.setenv("RBE_GROUP_REPL", repl)
    ctx = Context(device=0, robot=model.robot_desc())
    try:
        ctx.group_init_rccl(0, 1, native.rccl_unique_id())
        s = _check(ctx, name)
        if repl == "0":
            assert s["exchange_ms"] > 0.0
        ctx.group_leave()
        _check(ctx, name)
    finally:
        ctx.close()


def test_rccl_replicated_timeout_vote_world1(oracle_lib):
    """The RCCL branch of the timeout vote (rp_lib.hip group_vote: a one-word
    ncclAllGather and read-back) on a 1-rank communicator: a plan whose iterations all
    open replicated (1,152-sample batches, every sub-batch <= 4,096) with an expired
    budget runs iterations 0-6, votes through RCCL at iteration 7 and stops; its
    APPROXIMATE path is the oracle's after exactly 7 iterations (max_iters = 7, no
    timeout) and the same context's after group_leave."""
    q = json.load(open(os.path.join(GOLD, "workloads", "clutter64_well.json")))["queries"][0]
    sc = scenes.Scene.from_json(q["scene"])
    p = _abi.make_params(seed=3, batch=1152, n_waypoints=150, timeout_s=1e-9, straight_first=False)
    ctx = Context(device=0, robot=model.robot_desc())
    try:
        ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
        ctx.set_attached(q["attached"])
        ctx.group_init_rccl(0, 1, native.rccl_unique_id())
        assert ctx.group_info()["transport"] == "rccl"
        path, st = ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
        s = ctx.stats()
        assert s["iterations"] == 7, s
        assert s["exchange_ms"] > 0.0, s   # the vote went through RCCL
        assert st == _abi.STATUS_APPROXIMATE
        p7 = _abi.make_params(seed=3, batch=1152, n_waypoints=150, timeout_s=3600.0, straight_first=False,
                              max_iters=7)
        o = oracle_lib.OracleScene()
        o.set_scene(sc.boxes, sc.plane_z, sc.base)
        o.set_attached(q["attached"])
        ref, st_ref, ost = o.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p7)
        assert st_ref == _abi.STATUS_APPROXIMATE and ost["iterations"] == 7
        assert np.array_equal(path, ref)
        assert (s["start_tree_size"], s["goal_tree_size"]) == (ost["start_tree_size"], ost["goal_tree_size"])
        ctx.group_leave()
        path1, st1 = ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p7)
        assert st1 == st_ref and np.array_equal(path1, ref)
    finally:
        ctx.close()


@pytest.mark.parametrize("name,split", [("C2_q0_s1", "1"), ("C4_q5", "1"), ("C5_well_s4", "0"), ("C5_well_s2", "1")])
@pytest.mark.parametrize("grouped", ["0", "1"])
@pytest.mark.parametrize("mfma", ["4", "0"])
def test_nearest_node_split_forced(gpu_ctx, name, split, grouped, mfma, monkeypatch):
    """The split nearest-node search (queries x tree ranges, lexicographic (distance,
    index) minimum over the ranges) forced on / off, with the matrix-core filter
    (k_nn_mfma, the default) and the packed-f32 one (k_nn_part, RBE_NN_MFMA=0),
    through the two-phase and the group iteration: same plans as the oracle."""
    monkeypatch.setenv("RBE_NN_SPLIT", split)
    monkeypatch.setenv("RBE_PLAN_GROUPED", grouped)
    monkeypatch.setenv("RBE_NN_MFMA", mfma)
    _check(gpu_ctx, name)


@pytest.mark.parametrize("name", ["C5_well_s0", "C5_well_s3"])
@pytest.mark.parametrize("mfma", ["1", "4"])
def test_nearest_node_mfma_row_blocks(gpu_ctx, name, mfma, monkeypatch):
    """The matrix-core search with 1 and 4 row blocks of 16 queries per wave (8, the
    default, everywhere else) on the largest trees (3.3 x 10^5 nodes, 7-8
    iterations): same plans."""
    monkeypatch.setenv("RBE_NN_MFMA", mfma)
    _check(gpu_ctx, name)


@pytest.mark.parametrize("name", ["C5_well_s0", "C5_well_s3", "C4_q5", "C2_q0_s1"])
@pytest.mark.parametrize("pilot,mfma", [("0", "8"), ("4", "8"), ("0", "4"), ("16", "4"), ("2", "1"), ("32", "8")])
@pytest.mark.parametrize("share", ["0", "1"])
def test_nearest_node_pilot(gpu_ctx, name, pilot, mfma, share, monkeypatch):
    """The pilot search (every pilot-th tile of the whole tree first; its bests start
    every range of the full search, whose ranges then return their minimum over the
    nodes at or below that distance, or none): off, and at strides 2 / 4 / 16 / 32 with
    1 / 4 / 8 row blocks, on every search it applies to (host-sized, >= 2 ranges,
    T >= stride x 1,024 nodes: the C5 well's trees; the small configs' searches run
    without one); with and without the ranges sharing each query's bound (RBE_NN_SHARE:
    a range's threshold follows the smallest exact best any range has published, its
    own minimum stays its own). Same plans."""
    monkeypatch.setenv("RBE_NN_PILOT", pilot)
    monkeypatch.setenv("RBE_NN_MFMA", mfma)
    monkeypatch.setenv("RBE_NN_SHARE", share)
    monkeypatch.setenv("RBE_NN_SPLIT", "1")
    _check(gpu_ctx, name)


@pytest.mark.parametrize("name", ["C5_well_s0", "C5_well_s3", "C4_q5"])
@pytest.mark.parametrize("devgeom", ["0", "1"])
def test_nearest_node_status_geometry(gpu_ctx, name, devgeom, monkeypatch):
    """The connect searches' query count is on the device (the accepted extensions):
    their tree ranges follow the actual count in the kernel (rp_nn.h nn_geom,
    k_nn_reduce_g), or the host geometry of the largest count (RBE_NN_DEVGEOM=0).
    Same plans either way."""
    monkeypatch.setenv("RBE_NN_DEVGEOM", devgeom)
    monkeypatch.setenv("RBE_NN_SPLIT", "1")
    _check(gpu_ctx, name)


@pytest.mark.parametrize("name", ["C5_well_s0", "C5_well_s3", "C4_q5", "C2_q0_s1"])
@pytest.mark.parametrize("pk,cmin", [("0", ""), ("2", "0"), ("4", "0"), ("8", ""), ("-2", "0"), ("-3", "")])
@pytest.mark.parametrize("units", ["1", "0"])
def test_coarse_first_edge_passes_in_plans(gpu_ctx, name, pk, cmin, units, monkeypatch):
    """The planner's edge launches through the coarse-first passes (slot 0 and every
    pk-th interior slot first, then the rest of the edges still valid; RBE_EDGE_COARSE)
    or one pass (0), at the default size threshold and forced on every wave-compacted
    launch (RBE_EDGE_COARSE_MIN=0), pass 1 over the work list of its live (group,
    round) units (k_edge_units / k_edges_units) or the groups x rounds grid
    (RBE_EDGE_UNITS=0): same plans."""
    monkeypatch.setenv("RBE_EDGE_COARSE", pk)
    monkeypatch.setenv("RBE_EDGE_UNITS", units)
    if cmin:
        monkeypatch.setenv("RBE_EDGE_COARSE_MIN", cmin)
    _check(gpu_ctx, name)


@pytest.mark.parametrize("name", ["C5_well_s0", "C5_well_s3", "C4_q5", "C2_q0_s1"])
@pytest.mark.parametrize("lb", ["0", "1"])
def test_lookback_accepts(gpu_ctx, name, lb, monkeypatch):
    """Sub-batches above FUSE_MAX accept their extensions and connect chains in one
    launch each (flags, a decoupled look-back scan and the appends: k_ext_accept_lb,
    k_conn_accept_lb) or through flag + hipCUB scan + append (RBE_ACCEPT_LB=0): same
    trees, same plans."""
    monkeypatch.setenv("RBE_ACCEPT_LB", lb)
    _check(gpu_ctx, name)


@pytest.mark.parametrize("name", ["C5_well_s0", "C5_well_s2", "C5_well_s3", "C5_well_s4", "C4_q5", "C4_ring_q3",
                                  "C2_q0_s1", "C5_clutter64"])
@pytest.mark.parametrize("early", ["0", "1"])
@pytest.mark.parametrize("lb", ["0", "1"])
def test_early_status_publication(gpu_ctx, name, early, lb, monkeypatch):
    """Large single-rank sub-batches publish their status from k_finalize and skip the
    in-loop simplification steps (RBE_EARLY_STATUS); the sub-batch that solves then
    runs the whole program after the loop. Same plans, statuses and trees, with the
    look-back and the scan accepts alike (the approximate C5_well_s0 case included)."""
    monkeypatch.setenv("RBE_EARLY_STATUS", early)
    monkeypatch.setenv("RBE_ACCEPT_LB", lb)
    _check(gpu_ctx, name)


@pytest.mark.parametrize("name", ["C5_well_s0", "C5_well_s2", "C5_well_s3", "C5_well_s4", "C4_q5", "C4_ring_q3",
                                  "C2_q0_s1", "C5_clutter64"])
@pytest.mark.parametrize("speculate", ["0", "1"])
def test_pipelined_sub_batches(gpu_ctx, name, speculate, monkeypatch):
    """A two-phase sub-batch enqueues the next sub-batch's extension phase before it
    reads its own status (RBE_PLAN_PIPELINE); that phase is gated on the first REACHED
    word, so a sub-batch that solves leaves the trees, the simplification and the
    counters as they were. Same plans, statuses and trees as the golden ones, and the
    same edges / samples / iterations counted as without the pipeline
    (RBE_PLAN_SPECULATE=0: every sub-batch two-phase, small ones included). The states
    count is compared to 1e-4: an edge's remaining slots are skipped once another wave
    of the same launch has failed the edge, so it depends on the waves' timing (31 of
    10,031,082 states between two runs of the approximate C5_well_s0 plan). A gated
    sub-batch that still checked its edges' far endpoints (nd 0 instead of -1) showed
    here as 98,314 extra states on C5_well_s2."""
    monkeypatch.setenv("RBE_PLAN_SPECULATE", speculate)
    stats = {}
    for pipe in ("0", "1"):
        monkeypatch.setenv("RBE_PLAN_PIPELINE", pipe)
        s = _check(gpu_ctx, name)
        stats[pipe] = {k: s[k] for k in ("states_checked", "edges_checked", "samples", "iterations")}
    st0, st1 = stats["0"].pop("states_checked"), stats["1"].pop("states_checked")
    assert stats["0"] == stats["1"], (name, stats)
    assert abs(st0 - st1) <= 1e-4 * st0, (name, st0, st1)


def test_lookback_error_flag_is_not_sticky(gpu_ctx):
    """the look-back accepts' poll-budget flag lives on the device. A plan
    that finds it raised fails (NativeError) and clears it, so the context's next
    large plan succeeds with the golden answer instead of failing forever.
    (rp_debug_lb_poison raises the flag as an exhausted budget would.)"""
    import ctypes as C
    L = native.load()
    L.rp_debug_lb_poison.argtypes = [C.c_void_p]
    assert L.rp_debug_lb_poison(gpu_ctx._h) == 0
    m, q, p = _case("C5_well_s3")
    sc = scenes.Scene.from_json(q["scene"])
    gpu_ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
    gpu_ctx.set_attached(q["attached"])
    with pytest.raises(native.NativeError, match="poll budget"):
        gpu_ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
    _check(gpu_ctx, "C5_well_s3")
    _check(gpu_ctx, "C4_q5")


def test_kernel_profile_of_a_plan(gpu_ctx):
    """rp_set_profiling / rp_get_profile (bench.py's nearest-node and edge rooflines):
    the profiled plan is the same plan, and the profile counts its launches, time
    and work."""
    gpu_ctx.set_profiling(True)
    try:
        s = _check(gpu_ctx, "C5_well_s4")
        pr = gpu_ctx.profile()
    finally:
        gpu_ctx.set_profiling(False)
    assert pr["nn_launches"] >= META["C5_well_s4"]["iterations"] and pr["edge_launches"] > 0
    assert pr["nn_ms"] > 0 and pr["edge_ms"] > 0 and pr["nn_pairs"] > 1e8
    assert pr["edge_states"] == s["states_checked"]


def test_validity_kernel_timing_needs_profiling():
    """rp_last_kernel_ms: HIP events around rp_check_states_device only with
    profiling on (they cost two API calls per launch); an error before any timed
    call, a positive kernel time after one. (Device buffers through the HIP runtime
    the library itself loaded, not torch's.)"""
    import ctypes as C
    hip = C.CDLL("libamdhip64.so.7")
    ctx = Context(device=0, robot=model.robot_desc())
    n = 4096
    q = (np.random.default_rng(1).random((n, 9)) * (model.Q_HI - model.Q_LO) + model.Q_LO).astype(np.float32)
    dq, df = C.c_void_p(), C.c_void_p()
    assert hip.hipMalloc(C.byref(dq), C.c_size_t(q.nbytes)) == 0
    assert hip.hipMalloc(C.byref(df), C.c_size_t(n)) == 0
    try:
        assert hip.hipMemcpy(dq, q.ctypes.data_as(C.c_void_p), C.c_size_t(q.nbytes), 1) == 0
        sc = scenes.goal3_tallest()
        ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
        ctx.check_states_device(dq.value, n, df.value)
        with pytest.raises(native.NativeError):
            ctx.last_kernel_ms()
        ctx.set_profiling(True)
        ctx.check_states_device(dq.value, n, df.value)
        assert ctx.last_kernel_ms() > 0.0
        ctx.set_profiling(False)
    finally:
        ctx.close()
        hip.hipFree(dq)
        hip.hipFree(df)


@pytest.mark.parametrize("name", ["C2_q0_s0", "C4_q10", "C5_clutter64", "C5_well_s3", "C5_well_s0"])
@pytest.mark.parametrize("packed", ["0", "1"])
def test_configured_batch_edge_kernels(gpu_ctx, name, packed, monkeypatch):
    """Every large edge launch through one kernel: RBE_EDGE_PACKED=0 the
    wave-compacted (edge, slot) grid (k_edges: groups of 64 edges, kmax waves each,
    grid-striding when the grid is capped), 1 the globally scanned item list
    (k_edges_packed); whole iterations, so the launches are the configured sizes."""
    monkeypatch.setenv("RBE_EDGE_PACKED", packed)
    monkeypatch.setenv("RBE_PLAN_CHUNK", "-1")
    _check(gpu_ctx, name)
