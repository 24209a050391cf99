"""GPU parity: librbe_mi355x.so (HIP, gfx950) vs the CPU oracle on the same inputs.

Bar (BASELINE.json north_star): integer collision flags bit-exact; waypoints within
1e-5 rad (the implementation is bit-exact by the numerics contract, DESIGN.md §3,
so paths are compared for exact equality and the 1e-5 tolerance is the contract).
"""
import json
import os

import numpy as np
import pytest

from rbe550_final_project_amd import _abi, model, scenes

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
WAYPOINT_TOL = 1e-5


def _wl(name):
    return json.load(open(os.path.join(GOLD, "workloads", name + ".json")))


def _uniform(n, seed):
    rng = np.random.default_rng(seed)
    return (model.Q_LO + (model.Q_HI - model.Q_LO) * rng.random((n, 9))).astype(np.float32)


def _near(q0, n, seed, sigma=0.3):
    rng = np.random.default_rng(seed)
    q = np.asarray(q0)[None, :] + rng.normal(0, sigma, (n, 9))
    return np.clip(q, model.Q_LO, model.Q_HI).astype(np.float32)


SCENES = {
    "empty": scenes.Scene(),
    "goal1": scenes.goal1_scattered(0),
    "goal3": scenes.goal3_tallest(),
    "goal4_yawed": scenes.Scene.from_json(_wl("goal4_pentagon_10box")["queries"][14]["scene"]),
    "clutter64": scenes.Scene.from_json(_wl("clutter64")["queries"][0]["scene"]),
}


def _both(gpu_ctx, oracle_lib, sc, attached=-1):
    o = oracle_lib.OracleScene()
    o.set_scene(sc.boxes, sc.plane_z, sc.base)
    o.set_attached(attached)
    gpu_ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
    gpu_ctx.set_attached(attached)
    return o


@pytest.mark.parametrize("grid", ["auto", "0", "1"])
@pytest.mark.parametrize("name", list(SCENES))
def test_validity_flags_bit_exact(gpu_ctx, oracle_lib, name, grid, monkeypatch):
    """Both box broad phases (cluster AABBs, axis grid; RBE_SCENE_GRID forces one)
    must give the oracle's flags."""
    sc = SCENES[name]
    if grid != "auto":
        monkeypatch.setenv("RBE_SCENE_GRID", grid)
    o = _both(gpu_ctx, oracle_lib, sc)
    q = np.concatenate([_uniform(65536, 1), _near(model.SAFE_HOME, 65536, 2)])
    g = gpu_ctx.check_states(q)
    c = o.check_states(q)
    assert g.dtype == np.uint8 and set(np.unique(g)) <= {0, 1}
    mism = np.nonzero(g != c)[0]
    assert mism.size == 0, f"{mism.size} mismatches, first {q[mism[:3]]}"
    assert 0.02 < g.mean() < 0.98


def _quadrant_bound_states(n, seed):
    """States whose joint angles sit within 64 floats of a quadrant bound of the
    sin / cos reduction (odd multiples of pi/4) inside the limits, fingers uniform."""
    rng = np.random.default_rng(seed)
    q = _uniform(n, seed + 1)
    for j in range(7):
        bounds = [m * np.pi / 4 for m in range(-7, 8, 2) if model.Q_LO[j] < m * np.pi / 4 < model.Q_HI[j]]
        b = np.array(bounds, dtype=np.float32)[rng.integers(0, len(bounds), n)]
        steps = rng.integers(-64, 65, n)
        v = b.view(np.int32).astype(np.int64) + steps * np.where(b < 0, -1, 1)   # (same-sign floats)
        q[:, j] = v.astype(np.int32).view(np.float32)
    return q


@pytest.mark.parametrize("name", list(SCENES))
def test_validity_flags_bit_exact_large(gpu_ctx, oracle_lib, name):
    """The bench's kernel (one-wave k_validity: launches above 2^17 states) on 2^22
    uniform states and 2^20 states with every joint within 64 floats of a sin / cos
    quadrant bound, every flag against the oracle's (the round-5 quadrant bug changed
    flags of a few uniform states per 2^24)."""
    sc = SCENES[name]
    o = _both(gpu_ctx, oracle_lib, sc)
    q = np.concatenate([_uniform(1 << 22, 21), _quadrant_bound_states(1 << 20, 22)])
    g = gpu_ctx.check_states(q)
    c = o.check_states(q, threads=16)
    mism = np.nonzero(g != c)[0]
    assert mism.size == 0, f"{mism.size} mismatches, first {q[mism[:3]].tolist()}"


def test_validity_with_attached_box(gpu_ctx, oracle_lib):
    wl = _wl("goal3_tallest_10box")
    for qd in [x for x in wl["queries"] if x["attached"] >= 0][:3]:
        sc = scenes.Scene.from_json(qd["scene"])
        o = _both(gpu_ctx, oracle_lib, sc, qd["attached"])
        q = _near(qd["start"], 32768, 3, 0.2)
        assert np.array_equal(gpu_ctx.check_states(q), o.check_states(q))


def test_golden_flag_fixtures(gpu_ctx, oracle_lib):
    """Committed flag vectors (tests/golden/flags_*.npz, seed 0x5EED) — the GPU must
    reproduce them exactly."""
    files = sorted(f for f in os.listdir(GOLD) if f.startswith("flags_") and f.endswith(".npz"))
    assert files, "no golden flag fixtures"
    for f in files:
        d = np.load(os.path.join(GOLD, f), allow_pickle=False)
        sc = scenes.Scene.from_json(json.loads(str(d["scene"])))
        gpu_ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
        gpu_ctx.set_attached(int(d["attached"]))
        assert np.array_equal(gpu_ctx.check_states(d["q"]), d["flags"]), f


def test_large_batch_full_size_properties(gpu_ctx, oracle_lib):
    """4M-state batch (bench size): deterministic across launches, and a strided
    subsample equals the oracle."""
    sc = SCENES["goal3"]
    o = _both(gpu_ctx, oracle_lib, sc)
    q = _uniform(1 << 22, 7)
    a = gpu_ctx.check_states(q)
    b = gpu_ctx.check_states(q)
    assert np.array_equal(a, b)
    sub = slice(0, None, 97)
    assert np.array_equal(a[sub], o.check_states(q[sub]))


def test_edge_flags_bit_exact(gpu_ctx, oracle_lib):
    sc = SCENES["goal1"]
    o = _both(gpu_ctx, oracle_lib, sc)
    rng = np.random.default_rng(4)
    qa = _near(model.SAFE_HOME, 4096, 5, 0.4).astype(np.float64)
    qb = qa + rng.normal(0, 0.6, qa.shape)
    qb = np.clip(qb, model.Q_LO, model.Q_HI)
    res = 0.01 * model.max_extent()
    g = gpu_ctx.check_edges(qa, qb, res)
    c = o.check_edges(qa, qb, res)
    assert np.array_equal(g, c)
    assert 0.05 < g.mean() < 0.95
    # zero-length and very long edges
    g2 = gpu_ctx.check_edges(qa[:8], qa[:8], res)
    assert np.array_equal(g2, o.check_edges(qa[:8], qa[:8], res))


def test_contacts_match_oracle(gpu_ctx, oracle_lib):
    sc = SCENES["goal1"]
    o = _both(gpu_ctx, oracle_lib, sc)
    q = _near(model.SAFE_HOME, 200, 9, 0.5).astype(np.float64)
    for x in q:
        assert sorted(gpu_ctx.contacts(x)) == sorted(o.contacts(x))


def test_f64_device_numerics(gpu_ctx):
    """sqrt / div / ceil / f64->f32 on the device are IEEE correctly rounded (the
    planner's steering and segment counts depend on it)."""
    rng = np.random.default_rng(1)
    x = np.concatenate([rng.random(100000) * 20.0, rng.random(1000) * 1e-6, [0.0, 1.0, 2.0, 0.13037 * 3]])
    out = gpu_ctx.selftest_f64(x)
    assert np.array_equal(out[:, 0], np.sqrt(np.abs(x)))
    assert np.array_equal(out[:, 1], 0.13037 / np.where(x == 0, 1.0, x))
    assert np.array_equal(out[:, 2], np.ceil(x * 7.0))
    assert np.array_equal(out[:, 3], x.astype(np.float32).astype(np.float64))


def _ulps_around(v, k):
    f = np.float32(v)
    out = [f]
    lo = hi = f
    for _ in range(k):
        lo, hi = np.nextafter(lo, np.float32(-np.inf)), np.nextafter(hi, np.float32(np.inf))
        out += [lo, hi]
    return out


def test_sincos_quadrant_bounds(gpu_ctx, oracle_lib):
    """The forward kinematics' joint sin / cos (rp_math.h rp_sincos) equal the
    oracle's ro_sincos bit for bit, on 64 floats either side of every quadrant
    boundary (odd multiples of pi/4) in the joints' range and on 200,000 uniform
    angles. The float just below pi/4 once gave a negated sin on the device (the
    compiler rounded the quadrant's y + 0.5 differently from the reduction's): a
    clutter64 edge flag differed from the oracle's (tests/test_gpu_edges.py seed 7)."""
    xs = []
    for m in range(-7, 8, 2):
        xs += _ulps_around(m * np.pi / 4, 64)
    rng = np.random.default_rng(3)
    xs += list((rng.random(200000) * 6.0 - 3.0).astype(np.float32))
    x = np.array(xs, dtype=np.float32)
    out = gpu_ctx.selftest_f64(x.astype(np.float64))
    ref = np.array([oracle_lib.sincos(v) for v in x], dtype=np.float32)
    bad = np.nonzero((out[:, 4].astype(np.float32) != ref[:, 0]) | (out[:, 5].astype(np.float32) != ref[:, 1]))[0]
    assert bad.size == 0, f"{bad.size} sin / cos differ, first at x = {float(x[bad[0]])!r}"


def test_state_at_quadrant_bound(gpu_ctx, oracle_lib):
    """The state of that edge (joint 0 at the float just below pi/4): flags and
    contacts equal the oracle's."""
    sc = scenes.Scene.from_json(json.load(open(os.path.join(GOLD, "workloads", "clutter64.json")))["queries"][0]["scene"])
    o = _both(gpu_ctx, oracle_lib, sc)
    q = np.array([0.7853981256484985, 0.7177550196647644, 0.42281287908554077, -2.4574007987976074,
                  0.8535553216934204, 0.8303852081298828, -2.0884807109832764, 0.032658882439136505,
                  0.03345468267798424], dtype=np.float32)
    assert gpu_ctx.check_states(q[None])[0] == o.check_states(q[None])[0] == 1
    assert sorted(gpu_ctx.contacts(q.astype(np.float64))) == sorted(o.contacts(q.astype(np.float64))) == []


PLAN_CASES = [("goal1_scattered_6box", 7), ("single_pick_place_5box", 0), ("single_pick_place_5box", 1), ("goal3_tallest_10box", 2),
              ("goal3_tallest_10box", 5), ("goal4_pentagon_10box", 2), ("goal4_pentagon_10box", 14),
              ("clutter64", 0)]


@pytest.mark.parametrize("wl,qi", PLAN_CASES)
@pytest.mark.parametrize("batch,seed,batch_min", [(1, 3, 0), (64, 11, 0), (4096, 5, 0), (16384, 8, 8192)])
@pytest.mark.parametrize("speculate", ["1", "0"])
def test_plan_parity(gpu_ctx, oracle_lib, wl, qi, batch, seed, batch_min, speculate, monkeypatch):
    """Speculative (one edge launch per iteration) and two-phase single-rank
    iterations build the oracle's trees; batch_min 8192 > FUSE_MAX starts on the
    multi-kernel accept path."""
    monkeypatch.setenv("RBE_PLAN_SPECULATE", speculate)
    q = _wl(wl)["queries"][qi]
    sc = scenes.Scene.from_json(q["scene"])
    o = _both(gpu_ctx, oracle_lib, sc, q["attached"])
    p = _abi.make_params(seed=seed, batch=batch, batch_min=batch_min, n_waypoints=150, timeout_s=60, straight_first=False)
    ref, st_ref, stats_ref = o.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
    path, st = gpu_ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
    gst = gpu_ctx.stats()
    assert st == st_ref == _abi.STATUS_EXACT
    assert path.shape == ref.shape == (150, 9)
    assert np.max(np.abs(path - ref)) <= WAYPOINT_TOL
    assert np.array_equal(path, ref)
    assert (gst["start_tree_size"], gst["goal_tree_size"], gst["iterations"]) == \
        (stats_ref["start_tree_size"], stats_ref["goal_tree_size"], stats_ref["iterations"])


@pytest.mark.parametrize("wl,qi", PLAN_CASES)
@pytest.mark.parametrize("chunk,growth,speculate", [("-1", "", "1"), ("64", "", "1"), ("1000", "2", "1"),
                                                    ("4096", "", "0"), ("256", "3", "0"), ("", "", "1")])
def test_plan_parity_sub_batches(gpu_ctx, oracle_lib, wl, qi, chunk, growth, speculate, monkeypatch):
    """Iterations of 16,384 samples (batch_min = batch) run as ordered sub-batches
    (rp_plan_params.chunk: first sub-batch, x growth after) that end after the one
    holding the first REACHED sample; "-1" = the whole iteration in one launch
    sequence. The oracle appends up to the winning sample whatever the split: the
    trees and paths are the same for every sub-batching."""
    monkeypatch.setenv("RBE_PLAN_SPECULATE", speculate)
    if chunk:
        monkeypatch.setenv("RBE_PLAN_CHUNK", chunk)
    if growth:
        monkeypatch.setenv("RBE_CHUNK_GROWTH", growth)
    q = _wl(wl)["queries"][qi]
    sc = scenes.Scene.from_json(q["scene"])
    o = _both(gpu_ctx, oracle_lib, sc, q["attached"])
    p = _abi.make_params(seed=qi + 7, batch=16384, batch_min=16384, n_waypoints=150, timeout_s=60,
                         straight_first=False)
    ref, st_ref, stats_ref = o.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
    path, st = gpu_ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
    gst = gpu_ctx.stats()
    assert st == st_ref == _abi.STATUS_EXACT
    assert np.array_equal(path, ref)
    assert (gst["start_tree_size"], gst["goal_tree_size"], gst["iterations"]) == \
        (stats_ref["start_tree_size"], stats_ref["goal_tree_size"], stats_ref["iterations"])
    # samples processed: whole sub-batches up to the solving one, never past the schedule
    assert 0 < gst["samples"] <= stats_ref["samples"]


@pytest.mark.parametrize("wl,qi", PLAN_CASES[:5])
@pytest.mark.parametrize("batch,seed", [(64, 11), (4096, 5)])
@pytest.mark.parametrize("knob", ["RBE_FUSE_INIT", "RBE_STRAIGHT_RIDE"])
def test_plan_parity_latency_paths_off(gpu_ctx, oracle_lib, wl, qi, batch, seed, knob, monkeypatch):
    """The plan-latency shortcuts turned off, one at a time: RBE_FUSE_INIT=0 runs the
    prologue as its own launch (k_plan_init) instead of block 0 of the first
    speculative front; RBE_STRAIGHT_RIDE=0 leaves the straight edge out of the first
    edge launch, so a solving iteration runs the shortcut stage's launches instead of
    finishing the plan itself. Same trees, same paths (the default runs them on)."""
    monkeypatch.setenv(knob, "0")
    q = _wl(wl)["queries"][qi]
    sc = scenes.Scene.from_json(q["scene"])
    o = _both(gpu_ctx, oracle_lib, sc, q["attached"])
    p = _abi.make_params(seed=seed, batch=batch, n_waypoints=150, timeout_s=60, straight_first=False)
    ref, st_ref, stats_ref = o.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
    path, st = gpu_ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
    gst = gpu_ctx.stats()
    assert st == st_ref == _abi.STATUS_EXACT
    assert np.array_equal(path, ref)
    assert (gst["start_tree_size"], gst["goal_tree_size"], gst["iterations"]) == \
        (stats_ref["start_tree_size"], stats_ref["goal_tree_size"], stats_ref["iterations"])


@pytest.mark.parametrize("wl,qi", PLAN_CASES)
@pytest.mark.parametrize("batch,seed,batch_min", [(64, 11, 0), (16384, 8, 8192)])
def test_plan_parity_packed_edges(gpu_ctx, oracle_lib, wl, qi, batch, seed, batch_min, monkeypatch):
    """Two-phase iterations whose connect launches are work-compacted
    (k_edges_packed forced on): same trees and paths as the oracle."""
    monkeypatch.setenv("RBE_PLAN_SPECULATE", "0")
    monkeypatch.setenv("RBE_EDGE_PACKED", "1")
    q = _wl(wl)["queries"][qi]
    sc = scenes.Scene.from_json(q["scene"])
    o = _both(gpu_ctx, oracle_lib, sc, q["attached"])
    p = _abi.make_params(seed=seed, batch=batch, batch_min=batch_min, n_waypoints=150, timeout_s=60, straight_first=False)
    ref, st_ref, stats_ref = o.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
    path, st = gpu_ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
    assert st == st_ref == _abi.STATUS_EXACT
    assert np.array_equal(path, ref)
    gst = gpu_ctx.stats()
    assert (gst["start_tree_size"], gst["goal_tree_size"]) == (stats_ref["start_tree_size"],
                                                                stats_ref["goal_tree_size"])


@pytest.mark.parametrize("simplify,rng,dev_max", [(0, 0.3, ""), (1, 0.3, ""), (2, 0.3, ""), (1, 0.15, ""),
                                                   (1, 0.15, "2"), (2, 0.3, "2")])
def test_plan_parity_hard_iterations(gpu_ctx, oracle_lib, simplify, rng, dev_max, monkeypatch):
    """Many iterations with a small range (more nodes, more NN work, long raw paths)
    and every simplification level: path equality. dev_max "2" moves the
    simplification to the host-driven fallback (raw paths > RBE_SIMPLIFY_DEVICE_MAX)."""
    if dev_max:
        monkeypatch.setenv("RBE_SIMPLIFY_DEVICE_MAX", dev_max)
    q = _wl("goal4_pentagon_10box")["queries"][8]
    sc = scenes.Scene.from_json(q["scene"])
    o = _both(gpu_ctx, oracle_lib, sc, q["attached"])
    p = _abi.make_params(seed=21, batch=256, range_=rng, n_waypoints=0, timeout_s=120, straight_first=False)
    p.simplify = simplify
    ref, st_ref, s_ref = o.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
    path, st = gpu_ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
    assert st == st_ref
    assert np.array_equal(path, ref)
    gs = gpu_ctx.stats()
    assert gs["start_tree_size"] == s_ref["start_tree_size"]
    assert gs["path_states_raw"] == s_ref["path_states_raw"]
    assert gs["path_states_simplified"] == s_ref["path_states_simplified"]


@pytest.mark.parametrize("wl,qi", [("clutter64", 0), ("goal3_tallest_10box", 20)])
@pytest.mark.parametrize("dev_max", ["", "2"])
def test_plan_parity_smoothing(gpu_ctx, oracle_lib, wl, qi, dev_max, monkeypatch):
    """Queries whose simplified path keeps corners, so the B-spline rounds change
    it (oracle: level 1 shorter than level 2); device and host-driven paths."""
    if dev_max:
        monkeypatch.setenv("RBE_SIMPLIFY_DEVICE_MAX", dev_max)
    q = _wl(wl)["queries"][qi]
    sc = scenes.Scene.from_json(q["scene"])
    o = _both(gpu_ctx, oracle_lib, sc, q["attached"])
    lens = {}
    for level in (2, 1):
        p = _abi.make_params(seed=qi, batch=64, range_=0.15, n_waypoints=0, timeout_s=120, straight_first=False)
        p.simplify = level
        ref, st_ref, _ = o.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
        path, st = gpu_ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
        assert st == st_ref == _abi.STATUS_EXACT
        assert np.array_equal(path, ref)
        lens[level] = float(np.sum(np.linalg.norm(np.diff(path, axis=0), axis=1)))
    assert lens[1] < lens[2]


@pytest.mark.parametrize("max_iters,simplify", [(1, 0), (4, 1), (8, 2)])
def test_plan_parity_approximate(gpu_ctx, oracle_lib, max_iters, simplify):
    """Unsolved within the iteration cap: APPROXIMATE status and the same path to the
    start-tree node closest to the goal (and its simplification)."""
    from test_oracle_planner import WALLS, walled_query
    sc = scenes.Scene(boxes=WALLS)
    o = _both(gpu_ctx, oracle_lib, sc)
    start, goal = walled_query()
    p = _abi.make_params(seed=1, batch=64, max_iters=max_iters, range_=0.3, timeout_s=60, n_waypoints=100, straight_first=False)
    p.simplify = simplify
    ref, st_ref, s_ref = o.plan(start, goal, model.Q_LO, model.Q_HI, p)
    path, st = gpu_ctx.plan(start, goal, model.Q_LO, model.Q_HI, p)
    assert st == st_ref == _abi.STATUS_APPROXIMATE
    assert np.array_equal(path, ref)
    assert gpu_ctx.stats()["start_tree_size"] == s_ref["start_tree_size"]


def test_plan_invalid_start_goal(gpu_ctx, oracle_lib):
    gpu_ctx.set_scene([])
    gpu_ctx.set_attached(-1)
    p = _abi.make_params(seed=0, batch=64, max_iters=3, straight_first=False)
    bad = model.SAFE_HOME.copy()
    bad[7:] = 0.04
    _, st = gpu_ctx.plan(bad, model.SAFE_HOME, model.Q_LO, model.Q_HI, p)
    assert st == _abi.STATUS_INVALID_START
    ok = model.SAFE_HOME.copy()
    ok[7:] = np.float32(0.04)
    _, st = gpu_ctx.plan(ok, bad, model.Q_LO, model.Q_HI, p)
    assert st == _abi.STATUS_INVALID_GOAL


def _hand_built_cases(oracle_lib):
    """SURVEY.md §4 item 2 on the GPU: capsule end touching / missing a box face and
    a yawed box corner (±2e-4 m), a closed grasp with the exemption on / partial /
    off, the base against the plane with and without the 1 cm raise."""
    import franka_np as F
    o = oracle_lib.OracleScene()
    caps = o.fk_capsules(model.SAFE_HOME)
    a, b = caps[9]
    end = b if b[1] > a[1] else a
    r, h = 0.04, 0.02
    home = model.SAFE_HOME.copy()
    home[7:] = np.float32(0.04)
    cases = []
    for gap in (2e-4, -2e-4):
        cases.append(([((float(end[0]), float(end[1] + r + h + gap), float(end[2])), (h, h, h), 0.0)],
                      (0.0, 0.0, 0.01), -1, _abi.ATTACH_EXEMPT_MASK, model.SAFE_HOME, 1 if gap > 0 else 0))
        cases.append(([((float(end[0]), float(end[1] + r + h * np.sqrt(2) + gap), float(end[2])), (h, h, h),
                        np.pi / 4)], (0.0, 0.0, 0.01), -1, _abi.ATTACH_EXEMPT_MASK, model.SAFE_HOME,
                      1 if gap > 0 else 0))
    q = model.SAFE_HOME.copy()
    q[7:] = 0.0
    R, p = F.hand_pose(q, model.BASE_POS)
    c = p + R @ np.array([0, 0, 0.0584 + 0.03])
    grasp = [(tuple(map(float, c)), (0.02, 0.02, 0.02), 0.0)]
    cases += [(grasp, (0.0, 0.0, 0.01), -1, _abi.ATTACH_EXEMPT_MASK, q, 0),
              (grasp, (0.0, 0.0, 0.01), 0, _abi.ATTACH_EXEMPT_MASK, q, 1),
              (grasp, (0.0, 0.0, 0.01), 0, 1 << 9, q, 0),
              ([], (0.0, 0.0, 0.0), -1, _abi.ATTACH_EXEMPT_MASK, home, 0),
              ([], (0.0, 0.0, 0.01), -1, _abi.ATTACH_EXEMPT_MASK, home, 1)]
    return cases


def test_hand_built_collision_cases(gpu_ctx, oracle_lib):
    for boxes, base, att, mask, q, expect in _hand_built_cases(oracle_lib):
        o = oracle_lib.OracleScene()
        o.set_scene(boxes, 0.0, base)
        o.set_attached(att, mask)
        gpu_ctx.set_scene(boxes, 0.0, base)
        gpu_ctx.set_attached(att, mask)
        qq = np.asarray(q, dtype=np.float32)[None, :]
        assert o.check_states(qq)[0] == expect
        assert gpu_ctx.check_states(qq)[0] == expect
        assert sorted(gpu_ctx.contacts(np.asarray(q, dtype=np.float64))) == sorted(o.contacts(q))


@pytest.mark.parametrize("wl", ["goal1_scattered_6box", "goal3_tallest_10box", "goal4_pentagon_10box", "clutter64",
                                "single_pick_place_5box", "goal4_pentagon_ring"])
def test_plan_parity_rrt_forced_every_query(gpu_ctx, oracle_lib, wl):
    """RRT-Connect forced on every query of the workload (the C1 / C3 RRT-forced
    bench legs): queries whose straight edge holds finish inside the solving
    iteration (the ride-along), the others run the shortcut / smoothing launches;
    every path, status, tree and iteration count equals the oracle's."""
    for qi, q in enumerate(_wl(wl)["queries"]):
        sc = scenes.Scene.from_json(q["scene"])
        o = _both(gpu_ctx, oracle_lib, sc, q["attached"])
        p = _abi.make_params(seed=qi, batch=4096, n_waypoints=150, timeout_s=60, straight_first=False)
        ref, st_ref, stats_ref = o.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
        path, st = gpu_ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
        g = gpu_ctx.stats()
        assert st == st_ref == _abi.STATUS_EXACT, (wl, qi)
        assert np.array_equal(path, ref), (wl, qi)
        assert (g["start_tree_size"], g["goal_tree_size"], g["iterations"]) == \
            (stats_ref["start_tree_size"], stats_ref["goal_tree_size"], stats_ref["iterations"]), (wl, qi)


@pytest.mark.parametrize("wl", ["goal1_scattered_6box", "goal3_tallest_10box", "goal4_pentagon_10box", "clutter64",
                                "single_pick_place_5box", "goal4_pentagon_ring"])
def test_plan_parity_straight_first(gpu_ctx, oracle_lib, wl):
    """Default plans (straight edge first): every query of the workload gives the
    oracle's status, path and iteration count (straight edge valid: no iteration;
    invalid: the RRT-Connect run)."""
    for qi, q in enumerate(_wl(wl)["queries"]):
        sc = scenes.Scene.from_json(q["scene"])
        o = _both(gpu_ctx, oracle_lib, sc, q["attached"])
        p = _abi.make_params(seed=qi, batch=4096, n_waypoints=150, timeout_s=60)
        ref, st_ref, stats_ref = o.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
        path, st = gpu_ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
        assert st == st_ref == _abi.STATUS_EXACT, (wl, qi)
        assert np.array_equal(path, ref), (wl, qi)
        assert gpu_ctx.stats()["iterations"] == stats_ref["iterations"], (wl, qi)


def test_plan_straight_first_endpoint_status(gpu_ctx, oracle_lib):
    """Invalid start / goal are reported through the straight-first launch as by
    the RRT path (planning.py PlannerInputStates semantics)."""
    sc = SCENES["goal3"]
    o = _both(gpu_ctx, oracle_lib, sc)
    home = np.array(model.SAFE_HOME, dtype=np.float64)
    home[7:] = 0.035       # inside the float32 finger bound
    bad = home.copy()
    bad[1] = 1.7           # shoulder down: the arm goes through the table
    bad[3] = -0.2
    assert o.check_states(home[None].astype(np.float32))[0]
    assert not o.check_states(bad[None].astype(np.float32))[0]
    p = _abi.make_params(seed=0, batch=256, n_waypoints=150, timeout_s=10)
    for s, g, want in ((bad, home, _abi.STATUS_INVALID_START), (home, bad, _abi.STATUS_INVALID_GOAL)):
        _, st_ref, _ = o.plan(s, g, model.Q_LO, model.Q_HI, p)
        _, st = gpu_ctx.plan(s, g, model.Q_LO, model.Q_HI, p)
        assert st == st_ref == want


@pytest.mark.parametrize("name", ["empty", "goal3", "clutter64"])
@pytest.mark.parametrize("mode", ["wide", "one_per_wave"])
def test_validity_flags_outside_joint_limits(gpu_ctx, oracle_lib, name, mode):
    """Waves with states outside the joint limits test the never pairs (rp_model.h
    NEVER_PAIRS) that in-limit waves skip: flags stay bit-exact either way. "wide":
    states from the limits widened by 0.6 rad / 0.02 m; "one_per_wave": one
    out-of-limit state in every 64."""
    sc = SCENES[name]
    o = _both(gpu_ctx, oracle_lib, sc)
    rng = np.random.default_rng(17)
    n = 1 << 17
    pad = np.array([0.6] * 7 + [0.02] * 2)
    if mode == "wide":
        q = (model.Q_LO - pad + (model.Q_HI - model.Q_LO + 2 * pad) * rng.random((n, 9))).astype(np.float32)
    else:
        q = _uniform(n, 17)
        q[::64] = (model.Q_HI + pad * rng.random((n // 64, 9))).astype(np.float32)
    g = gpu_ctx.check_states(q)
    c = o.check_states(q)
    assert np.array_equal(g, c), f"{(g != c).sum()} flags differ"


@pytest.mark.parametrize("name", ["goal1", "goal3", "goal4_yawed", "clutter64"])
@pytest.mark.parametrize("n", [4097, 8192, 65536, 65537, 131072, 131073])
def test_validity_flags_every_launch_kernel(gpu_ctx, oracle_lib, name, n):
    """The launch sizes at the kernels' boundaries: <= 4,096 states the lane-group
    kernel, up to 65,536 the three-role split kernel, up to 131,072 the two-role one,
    above it the one-wave k_validity (rp_lib.hip launch_validity). Uniform states,
    states near the home pose, every 64th state outside the joint limits, box 0
    attached:
    flags bit-exact."""
    sc = SCENES[name]
    o = _both(gpu_ctx, oracle_lib, sc, attached=0)
    rng = np.random.default_rng(n)
    q = _uniform(n, n + 1)
    q[: n // 10] = _near(model.SAFE_HOME, n // 10, n + 2, sigma=0.5)   # a tenth near the home pose
    pad = np.array([0.6] * 7 + [0.02] * 2)
    q[::64] = (model.Q_HI + pad * rng.random((len(q[::64]), 9))).astype(np.float32)
    g = gpu_ctx.check_states(q)
    r = o.check_states(q)
    assert np.array_equal(g, r), f"{(g != r).sum()} of {n} flags differ"
