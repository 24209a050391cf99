"""GPU edge cases of the C-ABI (SURVEY.md §4 style: empty and ragged inputs, maximum
sizes, degenerate edges and plans, argument errors), each against the CPU oracle."""
import ctypes as C

import numpy as np
import pytest

from rbe550_final_project_amd import _abi, model, scenes
from rbe550_final_project_amd.native import NativeError, load

pytestmark = pytest.mark.gpu


def _pair(gpu_ctx, oracle_lib, sc, attached=-1):
    o = oracle_lib.OracleScene()
    o.set_scene(sc.boxes, sc.plane_z, sc.base)
    o.set_attached(attached)
    gpu_ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
    gpu_ctx.set_attached(attached)
    return o


@pytest.mark.parametrize("n", [0, 1, 63, 65, 127, 1000, 4097])
def test_ragged_state_counts(gpu_ctx, oracle_lib, n):
    """State counts that are not multiples of the 64-lane wave (and zero)."""
    o = _pair(gpu_ctx, oracle_lib, scenes.goal3_tallest())
    rng = np.random.default_rng(n)
    q = (model.Q_LO + (model.Q_HI - model.Q_LO) * rng.random((n, 9))).astype(np.float32)
    g = gpu_ctx.check_states(q)
    assert g.shape == (n,)
    assert np.array_equal(g, o.check_states(q))


def test_max_boxes_scene(gpu_ctx, oracle_lib):
    """64 boxes (MAX_BOXES) with yaw and an attached box: flags bit-exact."""
    rng = np.random.default_rng(64)
    boxes = [(tuple(rng.uniform([0.2, -0.6, 0.02], [0.9, 0.6, 0.7])), tuple(rng.uniform(0.01, 0.06, 3)),
              float(rng.uniform(-np.pi, np.pi))) for i in range(64)]
    sc = scenes.Scene(boxes=boxes)
    o = _pair(gpu_ctx, oracle_lib, sc, attached=5)
    q = (model.Q_LO + (model.Q_HI - model.Q_LO) * np.random.default_rng(1).random((50000, 9))).astype(np.float32)
    assert np.array_equal(gpu_ctx.check_states(q), o.check_states(q))


def test_too_many_boxes_rejected(gpu_ctx):
    boxes = [((0.5, 0.0, 0.02 + 0.05 * i), (0.02, 0.02, 0.02), 0.0) for i in range(65)]
    with pytest.raises(NativeError):
        gpu_ctx.set_scene(boxes)


def test_zero_length_and_long_edges(gpu_ctx, oracle_lib):
    """Zero-length edges (only the endpoint is checked) and bound-to-bound edges
    (the longest in the space): edge flags bit-exact."""
    o = _pair(gpu_ctx, oracle_lib, scenes.goal3_tallest())
    rng = np.random.default_rng(3)
    a = model.Q_LO + (model.Q_HI - model.Q_LO) * rng.random((300, 9))
    b = a.copy()
    b[100:200] = model.Q_LO + (model.Q_HI - model.Q_LO) * rng.random((100, 9))
    b[200:] = np.where(rng.random((100, 9)) < 0.5, model.Q_LO, model.Q_HI)
    a[200:] = np.where(b[200:] == model.Q_LO, model.Q_HI, model.Q_LO)
    res = 0.01 * model.max_extent()
    assert np.array_equal(gpu_ctx.check_edges(a, b, res), o.check_edges(a, b, res))
    assert np.array_equal(gpu_ctx.check_edges(a[:0], b[:0], res), np.zeros(0, np.uint8))


@pytest.mark.parametrize("straight", [True, False])
def test_plan_start_equals_goal(gpu_ctx, oracle_lib, straight):
    """start == goal: an exact solution with the oracle's path."""
    o = _pair(gpu_ctx, oracle_lib, scenes.goal3_tallest())
    s = np.array(model.SAFE_HOME)
    s[7:] = 0.035
    p = _abi.make_params(seed=4, batch=64, n_waypoints=150, timeout_s=10, straight_first=straight)
    ref, st_ref, _ = o.plan(s, s, model.Q_LO, model.Q_HI, p)
    path, st = gpu_ctx.plan(s, s, model.Q_LO, model.Q_HI, p)
    assert st == st_ref == _abi.STATUS_EXACT
    assert np.array_equal(path, ref) and len(path) == 150


def test_plan_out_of_bounds_goal(gpu_ctx, oracle_lib):
    """A goal outside the bounds is INVALID_GOAL (OMPL PlannerInputStates), with and
    without the straight-first check."""
    o = _pair(gpu_ctx, oracle_lib, scenes.goal3_tallest())
    s = np.array(model.SAFE_HOME)
    s[7:] = 0.035
    g = s.copy()
    g[0] = model.Q_HI[0] + 0.1
    for straight in (True, False):
        p = _abi.make_params(seed=1, batch=64, n_waypoints=150, timeout_s=10, straight_first=straight)
        st_gpu = gpu_ctx.plan(s, g, model.Q_LO, model.Q_HI, p)[1]
        st_cpu = o.plan(s, g, model.Q_LO, model.Q_HI, p)[1]
        assert st_gpu == st_cpu == _abi.STATUS_INVALID_GOAL


def test_argument_errors(gpu_ctx):
    """Negative counts and null buffers return errors, not crashes."""
    L = load()
    out = (C.c_uint8 * 4)()
    assert L.rp_check_states(gpu_ctx._h, None, -1, out) < 0
    assert L.rp_check_states(gpu_ctx._h, None, 4, out) < 0
    assert L.rp_check_edges(gpu_ctx._h, None, None, 4, 0.1, out) < 0
    n, st = C.c_int32(0), C.c_int32(0)
    p = _abi.make_params()
    assert L.rp_plan(gpu_ctx._h, None, None, None, None, C.byref(p), None, 0, C.byref(n), C.byref(st)) < 0


@pytest.mark.parametrize("base", [(0.0, 0.0, 0.01), (0.02, -0.03, 0.01), (0.0, 0.0, 0.0), (0.0, 0.0, 0.0100001)])
@pytest.mark.parametrize("name", ["goal3", "clutter64"])
def test_validity_robot_base(gpu_ctx, oracle_lib, base, name):
    """The reference's base (0, 0, 0.01) runs kernels with the base folded in as a
    constant (rp_math.h BASE_FIXED); any other base the general ones: flags
    bit-exact for both."""
    import json
    import os
    if name == "goal3":
        sc = scenes.goal3_tallest()
    else:
        gold = os.path.join(os.path.dirname(__file__), "golden", "workloads", "clutter64.json")
        sc = scenes.Scene.from_json(json.load(open(gold))["queries"][0]["scene"])
    sc.base = base
    o = _pair(gpu_ctx, oracle_lib, sc)
    q = (model.Q_LO + (model.Q_HI - model.Q_LO) * np.random.default_rng(8).random((1 << 17, 9))).astype(np.float32)
    assert np.array_equal(gpu_ctx.check_states(q), o.check_states(q))


def _clusters(rng, n_clusters, jitter, bases=None):
    """n_clusters groups of 64 near-identical states (one wave each): whenever a
    broad phase passes for one lane it passes for all 64 at once, so every queue
    batch is a full wave (a 64-item batch after a pop pass). bases: the
    cluster centres to cycle through (default uniform states)."""
    if bases is None:
        base = model.Q_LO + (model.Q_HI - model.Q_LO) * rng.random((n_clusters, 1, 9))
    else:
        base = np.asarray(bases, dtype=np.float64)[np.arange(n_clusters) % len(bases)][:, None, :]
    q = base + jitter * rng.standard_normal((n_clusters, 64, 9))
    return np.clip(q, model.Q_LO, model.Q_HI).reshape(-1, 9).astype(np.float32)


_BASES = {}


def _contact_bases(o, key, kind, n=256, seed=5):
    """Up to n states whose contacts (the oracle's rp_state_contacts) include a self
    pair (kind "self") or a box (kind "box"): cluster centres whose waves queue the
    corresponding narrow phases in every lane at once. Half of the result is uniform
    states, so both verdicts occur in every launch."""
    if (key, kind) in _BASES:
        return _BASES[(key, kind)]
    rng = np.random.default_rng(seed)
    found = []
    for _ in range(40):
        q = model.Q_LO + (model.Q_HI - model.Q_LO) * rng.random((4096, 9))
        if kind == "box":   # arm low over the table: hand / fingers among the blocks
            q[:, 1] = rng.uniform(0.2, 1.7, 4096)
            q[:, 3] = rng.uniform(-2.6, -0.8, 4096)
        for s in q:
            c = o.contacts(s)
            if (kind == "self" and any(ob <= -2 for _, ob in c)) or (kind == "box" and any(ob >= 0 for _, ob in c)):
                found.append(s)
        if len(found) >= n:
            break
    assert len(found) >= 16, f"only {len(found)} {kind}-contact states"
    found = np.array(found[:n])
    uni = model.Q_LO + (model.Q_HI - model.Q_LO) * rng.random((len(found), 9))
    out = np.empty((2 * len(found), 9))
    out[0::2], out[1::2] = found, uni
    _BASES[(key, kind)] = out
    return out


def _sat_scene(name):
    import json
    import os
    if name == "goal3":
        return scenes.goal3_tallest()
    gold = os.path.join(os.path.dirname(__file__), "golden", "workloads", "clutter64.json")
    return scenes.Scene.from_json(json.load(open(gold))["queries"][0]["scene"])


# launch sizes that select each validity kernel (rp_lib.hip launch_validity): the
# 64- and 32-lane groups, the three-role split (<= 65,536), the two-role split
# (<= 131,072) and the one-wave k_validity that bench.py times (> 131,072)
SAT_CLUSTERS = [16, 64, 1024, 2048, 4096]


@pytest.mark.parametrize("name", ["goal3", "clutter64"])
@pytest.mark.parametrize("variant", ["uniform", "self", "box"])
@pytest.mark.parametrize("jitter", [0.0, 1e-4, 2e-3])
@pytest.mark.parametrize("n_clusters", SAT_CLUSTERS)
def test_wave_saturated_queues(gpu_ctx, oracle_lib, name, variant, jitter, n_clusters):
    """Waves whose 64 states are (near-)identical: box and self-pair candidates
    arrive 64 at a time, so the narrow-phase queues take full-wave batches right
    after a pop pass — at every launch size, i.e. through every validity kernel, with
    cluster centres at uniform states, at states with a self contact, and at states
    with a box contact. Flags bit-exact (the round-3 QCAP overflow corrupted 165-3,630
    of 131,072 flags on exactly these inputs)."""
    sc = _sat_scene(name)
    o = _pair(gpu_ctx, oracle_lib, sc, attached=3)
    rng = np.random.default_rng(int(jitter * 1e5) + len(name) + 7 * n_clusters + len(variant))
    bases = None if variant == "uniform" else _contact_bases(o, name, variant)
    q = _clusters(rng, n_clusters, jitter, bases)
    g = gpu_ctx.check_states(q)
    c = o.check_states(q)
    assert np.array_equal(g, c), f"{(g != c).sum()} of {len(q)} flags differ"
    # both outcomes occur, so a corrupted hit word would show
    assert 0 < c.sum() < len(c)


@pytest.mark.parametrize("name", ["goal3", "clutter64"])
@pytest.mark.parametrize("variant", ["uniform", "self", "box"])
@pytest.mark.parametrize("jitter", [0.0, 1e-4, 2e-3])
def test_wave_saturated_edges(gpu_ctx, oracle_lib, name, variant, jitter):
    """Edges of one slot each (shorter than the resolution: only the endpoint is
    checked) whose endpoints form (near-)identical waves: the edge kernels' queues
    take full-wave batches too."""
    sc = _sat_scene(name)
    o = _pair(gpu_ctx, oracle_lib, sc, attached=3)
    rng = np.random.default_rng(int(jitter * 1e5) + len(name) + len(variant))
    bases = None if variant == "uniform" else _contact_bases(o, name, variant)
    b = _clusters(rng, 256, jitter, bases).astype(np.float64)
    a = np.clip(b + 0.02 * rng.standard_normal(b.shape), model.Q_LO, model.Q_HI)
    res = 0.01 * model.max_extent()
    ref = o.check_edges(a, b, res)
    assert np.array_equal(gpu_ctx.check_edges(a, b, res), ref)
    assert 0 < ref.sum() < len(ref)


@pytest.mark.parametrize("name", ["goal3", "clutter64"])
@pytest.mark.parametrize("variant", ["self", "box"])
@pytest.mark.parametrize("n_edges", [256, 4096])
@pytest.mark.parametrize("entry", ["host", "device"])
def test_fine_resolution_saturated_edges(gpu_ctx, oracle_lib, name, variant, n_edges, entry):
    """Short edges (0.006 rad) at a fine resolution (1e-4: 60 slots each) around
    contact states: consecutive items of an edge group are near-identical states, so
    the queues saturate inside the edge kernels; a group of 64 such edges has 60
    rounds, so rp_check_edges_device runs the loop-free kernel over rounds 0-23 and
    the grid-striding remainder over the rest, and rp_check_edges the one-lane
    loop-free kernel (4,096 edges) or the 16-lane group kernel (256 edges). Edge
    flags bit-exact."""
    import torch
    sc = _sat_scene(name)
    o = _pair(gpu_ctx, oracle_lib, sc, attached=3)
    rng = np.random.default_rng(n_edges + len(name) + len(variant))
    bases = _contact_bases(o, name, variant)
    qb = np.clip(bases[np.arange(n_edges) % len(bases)] + 2e-3 * rng.standard_normal((n_edges, 9)),
                 model.Q_LO, model.Q_HI)
    d = rng.standard_normal((n_edges, 9))
    d *= 0.006 / np.linalg.norm(d, axis=1, keepdims=True)
    qa = np.clip(qb + d, model.Q_LO, model.Q_HI)
    res = 1e-4
    ref = o.check_edges(qa, qb, res)
    if entry == "host":
        got = gpu_ctx.check_edges(qa, qb, res)
    else:
        dev = torch.device("cuda", 0)
        ta, tb = torch.from_numpy(qa).to(dev), torch.from_numpy(qb).to(dev)
        out = torch.empty(n_edges, dtype=torch.uint8, device=dev)
        gpu_ctx.check_edges_device(ta.data_ptr(), tb.data_ptr(), n_edges, res, out.data_ptr())
        torch.cuda.synchronize()
        got = out.cpu().numpy()
    assert np.array_equal(got, ref), f"{int((got != ref).sum())} of {n_edges} edge flags differ"
    assert 0 < ref.sum() < n_edges
