"""Axis-grid scenes (> 16 boxes) with the scene staged in the block's LDS
(rp_math.h SceneGrid; k_validity_gl, k_edges_units_gl and, with RBE_SCENE_LDS bit 1,
k_edges_gl, bit 2 the same over a resident grid) against the CPU oracle and against the global-memory kernels
(RBE_SCENE_LDS=0): validity flags, edge flags through the coarse-first passes and
whole plans. The staged fields are DevScene's own values and the tests are the same
arithmetic, so every result is bit for bit the same (reference: the per-state check
_is_ompl_state_valid, /root/reference/code/planning.py:209-219, and OMPL checkMotion
inside ss.solve, :190)."""
import json
import os

import numpy as np
import pytest
import torch

from rbe550_final_project_amd import model
import tilt_scenes as T
from test_gpu_configs import _check
from test_gpu_edges import _edges, _scene

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
MODES = ["0", "1", "3", "5"]


def _grid_scene(name):
    """clutter64, or its copy with tilted boxes (tests/tilt_scenes.py)."""
    return T.tilted_clutter64()[0] if name == "tilted" else _scene(name)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("n", [1000, 70000, 300000])
def test_grid_scene_flags(gpu_ctx, oracle_lib, mode, n, monkeypatch):
    """k_validity_gl at sizes past the split kernels' (131,072), the lane-group and
    split kernels below: the oracle's flags, with an attached box."""
    monkeypatch.setenv("RBE_SCENE_LDS", mode)
    sc = _scene("clutter64")
    q = json.load(open(os.path.join(GOLD, "workloads", "clutter64.json")))["queries"][0]
    rng = np.random.default_rng(17 + n)
    states = (model.Q_LO + (model.Q_HI - model.Q_LO) * rng.random((n, 9))).astype(np.float32)
    for att in (-1, q["attached"]):
        o = oracle_lib.OracleScene()
        o.set_scene(sc.boxes, sc.plane_z, sc.base)
        o.set_attached(att)
        gpu_ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
        gpu_ctx.set_attached(att)
        ref = o.check_states(states)
        got = gpu_ctx.check_states(states)
        assert np.array_equal(got, ref), f"{int((got != ref).sum())} of {n} flags differ (attached {att})"


@pytest.mark.parametrize("mode", ["0", "1"])
def test_grid_scene_flags_device_large(gpu_ctx, mode, monkeypatch):
    """2^21 states on the device: the LDS kernel's flags equal the global-memory
    kernel's (RBE_SCENE_LDS=0), and its own on a second launch."""
    monkeypatch.setenv("RBE_SCENE_LDS", mode)
    sc = _scene("clutter64")
    gpu_ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
    gpu_ctx.set_attached(-1)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(9)
    lo = torch.tensor(model.Q_LO, dtype=torch.float32, device=dev)
    hi = torch.tensor(model.Q_HI, dtype=torch.float32, device=dev)
    n = 1 << 21
    q = (lo + (hi - lo) * torch.rand((n, 9), generator=g, device=dev)).contiguous()
    f = torch.empty(n, dtype=torch.uint8, device=dev)
    gpu_ctx.check_states_device(q.data_ptr(), n, f.data_ptr())
    torch.cuda.synchronize()
    monkeypatch.setenv("RBE_SCENE_LDS", "0")
    f0 = torch.empty_like(f)
    gpu_ctx.check_states_device(q.data_ptr(), n, f0.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(f, f0)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("scene", ["clutter64", "tilted"])
@pytest.mark.parametrize("n,scale", [(2049, 1.0), (40000, 1.0), (20000, 3.0)])
@pytest.mark.parametrize("units", ["1", "0"])
def test_grid_scene_edges(gpu_ctx, oracle_lib, mode, scene, n, scale, units, monkeypatch):
    """rp_check_edges through the coarse-first passes forced on (pass 1 over its work
    list or the groups x rounds grid) and the one-pass launch: the oracle's flags under
    every RBE_SCENE_LDS mode, on clutter64 and on a tilted copy of it."""
    monkeypatch.setenv("RBE_SCENE_LDS", mode)
    monkeypatch.setenv("RBE_EDGE_UNITS", units)
    monkeypatch.setenv("RBE_EDGE_COARSE_MIN", "0")
    monkeypatch.setenv("RBE_ML_LANES", "1")
    sc = _grid_scene(scene)
    o = oracle_lib.OracleScene()
    o.set_scene(sc.boxes, sc.plane_z, sc.base)
    o.set_attached(-1)
    gpu_ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
    gpu_ctx.set_attached(-1)
    qa, qb, res = _edges(n, 23 + n, scale)
    ref = o.check_edges(qa, qb, res)
    for pk in ("8", "0"):
        monkeypatch.setenv("RBE_EDGE_COARSE", pk)
        got = gpu_ctx.check_edges(qa, qb, res)
        assert np.array_equal(got, ref), f"pk {pk}: {int((got != ref).sum())} of {n} edge flags differ"


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("name", ["C5_well_s3", "C5_well_s0", "C5_clutter64"])
def test_grid_scene_plans(gpu_ctx, mode, name, monkeypatch):
    """Whole plans on the grid scenes at their configured batch (tests/test_gpu_configs.py
    golden plans): the same status, iterations, trees and waypoints in every mode."""
    monkeypatch.setenv("RBE_SCENE_LDS", mode)
    _check(gpu_ctx, name)
