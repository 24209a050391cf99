"""GPU test of the large-tree nearest-node searches (rp_selftest_nn): the
matrix-core filter (k_nn_mfma: the filter value of 16 queries x 16 nodes in one
v_mfma_f32_16x16x32_f16, exact f64 distance for the nodes that pass) and the
packed-f32 filter (k_nn_part) return, for every query, exactly the index the oracle's
strict-< scan returns (nearest node, lowest index among equal f64 distances), on
random trees, trees with duplicated nodes (exact ties), queries on nodes (distance
0), queries equidistant from two nodes, dense clusters around the queries (many
nodes inside the filter's margin) and the corners of the bounds. The planner's use
is covered by the plan parity tests (tests/test_gpu_configs.py, RBE_NN_MFMA)."""
import numpy as np
import pytest

from rbe550_final_project_amd import model

pytestmark = pytest.mark.gpu
LO, HI = model.Q_LO, model.Q_HI
MODES = [0, 1, 4, 8]


def _ref(q, tree):
    """the oracle's scan: dist2(node, query) = sum over d in order of (node_d - x_d)^2
    (no fused multiply-add), first index of the minimum"""
    out = np.empty(len(q), dtype=np.int32)
    for i, x in enumerate(q):
        s = np.zeros(len(tree))
        for d in range(9):
            e = tree[:, d] - x[d]
            s = s + e * e
        out[i] = int(np.argmin(s))
    return out


def _uniform(rng, n):
    return LO + (HI - LO) * rng.random((n, 9))


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("T,n", [(1, 5), (70, 300), (5000, 1000), (60000, 1500)])
def test_random_trees(gpu_ctx, mode, T, n):
    rng = np.random.default_rng(T + n)
    tree, q = _uniform(rng, T), _uniform(rng, n)
    assert np.array_equal(gpu_ctx.selftest_nn(q, tree, LO, HI, mode), _ref(q, tree))


@pytest.mark.parametrize("mode", MODES)
def test_ties_duplicates_and_zero_distance(gpu_ctx, mode):
    rng = np.random.default_rng(7)
    base = _uniform(rng, 3000)
    # every node three times (exact ties: the first copy must win), queries on nodes,
    # and queries exactly halfway between two nodes along a power-of-two offset
    tree = np.concatenate([base, base[::-1], base])
    q_on = base[rng.integers(0, len(base), 400)]
    mid = _uniform(rng, 400) * 0.5 + 0.25 * (LO + HI)
    delta = np.zeros(9)
    delta[0] = 2.0 ** -6
    tree2 = np.concatenate([tree, mid + delta, mid - delta])
    q = np.concatenate([q_on, mid])
    assert np.array_equal(gpu_ctx.selftest_nn(q, tree2, LO, HI, mode), _ref(q, tree2))


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("scale", [1e-3, 1e-6, 1e-9])
def test_dense_clusters_around_queries(gpu_ctx, mode, scale):
    """nodes within `scale` of the queries: many candidates inside the filter's
    margin (e0 ~ 3e-3 rad^2), near-ties decided by the exact f64 distance"""
    rng = np.random.default_rng(int(1 / scale) % 1000)
    q = _uniform(rng, 256) * 0.9 + 0.05 * (LO + HI)
    tree = np.concatenate([q[rng.integers(0, len(q), 20000)] + scale * rng.standard_normal((20000, 9)),
                           _uniform(rng, 5000)])
    tree = np.clip(tree, LO, HI)
    assert np.array_equal(gpu_ctx.selftest_nn(q, tree, LO, HI, mode), _ref(q, tree))


@pytest.mark.parametrize("mode", MODES)
def test_bounds_corners(gpu_ctx, mode):
    """states on the corners and faces of the bounds (the largest coordinates and
    norms the filter's f16 scaling must hold)"""
    rng = np.random.default_rng(3)
    corners = np.where(rng.random((4000, 9)) < 0.5, LO, HI)
    faces = _uniform(rng, 4000)
    faces[np.arange(4000), rng.integers(0, 9, 4000)] = HI[0]
    faces = np.clip(faces, LO, HI)
    tree = np.concatenate([corners, faces])
    q = np.concatenate([np.where(rng.random((300, 9)) < 0.5, LO, HI), _uniform(rng, 300)])
    assert np.array_equal(gpu_ctx.selftest_nn(q, tree, LO, HI, mode), _ref(q, tree))
