"""Never pairs (rp_model.h NEVER_PAIRS): self pairs that k_validity skips for waves
whose states are all inside the joint limits. The skip is exact because each pair is
proven unable to touch inside the limits (tools/prove_pairs.py; committed output
tests/golden/never_pairs_proof.json). CPU tests: the kernel's list and limits match
the proof, the tightest proof re-runs, and random in-limit states keep every never
pair farther apart than its radii."""
import json
import os
import re
import subprocess
import sys

import numpy as np

from rbe550_final_project_amd import model

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = open(os.path.join(ROOT, "rbe550_final_project_amd", "csrc", "rp_model.h")).read()
PROOF = json.load(open(os.path.join(ROOT, "tests", "golden", "never_pairs_proof.json")))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import prove_pairs as PP  # noqa: E402

CNAME = {"C_LINK0": "link0", "C_LINK1": "link1", "C_LINK2": "link2", "C_LINK3": "link3", "C_LINK4": "link4",
         "C_LINK5A": "link5a", "C_LINK5B": "link5b", "C_LINK6": "link6", "C_LINK7": "link7", "C_HAND": "hand",
         "C_LFINGER": "lfinger", "C_RFINGER": "rfinger"}


def _kernel_never():
    block = HDR[HDR.index("NEVER_PAIRS[][2]"):]
    block = block[:block.index("};")]
    return [(CNAME[a], CNAME[b]) for a, b in re.findall(r"\{(C_\w+), (C_\w+)\}", block)]


def test_kernel_list_is_the_proven_list():
    proven = [tuple(r["pair"]) for r in PROOF if r["proven"]]
    assert all(r["proven"] and r["margin"] > 0 for r in PROOF)
    assert sorted(_kernel_never()) == sorted(proven)


def test_kernel_limits_are_model_limits():
    def arr(name):
        m = re.search(name + r"\[NQ\] = \{([^}]*)\}", HDR)
        return np.array([np.float32(float(x.strip().rstrip("f"))) for x in m.group(1).split(",")], dtype=np.float64)
    assert np.array_equal(arr("Q_LO_F"), model.Q_LO) and np.array_equal(arr("Q_HI_F"), model.Q_HI)


def test_tightest_proof_reruns():
    """link5b-hand (margin 0.9 mm, two joints) re-proven from scratch."""
    I, J = PP.NAMES.index("link5b"), PP.NAMES.index("hand")
    r = PP.prove(I, J, PP.grid_for(I, J))
    assert r["proven"] and abs(r["min_dist"] - [x for x in PROOF if x["pair"] == ["link5b", "hand"]][0]["min_dist"]) < 1e-12


def test_random_in_limit_states_keep_never_pairs_apart():
    rng = np.random.default_rng(11)
    q = model.Q_LO + (model.Q_HI - model.Q_LO) * rng.random((200000, 9))
    fr = PP.frames(q)
    for a, b in _kernel_never():
        I, J = PP.NAMES.index(a), PP.NAMES.index(b)
        a1, b1 = PP.endpoints(fr, I)
        a2, b2 = PP.endpoints(fr, J)
        d = PP.seg_seg(a1, b1, a2, b2)
        assert d.min() > PP.G[I, 6] + PP.G[J, 6], (a, b, d.min())


def test_proof_chain_matches_the_oracle_capsules(oracle_lib):
    """The proof's float64 chain places the capsules where the oracle (and so the
    kernel) does."""
    o = oracle_lib.OracleScene()
    rng = np.random.default_rng(5)
    q = model.Q_LO + (model.Q_HI - model.Q_LO) * rng.random((24, 9))
    fr = PP.frames(q)   # the proof's chain has its base at the origin, the oracle's at (0, 0, 0.01)
    for i in range(len(q)):
        k = o.fk_capsules(q[i].astype(np.float32))          # (12, 2, 3), base (0, 0, 0.01)
        for c in range(12):
            a, b = PP.endpoints([(R[i:i + 1], p[i:i + 1]) for R, p in fr], c)
            assert np.max(np.abs(k[c, 0] - (a[0] + [0, 0, 0.01]))) < 2e-6
            assert np.max(np.abs(k[c, 1] - (b[0] + [0, 0, 0.01]))) < 2e-6
