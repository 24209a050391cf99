"""The product rank group end to end across PROCESSES: two fresh
Python processes (tests/_group_worker.py) join torch.distributed (gloo), build
distributed.Group on GPU 0 (shared; the shared-memory transport, or the host
transport over gloo, carries the record exchange) and plan — a goal3 query at a 256-sample batch, and BASELINE C4 / C5
queries at their configured 262,144 / 131,072-sample iterations (C5 covered well:
3 iterations, trees of 1.5 x 10^5 nodes). Both ranks' plans must equal rank 0's
world-1 plan, the golden oracle plans (tests/golden/plans_configured.npz) and, for
the goal3 query, the live oracle.

This test starts GPU processes, so conftest.py runs it before any test that
initialises the GPU in the pytest process (no process is started from a
GPU-initialised one)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from rbe550_final_project_amd import _abi, model, scenes

pytestmark = [pytest.mark.gpu, pytest.mark.spawns_gpu_procs]
HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")

CASES = [
    {"name": "goal3_q5", "workload": "goal3_tallest_10box", "query": 5, "seed": 13, "batch": 256},
    {"name": "C4_q0", "workload": "goal4_pentagon_10box", "query": 0, "seed": 0, "batch": 262144,
     "batch_min": 262144},
    {"name": "C5_clutter64", "workload": "clutter64", "query": 0, "seed": 0, "batch": 131072, "batch_min": 131072},
    {"name": "C5_well_s4", "workload": "clutter64_well", "query": 0, "seed": 4, "batch": 131072,
     "batch_min": 131072, "max_iters": 8},
]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("transport", ["shm", "host"])
def test_two_process_group_plans_equal_world1_and_oracle(tmp_path, oracle_lib, transport):
    out = str(tmp_path / "res")
    port = str(_free_port())
    env = dict(os.environ, RBE_WAIT_WATCHDOG_S="30", RBE_WORKER_TRANSPORT=transport)
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "_group_worker.py"), str(r), "2", port, out,
                               json.dumps(CASES)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                              env=env)
             for r in range(2)]
    logs = []
    for pr in procs:
        try:
            logs.append(pr.communicate(timeout=160)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    for pr, log in zip(procs, logs):
        assert pr.returncode == 0, log[-3000:]
    r0, r1 = (np.load(f"{out}.{r}.npz") for r in range(2))
    fix = np.load(os.path.join(GOLD, "plans_configured.npz"))
    meta = json.loads(str(fix["meta"]))
    assert int(r0["calls"][0]) >= len(CASES) and int(r1["calls"][0]) == int(r0["calls"][0])
    for c in CASES:
        n = c["name"]
        for r in (r0, r1):
            assert np.array_equal(r[f"group/{n}/path"], r0[f"single/{n}/path"]), n
            assert np.array_equal(r[f"group/{n}/info"], r0[f"single/{n}/info"]), n
        if n in meta:
            m = meta[n]
            assert list(r0[f"group/{n}/info"]) == [m["status"], m["iterations"], m["start_tree"], m["goal_tree"]], n
            assert np.array_equal(r0[f"group/{n}/path"], fix[n]), n
        else:
            q = json.load(open(os.path.join(GOLD, "workloads", c["workload"] + ".json")))["queries"][c["query"]]
            sc = scenes.Scene.from_json(q["scene"])
            o = oracle_lib.OracleScene()
            o.set_scene(sc.boxes, sc.plane_z, sc.base)
            o.set_attached(q["attached"])
            p = _abi.make_params(seed=c["seed"], batch=c["batch"], n_waypoints=150, timeout_s=3600.0,
                                 straight_first=False)
            ref, st, stats = o.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
            assert st == _abi.STATUS_EXACT and int(r0[f"group/{n}/info"][0]) == st
            assert np.array_equal(r0[f"group/{n}/path"], ref), n
