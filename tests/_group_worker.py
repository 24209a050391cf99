"""One rank of tests/test_gpu_group_procs.py: a fresh process with torch.distributed
(gloo) and the product rank group (distributed.Group, host transport) on GPU 0,
shared with the other rank. Plans the cases, then rank 0 leaves the group and
plans them again at world 1. Writes <out>.<rank>.npz."""
import faulthandler
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402

from rbe550_final_project_amd import _abi, model, scenes  # noqa: E402
from rbe550_final_project_amd.distributed import Group  # noqa: E402
from rbe550_final_project_amd.native import Context  # noqa: E402


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    cases = json.loads(sys.argv[5])
    # progress lines (on the GPU box: under gpurun_out/, which its hang detector watches)
    logdir = os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpurun_out") if os.environ.get("GRAFT_REPO_ROOT") else None
    logf = open(os.path.join(logdir, f"group_worker.{rank}.log"), "a") if logdir and os.path.isdir(logdir) else None

    t0 = time.time()

    def log(msg):
        line = f"[rank {rank} {time.time() - t0:7.2f}s] {msg}"
        print(line, flush=True)
        if logf:
            logf.write(line + "\n")
            logf.flush()
    faulthandler.dump_traceback_later(int(os.environ.get("RBE_WORKER_TIMEOUT", "150")), exit=True)
    log("start")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    log("process group up")
    ctx = Context(device=0, robot=model.robot_desc())
    transport = os.environ.get("RBE_WORKER_TRANSPORT", "shm")
    grp = Group(ctx, transport=transport)
    log(f"rank group up ({transport})")
    res = {}

    def run(tag):
        for c in cases:
            q = json.load(open(os.path.join(ROOT, "tests", "golden", "workloads", c["workload"] + ".json")))
            q = q["queries"][c["query"]]
            sc = scenes.Scene.from_json(q["scene"])
            ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
            ctx.set_attached(q["attached"])
            p = _abi.make_params(seed=c["seed"], batch=c["batch"], batch_min=c.get("batch_min", 0), n_waypoints=150,
                                 timeout_s=3600.0, straight_first=False, tree_capacity=1 << 23,
                                 max_iters=c.get("max_iters", 0), group_repl=c.get("group_repl", 0))
            log(f"{tag} {c['name']} ...")
            path, st = ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
            s = ctx.stats()
            log(f"{tag} {c['name']} status {st} iterations {s['iterations']} trees {s['start_tree_size']} "
                f"{s['goal_tree_size']} {s['total_ms']:.1f} ms (exchange {s['exchange_ms']:.1f} ms)")
            res[f"{tag}/{c['name']}/path"] = path
            res[f"{tag}/{c['name']}/info"] = np.array([st, s["iterations"], s["start_tree_size"], s["goal_tree_size"]])

    def broken_group(res):
        """a rank whose grouped plan fails must not go on with the group
        out of step. Rank 1 skips one plan; rank 0's plan gives up at the exchange
        (wait watchdog) and every later grouped plan on rank 0 fails at once until
        the group is initialised again; then both ranks plan together again."""
        nonlocal grp
        from rbe550_final_project_amd.native import NativeError
        c = cases[0]
        q = json.load(open(os.path.join(ROOT, "tests", "golden", "workloads", c["workload"] + ".json")))
        q = q["queries"][c["query"]]
        sc = scenes.Scene.from_json(q["scene"])
        ctx.set_scene(sc.boxes, sc.plane_z, sc.base)
        ctx.set_attached(q["attached"])
        # every iteration sharded (group_repl < 0): a rank planning alone waits at the
        # first exchange
        p = _abi.make_params(seed=c["seed"], batch=c["batch"], n_waypoints=150, timeout_s=3600.0,
                             straight_first=False, group_repl=-1)
        dist.barrier()
        if rank == 0:
            os.environ["RBE_WAIT_WATCHDOG_S"] = "2"
            errs = []
            for _ in range(2):
                try:
                    ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
                    errs.append("")
                except NativeError as e:
                    errs.append(str(e))
            os.environ["RBE_WAIT_WATCHDOG_S"] = "30"
            log(f"break: {errs}")
            res["break/first_failed"] = np.array([int(bool(errs[0]))])
            res["break/second_broken"] = np.array([int("broken" in errs[1])])
        dist.barrier()
        grp.leave()
        grp = Group(ctx, transport=transport)
        path, st = ctx.plan(q["start"], q["goal"], model.Q_LO, model.Q_HI, p)
        res["break/path_after_reinit"] = path
        log(f"break: plan after re-init status {st}")

    order = os.environ.get("RBE_WORKER_ORDER", "group_first")
    if order == "single_first" and rank == 0:
        grp.leave()
        run("single")
        grp = Group(ctx, transport=transport)
    dist.barrier()
    grp_info = ctx.group_info()
    run("group")
    calls = grp.calls if transport == "host" else len(cases)
    if os.environ.get("RBE_WORKER_BREAK") and world > 1:
        broken_group(res)
    dist.barrier()
    if rank == 0 and order != "single_first":
        grp.leave()
        run("single")
    res["calls"] = np.array([calls])
    res["info"] = np.array([grp_info["rank"], grp_info["world"]])
    np.savez(f"{out}.{rank}.npz", **res)
    if os.environ.get("RBE_WORKER_KEEP"):
        log("final barrier (context kept)")
        dist.barrier()
    log("closing")
    ctx.close()
    log("closed, final barrier")
    dist.barrier()
    dist.destroy_process_group()
    log("end")


if __name__ == "__main__":
    main()
