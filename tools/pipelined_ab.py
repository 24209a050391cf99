"""C3 pipelined leg (bench.py run_plans_pipelined) under one library build, for an A/B
of builds (RBE_LIB_PATH selects the build): python tools/pipelined_ab.py [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

wl = json.load(open(os.path.join(ROOT, "tests/golden/workloads/goal3_tallest_10box.json")))
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 9
lib = os.path.basename(os.environ.get("RBE_LIB_PATH", "librbe_mi355x.so"))
for sf in (True, False):
    r = bench.run_plans_pipelined(0, wl, 4096, sf, 0.0, reps=reps)
    print(lib, "sf" if sf else "rrt", {k: v["total_ms"] for k, v in r["per_contexts"].items()}, flush=True)
