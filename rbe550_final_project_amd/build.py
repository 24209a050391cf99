"""Build librbe_mi355x.so in-tree with hipcc for gfx950.

    python -m rbe550_final_project_amd.build
"""
import os
import subprocess
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(_HERE, "csrc", "rp_lib.hip")
OUT = os.path.join(_HERE, "librbe_mi355x.so")
HEADERS = [os.path.join(_HERE, "csrc", f) for f in ("rp_kernels.h", "rp_math.h", "rp_plan_math.h", "rp_model.h")]
HEADERS.append(os.path.join(os.path.dirname(_HERE), "include", "rbe_planner.h"))

# -ffp-contract=off: no FMA contraction on host or device — the numerics contract
# that makes the GPU flags/trees bit-identical to the CPU oracle.
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
         "-fno-fast-math", "-Wall", "-Wno-unused-result"]


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.exists(c) or c == "hipcc"):
            return c
    raise RuntimeError("hipcc not found")


def up_to_date():
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(p) <= t for p in [SRC] + HEADERS if os.path.exists(p))


def build(force=False, verbose=True):
    if not force and up_to_date():
        return OUT
    cmd = [hipcc()] + FLAGS + ["-o", OUT, SRC]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
