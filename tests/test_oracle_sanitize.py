"""Host sanitizer leg of the CPU oracle (SURVEY.md §5 "race detection /
sanitizers"): oracle/sanitize_main.c built with -fsanitize=address,undefined
(oracle/Makefile `asan`) runs every checker entry point the parity tests use —
state / edge checks cross-checked batched vs single, contacts, plans at three
batch sizes and all simplification levels, a two-rank plan (ranks as threads)
equal to the one-rank plan, interpolate, IK — on a workload scene with an
attached box. Any ASan / UBSan report aborts it. CPU only."""
import ctypes as C
import json
import os
import subprocess

import numpy as np
import pytest

from rbe550_final_project_amd import _abi, model, scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


def _input(path, wl, qi):
    q = json.load(open(os.path.join(ROOT, "tests", "golden", "workloads", wl + ".json")))["queries"][qi]
    sc = scenes.Scene.from_json(q["scene"])
    arr, n = _abi.make_boxes(sc.boxes)
    with open(path, "wb") as f:
        f.write(bytes(model.robot_desc()))
        f.write(np.int32(n).tobytes())
        f.write(C.string_at(arr, C.sizeof(_abi.Box) * n))
        f.write(np.int32(q["attached"]).tobytes())
        for v in (q["start"], q["goal"], model.Q_LO, model.Q_HI):
            f.write(np.asarray(v, dtype=np.float64).tobytes())


@pytest.mark.parametrize("wl,qi", [("goal3_tallest_10box", 2), ("clutter64", 0)])
def test_oracle_under_asan_ubsan(tmp_path, wl, qi):
    try:
        subprocess.run(["make", "-s", "-C", ORACLE, "asan"], check=True, capture_output=True, timeout=300)
    except subprocess.CalledProcessError as ex:
        if b"sanitize" in ex.stderr and b"cannot find" in ex.stderr:
            pytest.skip("no ASan runtime in this toolchain")
        raise
    inp = tmp_path / "in.bin"
    _input(str(inp), wl, qi)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1",
               OMP_NUM_THREADS="2")
    r = subprocess.run([os.path.join(ORACLE, "_build", "sanitize_main"), str(inp)], capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "sanitize ok" in r.stdout and "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
