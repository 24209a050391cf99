"""C-ABI boundary (CPU): librbe_mi355x.so builds, loads, exports every symbol the
header declares, and has no CPU path (rp_create fails loudly without a gfx950)."""
import ctypes as C
import os
import re

import pytest

from rbe550_final_project_amd import _abi, build, model, native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rbe_planner.h")


def _declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(rp_[a-z0-9_]+)\s*\(", src)) - {"rp_allgather_fn"})


def test_library_exports_header_symbols():
    build.build(verbose=False)
    lib = C.CDLL(native.LIB_PATH)
    names = _declared()
    assert len(names) >= 17
    for n in names:
        assert hasattr(lib, n), f"missing export {n}"
    assert set(names) <= set(native.EXPORTS)


def test_struct_layouts_match_header(tmp_path):
    """ctypes mirrors == the C compiler's view of include/rbe_planner.h."""
    import subprocess
    src = tmp_path / "sz.c"
    src.write_text("#include <stdio.h>\n#include <stddef.h>\n#include \"rbe_planner.h\"\n"
                   "int main(void){printf(\"%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\\n\", sizeof(rp_capsule), sizeof(rp_box),"
                   " sizeof(rp_plan_params), sizeof(rp_stats), sizeof(rp_robot_desc),"
                   " offsetof(rp_plan_params, n_waypoints), offsetof(rp_robot_desc, self_pairs),"
                   " sizeof(rp_ik_params), offsetof(rp_ik_params, damping), sizeof(rp_profile));"
                   "printf(\"%zu %zu %zu\\n\", sizeof(rp_query), offsetof(rp_query, start), offsetof(rp_query, params));"
                   "return 0;}")
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    want = [C.sizeof(_abi.Capsule), C.sizeof(_abi.Box), C.sizeof(_abi.PlanParams), C.sizeof(_abi.Stats),
            C.sizeof(_abi.RobotDesc), _abi.PlanParams.n_waypoints.offset, _abi.RobotDesc.self_pairs.offset,
            C.sizeof(_abi.IkParams), _abi.IkParams.damping.offset, C.sizeof(_abi.Profile),
            C.sizeof(_abi.Query), _abi.Query.start.offset, _abi.Query.params.offset]
    assert got == want


def test_default_robot_equals_spec():
    d = native.default_robot()
    s = model.robot_desc()
    assert d.n_capsules == s.n_capsules and d.n_self_pairs == s.n_self_pairs
    for i in range(s.n_capsules):
        assert d.capsules[i].link == s.capsules[i].link
        assert list(d.capsules[i].a) == list(s.capsules[i].a)
        assert list(d.capsules[i].b) == list(s.capsules[i].b)
        assert d.capsules[i].radius == s.capsules[i].radius
    for i in range(s.n_self_pairs):
        assert list(d.self_pairs[i]) == list(s.self_pairs[i])


def test_version_string():
    assert b"gfx950" in native.load().rp_version()


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(native.NativeError, match="no CPU path|no HIP device|not gfx950"):
        native.Context(device=0)
    with pytest.raises(native.NativeError):
        native.Context(device=-1)


def test_wrong_structure_rejected():
    d = model.robot_desc()
    d.capsules[3].link = 7
    h = C.c_void_p()
    rc = native.load().rp_create(C.byref(h), 0, C.byref(d))
    assert rc == _abi.ERR_ARG
    assert b"structure" in native.load().rp_last_error(None)
