"""Static guards on the device code of librbe_mi355x.so (CPU; no GPU needed).

The bit-exact flags depend on the compiler emitting exactly the
arithmetic written in rp_math.h. A compiler fold broke them once (round 5: the sin
/ cos quadrant's `(int)floorf(y + 0.5f)` became `v_cvt_rpi_i32_f32(y)`, which rounds
y + 0.5 exactly, not to float first), and sampled tests found it only on a second
seed. These tests read the gfx950 code object out of the built library and check:

* no instruction of the code object is one of the rewrites that change results
  (DESIGN.md §3 lists them): v_cvt_rpi_i32_f32 / v_cvt_flr_i32_f32 (rounding
  conversions that skip the float rounding of their operand), v_sin_f32 /
  v_cos_f32 (hardware transcendentals instead of rp_sincos), v_fma_mix* / v_mad_mix*
  (mixed-precision multiply-adds);
* no kernel a plan or the bench dispatches uses scratch memory (no register
  spills, no stack arrays): ScratchSize (.private_segment_fixed_size) is 0.

Reference: the flags they protect are `_is_ompl_state_valid`'s,
/root/reference/code/planning.py:209-219.
"""
import os
import re
import struct
import subprocess

import pytest

from rbe550_final_project_amd import build

LLVM = "/opt/rocm/lib/llvm/bin"
FORBIDDEN = re.compile(r"\b(v_cvt_rpi_i32_f32|v_cvt_flr_i32_f32|v_sin_f32|v_cos_f32|v_fma_mix\w*|v_mad_mix\w*)\b")
# kernels allowed to use scratch: diagnostics outside the query's hot path
#   k_contacts: rp_state_contacts (the start / goal contact list planning.py's
#   diagnostics print when a plan reports INVALID_START / INVALID_GOAL; two states)
SCRATCH_ALLOWED = {"k_contacts"}
# instantiations that run only under a non-default A/B knob (never in a default plan or
# the bench), allowed a few dwords of spill under the iterative-ILP scheduler
# (build.py DEVICE_FLAGS): the scanned edge launch (RBE_EDGE_PACKED=1) and the one-wave
# pass-1 list kernel of grid scenes (RBE_SCENE_LDS without bit 0; the default runs
# k_edges_units_gl)
SCRATCH_ALLOWED_AB = ("k_edges_packed<", "k_edges_units<-1,")


def _code_object(lib_path):
    """The gfx950 code object of the library's offload bundle (.hip_fatbin)."""
    b = open(lib_path, "rb").read()
    o = b.find(b"__CLANG_OFFLOAD_BUNDLE__")
    assert o >= 0, "no offload bundle in the library"
    n, = struct.unpack_from("<Q", b, o + 24)
    p = o + 32
    for _ in range(n):
        off, size, tl = struct.unpack_from("<QQQ", b, p)
        p += 24
        triple = b[p:p + tl].decode()
        p += tl
        if triple.endswith("gfx950"):
            return b[o + off:o + off + size]
    raise AssertionError("no gfx950 code object in the bundle")


@pytest.fixture(scope="module")
def code_object(tmp_path_factory):
    lib = build.build(verbose=False)
    path = tmp_path_factory.mktemp("isa") / "co.elf"
    path.write_bytes(_code_object(lib))
    return str(path)


def _demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True).stdout
    return out.split("\n")[:len(names)]


def _kernels(code_object):
    """[(demangled name, scratch bytes, vgprs)] from the code object's metadata."""
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", code_object], capture_output=True, text=True,
                           check=True).stdout
    names = re.findall(r"^\s+\.name:\s+(\S+)", notes, re.M)
    scratch = [int(x) for x in re.findall(r"\.private_segment_fixed_size:\s+(\d+)", notes)]
    vgprs = [int(x) for x in re.findall(r"\.vgpr_count:\s+(\d+)", notes)]
    assert len(names) == len(scratch) == len(vgprs) and len(names) > 100
    return list(zip(_demangle(names), scratch, vgprs))


def _base(name):
    m = re.match(r"_ZN2rp(\d+)", name)   # (c++filt leaves names with _Float16 arguments mangled)
    if m:
        return name[m.end():m.end() + int(m.group(1))]
    return re.sub(r"^(void )?rp::", "", name).split("<")[0].split("(")[0]


def test_no_result_changing_opcodes(code_object):
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", code_object], capture_output=True,
                         text=True, check=True).stdout
    hits, fn = [], None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            fn = m.group(1)
            continue
        m = FORBIDDEN.search(line)
        if m:
            hits.append((fn, m.group(1)))
    assert len(dis) > 10_000_000   # (the whole code object was disassembled)
    assert not hits, f"forbidden opcodes (DESIGN.md §3): {sorted(set(hits))[:20]}"


def test_collision_kernels_present(code_object):
    """The kernels the guards are about exist under the names they look for."""
    names = {_base(n) for n, _, _ in _kernels(code_object)}
    for k in ("k_validity", "k_validity_split", "k_validity_ml", "k_edges", "k_edges_ml", "k_straight",
              "k_straight_ml", "k_nn_mfma", "k_iter_accept_small", "k_group_accept_small"):
        assert k in names, k


def test_no_scratch_in_dispatched_kernels(code_object):
    bad = [(n[:110], s, v) for n, s, v in _kernels(code_object)
           if s > 0 and _base(n) not in SCRATCH_ALLOWED
           and not re.sub(r"^(void )?rp::", "", n).startswith(SCRATCH_ALLOWED_AB)]
    assert not bad, "kernels using scratch (spills / stack arrays):\n" + "\n".join(map(str, bad))
