"""Per-wave phase durations of k_validity from a diagnostic build (-DRP_STAMPS):
s_memtime at kernel entry, after the state load, at link4 / link6 / hand, after the
walk, after the box and self-pair drains. Usage: python tools/stamp_probe.py lib.so"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rbe550_final_project_amd import _abi, model, scenes  # noqa: E402

NAMES = ["load", "link0-3", "link4-5", "link6-7", "hand+fingers", "box drain", "self drain"]


def main():
    L = C.CDLL(os.path.abspath(sys.argv[1]))
    L.rp_create.argtypes = [C.POINTER(C.c_void_p), C.c_int, C.c_void_p]
    L.rp_set_scene.argtypes = [C.c_void_p, C.POINTER(_abi.Box), C.c_int32, C.c_float, C.POINTER(C.c_float)]
    L.rp_check_states_device.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]
    L.rp_debug_stamps.argtypes = [C.c_void_p, C.c_int64]
    h = C.c_void_p()
    assert L.rp_create(C.byref(h), 0, None) == 0
    sc = scenes.goal3_tallest()
    arr, nb = _abi.make_boxes(sc.boxes)
    assert L.rp_set_scene(h, arr, nb, 0.0, (C.c_float * 3)(*sc.base)) == 0
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    lo = torch.tensor(model.Q_LO, dtype=torch.float32, device=dev)
    hi = torch.tensor(model.Q_HI, dtype=torch.float32, device=dev)
    N = 1 << 22
    q = (lo + (hi - lo) * torch.rand((N, 9), generator=g, device=dev)).contiguous()
    f = torch.empty(N, dtype=torch.uint8, device=dev)
    st = torch.cuda.Stream(dev)
    buf = np.zeros(65536 * 8, dtype=np.uint64)
    for n in (1 << 16, 1 << 22):
        for _ in range(3):
            L.rp_check_states_device(h, q.data_ptr(), n, f.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        assert L.rp_debug_stamps(buf.ctypes.data_as(C.c_void_p), buf.size) == 0
        waves = min(n // 64, 65536)
        s = buf[: waves * 8].reshape(waves, 8).astype(np.int64)
        ok = (np.diff(s, axis=1) >= 0).all(axis=1) & (s[:, 0] > 0)
        s = s[ok]
        d = np.diff(s, axis=1)
        tot = s[:, 7] - s[:, 0]
        print(f"n={n}: {ok.sum()} waves with all stamps; wave total median {np.median(tot):.0f} p90 "
              f"{np.percentile(tot, 90):.0f} max {tot.max()} (s_memtime ticks)")
        for k, name in enumerate(NAMES):
            print(f"   {name:14s} median {np.median(d[:, k]):8.0f}  mean {d[:, k].mean():8.0f}  p90 {np.percentile(d[:, k], 90):8.0f}")
        span = s[:, 7].max() - s[:, 0].min()
        print(f"   launch span (first entry -> last exit) {span} ticks")


if __name__ == "__main__":
    main()
