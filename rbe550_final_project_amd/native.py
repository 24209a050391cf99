"""Loader of librbe_mi355x.so (the HIP extension) and a thin Python handle over it.

The library is built in-tree (__graft_entry__.build() / `python -m
rbe550_final_project_amd.build`). There is no fallback: if the library or a gfx950
device is missing, every entry point raises.
"""
import ctypes as C
import os

import numpy as np

from . import _abi

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = "librbe_mi355x.so"
# RBE_LIB_PATH: an A/B build of the same library (tools/build_variants.sh), dev only
LIB_PATH = os.environ.get("RBE_LIB_PATH") or os.path.join(_HERE, LIB_NAME)

# every symbol include/rbe_planner.h declares
EXPORTS = ("rp_version", "rp_abi_version", "rp_default_robot", "rp_create", "rp_destroy", "rp_set_scene", "rp_set_scene_rot", "rp_set_attached",
           "rp_set_scene_poses",
           "rp_check_states", "rp_check_states_device", "rp_check_edges", "rp_check_edges_device",
           "rp_state_contacts", "rp_plan", "rp_plan_async", "rp_plan_wait", "rp_plan_many", "rp_reserve", "rp_group_init", "rp_group_init_shm", "rp_group_rccl_unique_id", "rp_group_init_rccl",
           "rp_group_init_local",
           "rp_get_stats", "rp_last_error", "rp_last_kernel_ms", "rp_selftest_f64", "rp_ik", "rp_set_profiling",
           "rp_get_profile", "rp_get_stream", "rp_group_info", "rp_selftest_nn")

# rp_allgather_fn(user, send, recv, bytes_per_rank): library-owned pinned host buffers
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64)
RCCL_ID_BYTES = 128

_lib = None


class NativeError(RuntimeError):
    pass


def load():
    """Load the HIP extension; raise loudly if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeError(f"{LIB_PATH} is not built; run __graft_entry__.build() "
                          "(there is no CPU fallback for the planner)")
    L = C.CDLL(LIB_PATH)
    vp, i32, i64, u32, f32, f64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint32, C.c_float, C.c_double
    L.rp_abi_version.restype = C.c_int
    if L.rp_abi_version() != _abi.ABI_VERSION:
        raise NativeError(f"{LIB_PATH}: ABI version {L.rp_abi_version()}, the ctypes mirrors are version "
                          f"{_abi.ABI_VERSION} (rebuild: __graft_entry__.build())")
    L.rp_version.restype = C.c_char_p
    L.rp_default_robot.argtypes = [C.POINTER(_abi.RobotDesc)]
    L.rp_create.argtypes = [C.POINTER(vp), C.c_int, C.POINTER(_abi.RobotDesc)]
    L.rp_destroy.argtypes = [vp]
    L.rp_destroy.restype = None
    L.rp_set_scene.argtypes = [vp, vp, i32, f32, C.POINTER(f32)]   # rp_box* (ctypes array or address)
    L.rp_set_scene_rot.argtypes = [vp, vp, i32, f32, C.POINTER(f32)]   # rp_box_rot*
    L.rp_set_attached.argtypes = [vp, i32, u32]
    L.rp_set_scene_poses.argtypes = [vp, vp, vp, i32, f32, vp, i32, u32]
    L.rp_check_states.argtypes = [vp, vp, i64, vp]
    L.rp_check_states_device.argtypes = [vp, vp, i64, vp, vp]
    L.rp_check_edges.argtypes = [vp, vp, vp, i64, f64, vp]
    L.rp_check_edges_device.argtypes = [vp, vp, vp, i64, f64, vp, vp]
    L.rp_state_contacts.argtypes = [vp, vp, vp, i32]
    L.rp_plan.argtypes = [vp, vp, vp, vp, vp, C.POINTER(_abi.PlanParams), vp, i32, C.POINTER(i32), C.POINTER(i32)]
    L.rp_plan_async.argtypes = L.rp_plan.argtypes
    L.rp_plan_wait.argtypes = [vp]
    L.rp_reserve.argtypes = [vp, i64, i64]
    L.rp_group_init.argtypes = [vp, i32, i32, vp, vp]
    L.rp_group_rccl_unique_id.argtypes = [vp]
    L.rp_group_init_shm.argtypes = [vp, i32, i32, vp, i64]
    L.rp_group_init_rccl.argtypes = [vp, i32, i32, vp]
    L.rp_group_init_local.argtypes = [vp, i32, i32, i64]
    L.rp_get_stats.argtypes = [vp, C.POINTER(_abi.Stats)]
    L.rp_group_info.argtypes = [vp, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32)]
    L.rp_set_profiling.argtypes = [vp, i32]
    L.rp_get_stream.argtypes = [vp, C.POINTER(vp)]
    L.rp_get_profile.argtypes = [vp, C.POINTER(_abi.Profile)]
    L.rp_last_error.argtypes = [vp]
    L.rp_last_error.restype = C.c_char_p
    L.rp_last_kernel_ms.argtypes = [vp, C.POINTER(f64)]
    L.rp_selftest_f64.argtypes = [vp, vp, i64, vp]
    L.rp_selftest_nn.argtypes = [vp, vp, i64, vp, i64, vp, vp, i32, vp]
    L.rp_ik.argtypes = [vp, i32, vp, vp, vp, vp, vp, C.POINTER(_abi.IkParams), vp, vp]
    _lib = L
    return L


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def rccl_unique_id():
    """ncclGetUniqueId (rank 0 of an RCCL rank group; broadcast it to the others)."""
    buf = (C.c_uint8 * RCCL_ID_BYTES)()
    rc = load().rp_group_rccl_unique_id(buf)
    if rc != 0:
        raise NativeError(f"rp_group_rccl_unique_id failed ({rc}): {load().rp_last_error(None).decode()}")
    return bytes(buf)


def group_init_local(ctxs, transport=None, nbytes=0):
    """rp_group_init_local: the contexts of this process become ranks 0..n-1 of one
    group ("rccl": ncclCommInitAll, distinct devices; "shm": a library-owned pinned
    segment, devices may repeat; None: rccl when the devices are distinct)."""
    codes = {None: 0, "none": 0, "rccl": 2, "shm": 3}
    if transport not in codes:
        raise ValueError(f"unknown transport {transport!r}")
    arr = (C.c_void_p * len(ctxs))(*[c._h.value for c in ctxs])
    rc = load().rp_group_init_local(arr, len(ctxs), codes[transport], int(nbytes))
    if rc < 0:
        raise NativeError(f"rp_group_init_local failed ({rc}): {load().rp_last_error(ctxs[0]._h).decode()}")


def default_robot():
    d = _abi.RobotDesc()
    load().rp_default_robot(C.byref(d))
    return d


class Context:
    """One planner context on one GPU (one per rank)."""

    def __init__(self, device=0, robot=None):
        L = load()
        self._h = C.c_void_p()
        self.robot = robot
        rc = L.rp_create(C.byref(self._h), int(device), C.byref(robot) if robot is not None else None)
        if rc != 0:
            raise NativeError(f"rp_create failed ({rc}): {L.rp_last_error(None).decode()}")
        self.device = device
        self.scene_gen = 0   # bumped by every set_scene / set_attached (callers that cache a scene)
        self._cb = None
        self._group_bufs = None
        self._in_flight = False   # a rp_plan_async query awaits its rp_plan_wait

    def close(self):
        if self._h:
            load().rp_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc < 0:
            raise NativeError(f"{what} failed ({rc}): {load().rp_last_error(self._h).decode()}")
        return rc

    # -- scene ---------------------------------------------------------------
    def set_scene(self, boxes, plane_z=0.0, base=(0.0, 0.0, 0.01)):
        """boxes: (center, half, yaw or quaternion (w, x, y, z)); rp_set_scene when every
        box is upright (a yaw), else rp_set_scene_rot (tilted boxes)."""
        kind, arr, n = _abi.scene_boxes(boxes)
        b = (C.c_float * 3)(*[float(v) for v in base])
        self.scene_gen += 1
        if kind == "rot":
            self._check(load().rp_set_scene_rot(self._h, arr, n, float(plane_z), b), "rp_set_scene_rot")
        else:
            self._check(load().rp_set_scene(self._h, arr, n, float(plane_z), b), "rp_set_scene")

    def set_scene_poses(self, poses, halves, plane_z, base, attached=-1, link_mask=_abi.ATTACH_EXEMPT_MASK):
        """rp_set_scene_poses: boxes from simulator poses (n, 7) float64 [x, y, z, qw,
        qx, qy, qz] and half extents (n, 3) float32, the robot base (3,) float64 and
        the attached box, in one call."""
        assert poses.dtype == np.float64 and halves.dtype == np.float32 and base.dtype == np.float64
        self.scene_gen += 1
        n = len(poses)
        self._check(load().rp_set_scene_poses(self._h, poses.ctypes.data if n else None,
                                              halves.ctypes.data if n else None, n, float(plane_z),
                                              base.ctypes.data, int(attached), int(link_mask)),
                    "rp_set_scene_poses")

    def set_attached(self, box_index, link_mask=_abi.ATTACH_EXEMPT_MASK):
        self.scene_gen += 1
        self._check(load().rp_set_attached(self._h, int(box_index), int(link_mask)), "rp_set_attached")

    # -- validity ------------------------------------------------------------
    def check_states(self, q):
        q = np.ascontiguousarray(q, dtype=np.float32).reshape(-1, _abi.NQ)
        out = np.empty(len(q), dtype=np.uint8)
        self._check(load().rp_check_states(self._h, _ptr(q), len(q), _ptr(out)), "rp_check_states")
        return out

    def check_states_device(self, q_ptr, n, flags_ptr, stream=None):
        self._check(load().rp_check_states_device(self._h, C.c_void_p(q_ptr), int(n), C.c_void_p(flags_ptr),
                                                  C.c_void_p(stream) if stream else None),
                    "rp_check_states_device")

    def last_kernel_ms(self):
        v = C.c_double()
        self._check(load().rp_last_kernel_ms(self._h, C.byref(v)), "rp_last_kernel_ms")
        return v.value

    def sub_batches(self, cap=1024):
        """The last plan's sub-batches: [(samples, host wall ms)] (rp_debug_subbatches,
        a diagnostic entry: bench.py's scaling model)."""
        buf = (C.c_double * (2 * cap))()
        m = load().rp_debug_subbatches(self._h, buf, 2 * cap)
        if m < 0:
            raise NativeError(f"rp_debug_subbatches failed ({m})")
        return [(int(buf[2 * i]), float(buf[2 * i + 1])) for i in range(min(m, cap))]

    def check_edges(self, qa, qb, resolution):
        qa = np.ascontiguousarray(qa, dtype=np.float64).reshape(-1, _abi.NQ)
        qb = np.ascontiguousarray(qb, dtype=np.float64).reshape(-1, _abi.NQ)
        out = np.empty(len(qa), dtype=np.uint8)
        self._check(load().rp_check_edges(self._h, _ptr(qa), _ptr(qb), len(qa), float(resolution), _ptr(out)),
                    "rp_check_edges")
        return out

    def check_edges_device(self, qa_ptr, qb_ptr, n, resolution, out_ptr, stream=None):
        """rp_check_edges_device on device buffers (N x 9 float64 endpoints, N uint8
        flags), asynchronous on `stream` (None: the context stream)."""
        self._check(load().rp_check_edges_device(self._h, C.c_void_p(qa_ptr), C.c_void_p(qb_ptr), int(n),
                                                 float(resolution), C.c_void_p(out_ptr),
                                                 C.c_void_p(stream) if stream else None), "rp_check_edges_device")

    def contacts(self, q, cap=64):
        q = np.ascontiguousarray(q, dtype=np.float64)
        out = np.zeros((cap, 2), dtype=np.int32)
        n = self._check(load().rp_state_contacts(self._h, _ptr(q), _ptr(out), cap), "rp_state_contacts")
        return [tuple(int(v) for v in x) for x in out[:min(n, cap)]]

    def selftest_f64(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        out = np.zeros((len(x), 6), dtype=np.float64)
        self._check(load().rp_selftest_f64(self._h, _ptr(x), len(x), _ptr(out)), "rp_selftest_f64")
        return out

    def selftest_nn(self, q, tree, lo, hi, mode):
        """rp_selftest_nn: nearest tree state of each query (lowest index on ties)."""
        q = np.ascontiguousarray(q, dtype=np.float64).reshape(-1, _abi.NQ)
        tree = np.ascontiguousarray(tree, dtype=np.float64).reshape(-1, _abi.NQ)
        lo = np.ascontiguousarray(lo, dtype=np.float64)
        hi = np.ascontiguousarray(hi, dtype=np.float64)
        out = np.zeros(len(q), dtype=np.int32)
        self._check(load().rp_selftest_nn(self._h, _ptr(q), len(q), _ptr(tree), len(tree), _ptr(lo), _ptr(hi),
                                          int(mode), _ptr(out)), "rp_selftest_nn")
        return out

    # -- planning ------------------------------------------------------------
    def _plan_buffers(self, path_cap):
        # A plan of a few tens of microseconds: the call's own overhead matters, so the
        # inputs go into one reused buffer whose address (and the output's) is taken
        # once (ndarray.ctypes costs microseconds per use)
        b = getattr(self, "_plan_bufs", None)
        if b is None or len(b["out"]) < path_cap:
            inp = np.empty(4 * _abi.NQ, dtype=np.float64)
            out = np.empty((path_cap, _abi.NQ), dtype=np.float64)
            n, status = C.c_int32(0), C.c_int32(0)
            a = inp.ctypes.data
            L = load()
            b = self._plan_bufs = {"inp": inp, "out": out, "n": n, "status": status, "fn": L.rp_plan,
                                   "fn_async": L.rp_plan_async, "fn_wait": L.rp_plan_wait,
                                   "args": (a, a + 8 * _abi.NQ, a + 16 * _abi.NQ, a + 24 * _abi.NQ),
                                   "out_addr": out.ctypes.data, "rn": C.byref(n), "rs": C.byref(status)}
        return b

    def _plan_call(self, fn, start, goal, lo, hi, params, path_cap):
        # the planner thread writes into the out / n / status buffers of a query in
        # flight: nothing may replace them before its plan_wait; the
        # library refuses the call too (RP_ERR_STATE), but only after this point
        if self._in_flight:
            raise NativeError("rp_plan: a query is in flight on this context (plan_wait first)")
        b = self._plan_buffers(path_cap)
        inp, nq = b["inp"], _abi.NQ
        inp[0:nq] = start
        inp[nq:2 * nq] = goal
        inp[2 * nq:3 * nq] = lo
        inp[3 * nq:4 * nq] = hi
        a0, a1, a2, a3 = b["args"]
        rc = b[fn](self._h, a0, a1, a2, a3, C.byref(params), b["out_addr"], path_cap, b["rn"], b["rs"])
        if rc < 0:
            self._check(rc, "rp_plan" if fn == "fn" else "rp_plan_async")
        return b

    def plan(self, start, goal, lo, hi, params, path_cap=4096):
        """rp_plan: (path (n, 9) float64, status)."""
        b = self._plan_call("fn", start, goal, lo, hi, params, path_cap)
        return b["out"][:b["n"].value].copy(), b["status"].value

    def reserve(self, batch=0, tree_capacity=0):
        """rp_reserve: size the planner workspace ahead of the first query."""
        self._check(load().rp_reserve(self._h, int(batch), int(tree_capacity)), "rp_reserve")

    def plan_async(self, start, goal, lo, hi, params, path_cap=4096):
        """rp_plan_async: hand the query to the context's planner thread and return
        at once; plan_wait() returns what plan() would. The params struct is copied."""
        self._plan_call("fn_async", start, goal, lo, hi, params, path_cap)
        self._in_flight = True

    def plan_wait(self, out=None):
        """rp_plan_wait: (path, status) of the query in flight. With `out` (an (m, 9)
        float array, e.g. the numpy view of a float32 tensor) a path of exactly m
        states is written into it (float64 -> float32 rounds once, as astype) and
        `out` is returned; otherwise a float64 copy."""
        b = self._plan_bufs
        rc = b["fn_wait"](self._h)
        self._in_flight = False
        if rc < 0:
            self._check(rc, "rp_plan")
        n = b["n"].value
        if out is not None and len(out) == n:
            np.copyto(out, b["out"][:n], casting="same_kind")
            return out, b["status"].value
        return b["out"][:n].copy(), b["status"].value

    def ik(self, pos, quat, init, lo, hi, params=None):
        """Batched hand-link IK (rp_ik): pos (T, 3), quat (T, 4) as w, x, y, z, init
        (T, 9) -> (q (T, 9) float64, status (T,) int32)."""
        pos = np.ascontiguousarray(pos, dtype=np.float64).reshape(-1, 3)
        quat = np.ascontiguousarray(quat, dtype=np.float64).reshape(-1, 4)
        init = np.ascontiguousarray(init, dtype=np.float64).reshape(-1, _abi.NQ)
        lo = np.ascontiguousarray(lo, dtype=np.float64)
        hi = np.ascontiguousarray(hi, dtype=np.float64)
        n = len(pos)
        assert len(quat) == n and len(init) == n
        p = params if params is not None else _abi.make_ik_params()
        q = np.zeros((n, _abi.NQ), dtype=np.float64)
        st = np.zeros(n, dtype=np.int32)
        self._check(load().rp_ik(self._h, n, _ptr(pos), _ptr(quat), _ptr(init), _ptr(lo), _ptr(hi), C.byref(p),
                                 _ptr(q), _ptr(st)), "rp_ik")
        return q, st

    def stream_handle(self):
        """The context's hipStream_t (as an int), for events / ordering (rp_get_stream)."""
        h = C.c_void_p()
        self._check(load().rp_get_stream(self._h, C.byref(h)), "rp_get_stream")
        return int(h.value or 0)

    def set_profiling(self, on=True):
        self._check(load().rp_set_profiling(self._h, 1 if on else 0), "rp_set_profiling")

    def profile(self):
        """Kernel-class timing of the last plan (rp_get_profile)."""
        pr = _abi.Profile()
        self._check(load().rp_get_profile(self._h, C.byref(pr)), "rp_get_profile")
        return pr.as_dict()

    def stats(self):
        st = _abi.Stats()
        self._check(load().rp_get_stats(self._h, C.byref(st)), "rp_get_stats")
        return st.as_dict()

    # -- rank group ----------------------------------------------------------
    def group_init(self, rank, world, allgather):
        """Host transport: allgather(send, recv) gathers the uint8 array `send` of
        every rank into `recv` (rank-major, world * len(send) bytes); both are numpy
        views of library-owned pinned host buffers, valid during the call."""
        if allgather is None or world == 1:
            return self.group_leave()

        def _cb(_user, send_p, recv_p, nbytes):
            try:
                n = int(nbytes)
                send = np.ctypeslib.as_array((C.c_uint8 * n).from_address(send_p))
                recv = np.ctypeslib.as_array((C.c_uint8 * (n * int(world))).from_address(recv_p))
                allgather(send, recv)
                return 0
            except Exception:  # never let a Python exception cross into C
                import traceback
                traceback.print_exc()
                return 1
        self._cb = ALLGATHER_FN(_cb)
        self._check(load().rp_group_init(self._h, int(rank), int(world), C.cast(self._cb, C.c_void_p), None),
                    "rp_group_init")

    def group_init_rccl(self, rank, world, unique_id):
        """RCCL transport (ncclAllGather on the context stream); collective over the
        group, ranks on distinct GPUs. unique_id: rccl_unique_id() of rank 0."""
        uid = (C.c_uint8 * RCCL_ID_BYTES).from_buffer_copy(bytes(unique_id))
        self._check(load().rp_group_init_rccl(self._h, int(rank), int(world), uid), "rp_group_init_rccl")

    def group_init_shm(self, rank, world, address, nbytes):
        """Shared-memory transport over a host segment mapped by every rank of the node."""
        self._check(load().rp_group_init_shm(self._h, int(rank), int(world), C.c_void_p(address), int(nbytes)),
                    "rp_group_init_shm")

    def group_info(self):
        """The rank group as its transport sees it (rp_group_info): for RCCL the
        communicator's ncclCommUserRank / ncclCommCount."""
        r, w, t = C.c_int32(), C.c_int32(), C.c_int32()
        self._check(load().rp_group_info(self._h, C.byref(r), C.byref(w), C.byref(t)), "rp_group_info")
        return {"rank": r.value, "world": w.value, "transport": _abi.TRANSPORT_NAMES.get(t.value, str(t.value))}

    def group_leave(self):
        """Back to single-rank planning."""
        self._check(load().rp_group_init(self._h, 0, 1, None, None), "rp_group_init")
        self._cb = None


def make_queries(jobs):
    """rp_query records of plan_pipelined's jobs (dicts with scene (scenes.Scene,
    upright boxes), attached, start, goal, params): (array, keep-alive list)."""
    qs = (_abi.Query * max(1, len(jobs)))()
    keep = []
    for i, job in enumerate(jobs):
        sc = job["scene"]
        kind, arr, n = _abi.scene_boxes(sc.boxes)
        if kind != "yaw":
            raise ValueError("rp_plan_many takes upright boxes (rp_set_scene records); plan tilted scenes one by one")
        keep.append(arr)
        q = qs[i]
        q.boxes = C.cast(arr, C.POINTER(_abi.Box)) if n else None
        q.n_boxes = n
        q.plane_z = float(sc.plane_z)
        q.base_pos[:] = [float(v) for v in sc.base]
        q.attached_box = int(job.get("attached", -1))
        q.start[:] = [float(v) for v in job["start"]]
        q.goal[:] = [float(v) for v in job["goal"]]
        q.params = job["params"]
    return qs, keep


def plan_many(ctxs, queries, n, lo, hi, path_cap=4096):
    """rp_plan_many over prepared rp_query records (make_queries): [(path, status,
    stats)] in query order; raises NativeError (after every query ran) if any failed."""
    k = len(ctxs)
    arr = (C.c_void_p * k)(*[c._h.value for c in ctxs])
    out = np.empty((max(n, 1), path_cap, _abi.NQ), dtype=np.float64)
    n_out = np.zeros(max(n, 1), dtype=np.int32)
    st = np.zeros(max(n, 1), dtype=np.int32)
    rcs = np.zeros(max(n, 1), dtype=np.int32)
    lo = np.ascontiguousarray(lo, dtype=np.float64)
    hi = np.ascontiguousarray(hi, dtype=np.float64)
    rc = load().rp_plan_many(arr, k, queries, int(n), _ptr(lo), _ptr(hi), _ptr(out), int(path_cap), _ptr(n_out),
                             _ptr(st), _ptr(rcs))
    if rc < 0:
        bad = [i for i in range(n) if rcs[i] < 0]
        raise NativeError(f"rp_plan_many failed ({rc}) at queries {bad[:8]}: "
                          f"{load().rp_last_error(ctxs[bad[0] % k]._h if bad else None).decode()}")
    # (each context holds the stats of its last query only: per-query stats are those)
    last = {}
    for i in range(n):
        last[i % k] = i
    res = []
    for i in range(n):
        s = ctxs[i % k].stats() if last[i % k] == i else None
        res.append((out[i, :n_out[i]].copy(), int(st[i]), s))
    return res


def plan_pipelined(ctxs, jobs, path_cap=4096):
    """Independent queries kept in flight on several contexts of one device (BASELINE
    config 3: goal3's ~20 RRT queries "pipelined"): job i runs on ctxs[i % len(ctxs)]
    through its planner thread, after that context's previous job, all driven by one
    library call (rp_plan_many; the host side of a query is C++, not this loop). Each
    context has its own HIP stream, so one query's dependent small kernels overlap the
    others'. A job is a dict with scene (scenes.Scene), attached, start, goal, params;
    lo / hi are the jobs' common bounds (jobs[0]["lo"] / ["hi"]). Returns [(path,
    status, stats)] in job order (stats: that context's stats when the job was its last,
    else None); every path and status is the one ctx.plan gives for that job alone."""
    if not ctxs:
        raise ValueError("plan_pipelined needs a context")
    if not jobs:
        return []
    qs, keep = make_queries(jobs)
    res = plan_many(ctxs, qs, len(jobs), jobs[0]["lo"], jobs[0]["hi"], path_cap)
    del keep
    return res
