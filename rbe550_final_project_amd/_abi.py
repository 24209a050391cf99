"""ctypes mirrors of the C-ABI structs in include/rbe_planner.h (plain data only)."""
import ctypes as C
import math

ABI_VERSION = 7   # RP_ABI_VERSION of include/rbe_planner.h these mirrors follow
NQ = 9
MAX_CAPSULES = 32
MAX_SELF_PAIRS = 64
MAX_BOXES = 64

LINK_NAMES = ["link0", "link1", "link2", "link3", "link4", "link5", "link6", "link7",
              "hand", "left_finger", "right_finger"]
LINK_INDEX = {n: i for i, n in enumerate(LINK_NAMES)}
# links whose contacts with the attached object are ignored (code/planning.py:222)
ATTACH_EXEMPT_LINKS = ("left_finger", "right_finger", "hand")
ATTACH_EXEMPT_MASK = sum(1 << LINK_INDEX[n] for n in ATTACH_EXEMPT_LINKS)

OK = 0
ERR_ARG, ERR_DEVICE, ERR_STATE, ERR_CAPACITY, ERR_EXCHANGE = -1, -2, -3, -4, -5

STATUS_NONE, STATUS_EXACT, STATUS_APPROXIMATE, STATUS_TIMEOUT, STATUS_INVALID_START, STATUS_INVALID_GOAL = range(6)
TRANSPORT_NAMES = {0: "none", 1: "host", 2: "rccl", 3: "shm"}   # RP_TRANSPORT_*
STATUS_NAMES = {0: "NONE", 1: "EXACT", 2: "APPROXIMATE", 3: "TIMEOUT", 4: "INVALID_START", 5: "INVALID_GOAL"}


class Capsule(C.Structure):
    _fields_ = [("link", C.c_int32), ("a", C.c_float * 3), ("b", C.c_float * 3), ("radius", C.c_float)]


class RobotDesc(C.Structure):
    _fields_ = [("n_capsules", C.c_int32), ("capsules", Capsule * MAX_CAPSULES),
                ("n_self_pairs", C.c_int32), ("self_pairs", (C.c_int32 * 2) * MAX_SELF_PAIRS)]


class Box(C.Structure):
    _fields_ = [("center", C.c_float * 3), ("half", C.c_float * 3), ("yaw", C.c_float)]


class BoxRot(C.Structure):
    """rp_box_rot: orientation quaternion (w, x, y, z) in double."""
    _fields_ = [("center", C.c_float * 3), ("half", C.c_float * 3), ("quat", C.c_double * 4)]


class PlanParams(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("batch", C.c_int64), ("batch_min", C.c_int64), ("range", C.c_double),
                ("resolution", C.c_double), ("timeout_s", C.c_double), ("max_iters", C.c_int64),
                ("n_waypoints", C.c_int32), ("simplify", C.c_int32), ("tree_capacity", C.c_int64),
                ("straight_first", C.c_int32), ("chunk", C.c_int32),
                ("group_repl", C.c_int64)]


class Query(C.Structure):
    """rp_query: one query of rp_plan_many (its scene, attached box, start, goal, params)."""
    _fields_ = [("boxes", C.POINTER(Box)), ("n_boxes", C.c_int32), ("plane_z", C.c_float),
                ("base_pos", C.c_float * 3), ("attached_box", C.c_int32), ("start", C.c_double * NQ),
                ("goal", C.c_double * NQ), ("params", PlanParams)]


class IkParams(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("n_seeds", C.c_int32), ("iters", C.c_int32), ("damping", C.c_double),
                ("pos_tol", C.c_double), ("rot_tol", C.c_double)]


IK_OK, IK_COLLIDING, IK_NOT_CONVERGED = 0, 1, 2


def make_ik_params(seed=0, n_seeds=0, iters=0, damping=0.0, pos_tol=0.0, rot_tol=0.0):
    p = IkParams()
    p.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    p.n_seeds = int(n_seeds)
    p.iters = int(iters)
    p.damping = float(damping)
    p.pos_tol = float(pos_tol)
    p.rot_tol = float(rot_tol)
    return p


class Stats(C.Structure):
    _fields_ = [("states_checked", C.c_int64), ("edges_checked", C.c_int64), ("samples", C.c_int64),
                ("iterations", C.c_int64), ("start_tree_size", C.c_int64), ("goal_tree_size", C.c_int64),
                ("path_states_raw", C.c_int64), ("path_states_simplified", C.c_int64),
                ("solve_ms", C.c_double), ("simplify_ms", C.c_double), ("total_ms", C.c_double),
                ("exchange_ms", C.c_double)]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


class Profile(C.Structure):
    _fields_ = [("nn_launches", C.c_int64), ("nn_ms", C.c_double), ("nn_pairs", C.c_double),
                ("edge_launches", C.c_int64), ("edge_ms", C.c_double), ("edge_states", C.c_int64)]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


def is_quat(rot):
    """A box orientation is a yaw (number) or a quaternion (w, x, y, z)."""
    return hasattr(rot, "__len__") and len(rot) == 4


def quat_of(rot):
    """Quaternion (w, x, y, z) of a box orientation (a yaw is a rotation about z)."""
    if is_quat(rot):
        return tuple(float(v) for v in rot)
    y = float(rot)
    return (math.cos(0.5 * y), 0.0, 0.0, math.sin(0.5 * y))


def make_boxes(boxes):
    """boxes: iterable of (center(3), half(3), yaw) -> ctypes rp_box array."""
    boxes = list(boxes)
    arr = (Box * max(1, len(boxes)))()
    for i, (c, h, yaw) in enumerate(boxes):
        arr[i].center[:] = [float(v) for v in c]
        arr[i].half[:] = [float(v) for v in h]
        arr[i].yaw = float(yaw)
    return arr, len(boxes)


def make_boxes_rot(boxes):
    """boxes: iterable of (center(3), half(3), yaw or quaternion) -> ctypes rp_box_rot array."""
    boxes = list(boxes)
    arr = (BoxRot * max(1, len(boxes)))()
    for i, (c, h, rot) in enumerate(boxes):
        arr[i].center[:] = [float(v) for v in c]
        arr[i].half[:] = [float(v) for v in h]
        arr[i].quat[:] = list(quat_of(rot))
    return arr, len(boxes)


def scene_boxes(boxes):
    """The records of a scene's boxes for the library / the oracle: ("yaw", rp_box
    array, n) when every box is upright (rp_set_scene), else ("rot", rp_box_rot array,
    n) with every box as a quaternion (rp_set_scene_rot)."""
    boxes = list(boxes)
    if any(is_quat(b[2]) for b in boxes):
        return ("rot",) + make_boxes_rot(boxes)
    return ("yaw",) + make_boxes(boxes)


def set_params(p, seed, batch, timeout_s, n_waypoints, simplify, tree_capacity, straight_first, batch_min=0):
    """Refill the per-query fields of a reused PlanParams (planning.plan_path)."""
    p.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    p.batch = int(batch)
    p.batch_min = int(batch_min)
    p.timeout_s = float(timeout_s)
    p.n_waypoints = int(n_waypoints or 0)
    p.simplify = 1 if simplify else 0
    p.tree_capacity = int(tree_capacity)
    p.straight_first = 0 if straight_first else -1
    return p


def make_params(seed=0, batch=4096, range_=0.0, resolution=0.0, timeout_s=5.0, max_iters=0, batch_min=0,
                n_waypoints=100, simplify=True, tree_capacity=0, straight_first=True, chunk=0, group_repl=0):
    p = PlanParams()
    p.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    p.batch = int(batch)
    p.batch_min = int(batch_min)
    p.range = float(range_)
    p.resolution = float(resolution)
    p.timeout_s = float(timeout_s)
    p.max_iters = int(max_iters)
    p.n_waypoints = int(n_waypoints or 0)
    p.simplify = 1 if simplify else 0
    p.tree_capacity = int(tree_capacity)
    p.straight_first = 0 if straight_first else -1   # 0 = default (on with simplification)
    p.chunk = int(chunk)   # first sub-batch of an iteration (execution only; 0 = 64, < 0 = none)
    p.group_repl = int(group_repl)   # rank groups: replicated iterations up to this size (0 = 4096, < 0 = none)
    return p
