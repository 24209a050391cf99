"""Drop-in replacement of the reference's code/planning.py (PlannerInterface).

Same class, same constructor, same plan_path signature and return contract as
code/planning.py:24-242, so code/motion_primitives.py:38/144 and the goal*.py
scripts run unchanged. The OMPL RRTConnect + per-state Python/Genesis callback
(planning.py:98-219) is replaced by one call into librbe_mi355x.so: batched
RRT-Connect whose validity checks (FK + capsule collision), edge checks and
nearest-neighbour searches run as HIP kernels on an MI355X.

Reference behaviour kept (file:line of code/planning.py):
  * planner name / batched-env / free-joint / shape checks raise    108-135
  * bounds = robot.q_limit, as float64 of the stored values         139-150
  * self.attached_object set; its box exempt for hand/fingers       153, 221-230
  * start/goal bound + validity diagnostics only warn                164-183
  * invalid start/goal or no solution -> [] + warning               190-202
  * EXACT and APPROXIMATE solutions are "solved"                     192
  * simplify when smooth_path, then interpolate(num_waypoints)       195-199
  * robot qpos restored at the end                                   205
  * returns a list of float32 tensors of shape (n_qs,)               232-242
    (CPU tensors: motion_primitives.py:176 calls np.array on them)

Not kept: the OMPL import, and planners other than RRTConnect (they are served by
the MI355X RRT-Connect with a warning; every reference call site uses RRTConnect).

Seeding (the reference is unseeded, scenes.py:9 / motion_primitives.py:153): the
seed is RBE_PLANNER_SEED (default 0) plus a per-process query counter, or set with
configure(seed=...). Batch size: RBE_PLANNER_BATCH / configure(batch=...).
"""
from __future__ import annotations

import logging
import os
import time
from typing import Any

import numpy as np
import torch

try:  # the real simulator, when present (the goal*.py scripts)
    import genesis as gs  # type: ignore
except Exception:  # pragma: no cover - Genesis is absent in CI
    gs = None

from . import _abi, model, scenes
from .native import Context, NativeError

_log = logging.getLogger("rbe550_final_project_amd.planning")

SUPPORTED_PLANNERS = ["PRM", "RRT", "RRTConnect", "RRTstar", "EST", "FMT", "BITstar", "ABITstar"]


class PlanningError(Exception):
    """Raised where the reference calls gs.raise_exception."""


def _raise(msg):
    if gs is not None and hasattr(gs, "raise_exception"):
        gs.raise_exception(msg)
    raise PlanningError(msg)


def _logger():
    if gs is not None and getattr(gs, "logger", None) is not None:
        return gs.logger
    return _log


_CONFIG = {"seed": None, "batch": None, "device": None, "tree_capacity": None, "straight_first": None,
           "devices": None, "batch_min": None}
_QUERY_COUNTER = [0]


def configure(seed=None, batch=None, device=None, tree_capacity=None, straight_first=None, devices=None,
              batch_min=None):
    """Set planner options without changing plan_path's signature.

    batch_min: samples of the first RRT-Connect iteration (each next one doubles, up
    to `batch`); 0 = the library default (min(batch, 64)).
    straight_first: with smooth_path, try the straight edge start -> goal before
    RRT-Connect (default on; env RBE_PLANNER_STRAIGHT=0 turns it off).
    devices: GPUs of a multi-GPU planner in this one process (env
    RBE_PLANNER_DEVICES="0,1,2,3"): a PlannerInterface opens one context per entry
    and every plan_path query runs as a rank group over them (rp_group_init_local:
    RCCL between distinct GPUs, a shared pinned segment when a device repeats); each
    RRT-Connect iteration's large sub-batches are sharded, the returned path is rank
    0's (every rank grows the same trees). () or None: one GPU (`device`)."""
    if devices is not None:
        _CONFIG["devices"] = tuple(int(d) for d in devices) or None
    if batch_min is not None:
        _CONFIG["batch_min"] = int(batch_min)
    if seed is not None:
        _CONFIG["seed"] = int(seed)
        _QUERY_COUNTER[0] = 0
    if batch is not None:
        _CONFIG["batch"] = int(batch)
    if device is not None:
        _CONFIG["device"] = int(device)
    if tree_capacity is not None:
        _CONFIG["tree_capacity"] = int(tree_capacity)
    if straight_first is not None:
        _CONFIG["straight_first"] = bool(straight_first)


def _straight_first():
    if _CONFIG["straight_first"] is not None:
        return _CONFIG["straight_first"]
    return os.environ.get("RBE_PLANNER_STRAIGHT", "1") not in ("0", "false", "False", "")


def _next_seed():
    base = _CONFIG["seed"]
    if base is None:
        base = int(os.environ.get("RBE_PLANNER_SEED", "0"))
    s = base + _QUERY_COUNTER[0]
    _QUERY_COUNTER[0] += 1
    return s


def _batch():
    if _CONFIG["batch"] is not None:
        return _CONFIG["batch"]
    return int(os.environ.get("RBE_PLANNER_BATCH", "4096"))


def _device():
    if _CONFIG["device"] is not None:
        return _CONFIG["device"]
    if "LOCAL_RANK" in os.environ:
        return int(os.environ["LOCAL_RANK"])
    return 0


def _devices():
    """The planner's GPUs: configure(devices=...), RBE_PLANNER_DEVICES, else one."""
    if _CONFIG["devices"]:
        return tuple(_CONFIG["devices"])
    e = os.environ.get("RBE_PLANNER_DEVICES", "").strip()
    if e:
        return tuple(int(x) for x in e.split(",") if x.strip())
    return (_device(),)


def tensor_to_array(x):
    """genesis.utils.misc.tensor_to_array equivalent (planning.py:10, 131-132)."""
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    return np.asarray(x)


def _ensure_adapter(robot: Any, scene: Any):
    """planning.py:14-22: wrap the raw entity in RobotAdapter if needed."""
    try:
        from robot_adapter import RobotAdapter  # the reference's own module (code/)
    except Exception:
        RobotAdapter = _Adapter
    if isinstance(robot, (RobotAdapter, _Adapter)):
        return robot
    return RobotAdapter(robot, scene)


class _Adapter:
    """Attribute-forwarding wrapper used when the reference's robot_adapter module
    is not on the path."""

    def __init__(self, robot, scene=None):
        self.robot = robot
        self.scene = scene

    def __getattr__(self, name):
        return getattr(self.robot, name)

    def get_qpos(self):
        return self.robot.get_qpos()

    def set_qpos(self, qpos):
        return self.robot.set_qpos(qpos)

    def detect_collision(self, *a, **k):
        return self.robot.detect_collision(*a, **k)


class _Bounds:
    def __init__(self, lo, hi):
        self.low = list(lo)
        self.high = list(hi)


class _SpaceInfo:
    """Minimal stand-in for OMPL's SpaceInformation used by the diagnostics."""

    def __init__(self, lo, hi):
        self._b = _Bounds(lo, hi)

    def getStateSpace(self):
        return self

    def getBounds(self):
        return self._b


def _f64(x):
    """float64 copy of a qpos (torch tensor or array-like); tensor_to_array + asarray."""
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy().astype(np.float64)
    return np.array(x, dtype=np.float64)


class PlannerInterface:
    def __init__(self, robot: Any, scene: Any):
        self.robot = _ensure_adapter(robot, scene)
        self.scene = scene
        self.attached_object = None
        self._ctx = None         # rank 0's context (diagnostics, IK, single-state checks)
        self._ctxs = []          # every rank's context (configure(devices=...)), rank order
        self._devs = None
        self._reader = None      # scenes.GenesisReader of self.scene
        self._pushed = None      # (ctx.scene_gen, box poses, base, attached box) last pushed
        self._qlim = None        # (robot.q_limit object, lo, hi)
        self._params = None
        self._reserved = None
        self._stats_ctx = None
        self._times = None
        self.last_status = None

    # -- GPU context -----------------------------------------------------------
    def _context(self):
        devs = _devices()
        if self._ctx is not None and (not self._ctxs or devs == self._devs):
            return self._ctx   # (also a context handed in from outside: bench.py)
        for c in self._ctxs:
            c.close()
        self._ctxs = [Context(device=d, robot=model.robot_desc()) for d in devs]
        if len(self._ctxs) > 1:
            from .native import group_init_local
            group_init_local(self._ctxs)
        self._ctx = self._ctxs[0]
        self._devs = devs
        self._pushed = None
        self._reserved = None
        return self._ctx

    def _reform_group(self):
        """A failed grouped plan leaves every rank's group broken (rp_plan refuses
        RP_ERR_EXCHANGE until the group is initialised again): re-form it, so that
        one HIP or watchdog error costs this query only, not every later one. If
        that fails too, drop the contexts; the next query opens fresh ones."""
        from .native import group_init_local
        try:
            group_init_local(self._ctxs)
        except NativeError as ex:
            _logger().warning(f"MI355X planner: re-forming the rank group failed ({ex}); reopening the contexts")
            for c in self._ctxs:
                try:
                    c.close()
                except Exception:   # noqa: BLE001 - a dead context is dropped either way
                    pass
            self._ctxs = []
            self._ctx = None
            self._devs = None
            self._pushed = None
        self._reserved = None

    def _reserve(self, ctx, batch, cap):
        """Workspace for this batch / tree capacity sized once (rp_reserve), so the
        first query does not allocate device memory inside the plan."""
        key = (id(ctx), batch, cap)
        if self._reserved != key and hasattr(ctx, "reserve"):
            for c in self._ctxs or [ctx]:
                c.reserve(batch, cap)
            self._reserved = key

    def _sync_scene(self):
        """Push the obstacle geometry (boxes at their simulated poses) and the attached
        box to the GPU context. The poses are read on every call (the simulation may
        have moved a block); the context is updated only when they, the attachment or
        the context's scene (someone else set one) changed."""
        rd = self._reader
        if rd is None or not rd.valid_for(self.scene, self.robot):
            rd = self._reader = scenes.GenesisReader(self.scene, self.robot)
            self._pushed = None
            self._scene_names = rd.names
        poses, base = rd.poses()
        ctx = self._context()
        idx = -1
        att = self.attached_object
        if att:
            idx = rd.box_of_entity.get(getattr(att, "idx", None), -1)
        gen = getattr(ctx, "scene_gen", None)
        pushed = self._pushed
        ctxs = self._ctxs or [ctx]   # every rank of a multi-GPU planner sees the same scene
        if gen is not None and pushed is not None and pushed[0] == gen and pushed[2] == base \
                and np.array_equal(pushed[1], poses):
            if pushed[3] != idx:
                for c in ctxs:
                    c.set_attached(idx)
                self._pushed = (ctx.scene_gen, poses, base, idx)
            return
        if hasattr(ctx, "set_scene_poses"):   # one library call (rp_set_scene_poses)
            P = np.ascontiguousarray(poses, dtype=np.float64).reshape(-1, 7)
            B = np.array(base, dtype=np.float64)
            for c in ctxs:
                c.set_scene_poses(P, rd.halves_f32, rd.plane_z, B, idx)
        else:
            for c in ctxs:
                c.set_scene(rd.boxes(poses), rd.plane_z, base)
                c.set_attached(idx)
        self._pushed = (getattr(ctx, "scene_gen", None), poses, base, idx)

    def _bounds(self):
        """planning.py:139-150: bounds = the robot's q_limit as float64 (of the stored
        float32 values); converted once per q_limit object."""
        ql = self.robot.q_limit
        c = self._qlim
        if c is None or c[0] is not ql:
            lo = np.asarray(tensor_to_array(ql[0]), dtype=float)
            hi = np.asarray(tensor_to_array(ql[1]), dtype=float)
            c = self._qlim = (ql, lo, hi)
        return c[1], c[2]

    @property
    def last_stats(self):
        """rp_get_stats of this planner's last query (None if it failed in the library)."""
        return self._stats_ctx.stats() if self._stats_ctx is not None else None

    @property
    def last_timing(self):
        """Where the last plan_path call's wall time went (ms): scene ingestion (entity
        poses -> boxes, rp_set_scene / rp_set_attached when they changed), rp_plan
        (from rp_plan_async to rp_plan_wait's return: the GPU query, with the waypoint
        tensors and the qpos restore overlapped), and everything else (argument
        checks, bounds, diagnostics, the output list)."""
        if self._times is None:
            return None
        t0, t1, t2, t3, t4 = self._times
        total = 1e3 * (t4 - t0)
        return {"total_ms": total, "scene_ms": 1e3 * (t1 - t0), "rp_plan_ms": 1e3 * (t3 - t2),
                "other_ms": total - 1e3 * (t1 - t0) - 1e3 * (t3 - t2)}

    # -- diagnostics (planning.py:32-57) ----------------------------------------
    def diagnose_bounds_violation(self, si, state):
        violated = []
        b = si.getStateSpace().getBounds()
        for i_q in range(self.robot.n_qs):
            val = state[i_q]
            low, high = b.low[i_q], b.high[i_q]
            if val < low or val > high:
                violated.append((i_q, val, low, high))
        _logger().warning(f"State violates bounds on joints: {violated}")

    def diagnose_valid_violation(self, state):
        pairs = self._context().contacts(np.asarray([float(state[i]) for i in range(self.robot.n_qs)]))
        bad = set()
        for link, obst in pairs:
            bad.add(_abi.LINK_NAMES[link])
            if obst == -1:
                bad.add("plane")
            elif obst >= 0:
                bad.add(f"box{obst}")
            else:
                bad.add(_abi.LINK_NAMES[-2 - obst])
        _logger().warning(f"State causes collisions between links: {sorted(bad)}")

    # -- the query (planning.py:59-207) -----------------------------------------
    def plan_path(self, qpos_goal, qpos_start=None, timeout=5.0, smooth_path=True, num_waypoints=100,
                  attached_object=None, planner="RRTConnect"):
        t_enter = time.perf_counter()
        if planner != "RRTConnect":
            if planner not in SUPPORTED_PLANNERS:
                _raise(f"Planner {planner} is not supported. Supported planners: {SUPPORTED_PLANNERS}.")
            _logger().warning(f"Planner {planner} is served by the MI355X batched RRT-Connect.")
        robot = self.robot
        solver = getattr(robot, "_solver", None)
        if solver is not None and getattr(solver, "n_envs", 0) > 0:
            _raise("Motion planning is not supported for batched envs (yet).")
        n_qs = robot.n_qs
        if n_qs != robot.n_dofs:
            _raise("Motion planning is not yet supported for rigid entities with free joints.")

        # planning.py:129-133 reads get_qpos() twice (current, and the start when none
        # is given): one read serves both
        qpos_cur = robot.get_qpos()
        qpos_start = _f64(qpos_cur if qpos_start is None else qpos_start)
        qpos_goal = _f64(qpos_goal)
        if qpos_start.shape != (n_qs,) or qpos_goal.shape != (n_qs,):
            _raise("Invalid shape for `qpos_start` or `qpos_goal`.")
        if n_qs != _abi.NQ:
            _raise(f"The MI355X planner is built for the 9-D Franka Panda (got n_qs={n_qs}).")
        lo, hi = self._bounds()

        self.attached_object = attached_object
        ctx = self._context()
        self._sync_scene()
        t_scene = time.perf_counter()

        p = self._params
        if p is None:
            p = self._params = _abi.make_params()
        world = len(self._ctxs) or 1
        batch = -(-_batch() // world) * world   # a rank group shards whole batches
        _abi.set_params(p, seed=_next_seed(), batch=batch, timeout_s=float(timeout),
                        n_waypoints=int(num_waypoints) if num_waypoints else 0, simplify=bool(smooth_path),
                        tree_capacity=_CONFIG["tree_capacity"] or 0, straight_first=_straight_first(),
                        batch_min=_CONFIG["batch_min"] or 0)
        self._reserve(ctx, p.batch, p.tree_capacity)
        nwp = p.n_waypoints
        cap = max(4096, nwp + 16)
        t_plan0 = time.perf_counter()
        path = out = None
        status = _abi.STATUS_NONE
        restored = False
        self._stats_ctx = None
        ranks = self._ctxs if len(self._ctxs) > 1 else [ctx]
        started = []
        views = None
        try:
            try:
                # every rank's query on its context's planner thread (a rank group
                # meets at its exchanges); rank 0's path is the answer
                for c in ranks:
                    c.plan_async(qpos_start, qpos_goal, lo, hi, p, path_cap=cap)
                    started.append(c)
                # while the GPU plans: the waypoint tensors of the expected path (an
                # interpolated solution has exactly num_waypoints states) and the
                # restore of the robot's qpos (planning.py:205; the planner never
                # moves the robot)
                if nwp > 0:
                    buf = torch.empty((nwp, n_qs), dtype=torch.float32)
                    views = buf.unbind(0)
                    out = buf.numpy()
                robot.set_qpos(qpos_cur)
                restored = True
            finally:
                err = None
                for k, c in enumerate(started):   # every started rank is waited for
                    try:
                        r = c.plan_wait(out if k == 0 else None)
                        if k == 0:
                            path, status = r
                    except NativeError as ex:
                        err = err or ex
                if err is not None:
                    raise err
            self._stats_ctx = ctx
        except NativeError as ex:
            # the reference never raises on a failed plan (planning.py:190-202):
            # a library error (capacity, HIP) is reported and planning "fails"
            _logger().warning(f"MI355X planner error: {ex}")
            path, status = None, _abi.STATUS_NONE
            if len(self._ctxs) > 1:
                self._reform_group()
                if self._ctx is None:   # reopened: the diagnostics below need a context with the scene
                    try:
                        ctx = self._context()
                        self._sync_scene()
                    except NativeError:
                        ctx = None
        t_plan1 = time.perf_counter()
        self.last_status = status

        if status in (_abi.STATUS_INVALID_START, _abi.STATUS_INVALID_GOAL) or path is None:
            self._diagnose(ctx, qpos_start, qpos_goal, lo, hi)

        waypoints = []
        if status in (_abi.STATUS_EXACT, _abi.STATUS_APPROXIMATE):
            _logger().info("Path solution found successfully.")
            print("Number of waypoints in path:", len(path))
            waypoints = list(views) if path is out and out is not None else self._states_to_tensor_list(path)
        else:
            _logger().warning("Path planning failed. Returning empty path.")
        if not restored:
            robot.set_qpos(qpos_cur)
        self._times = (t_enter, t_scene, t_plan0, t_plan1, time.perf_counter())
        return waypoints

    def _diagnose(self, ctx, qpos_start, qpos_goal, lo, hi):
        """planning.py:164-183: bound and validity diagnostics of start and goal, run
        when the plan reports an invalid start / goal (rp_plan applies OMPL's bound
        and validity checks to both itself) or did not run."""
        si = _SpaceInfo(lo, hi)
        eps = np.finfo(np.float64).eps
        if not bool(np.all(qpos_start - eps <= hi) and np.all(qpos_start + eps >= lo)):
            _logger().warning("OMPL start state out of bounds")
            self.diagnose_bounds_violation(si, qpos_start)
        if not bool(np.all(qpos_goal - eps <= hi) and np.all(qpos_goal + eps >= lo)):
            _logger().warning("OMPL goal state out of bounds")
            self.diagnose_bounds_violation(si, qpos_goal)
        if ctx is not None:
            self._diagnose_start_goal(ctx, qpos_start, qpos_goal)

    def _diagnose_start_goal(self, ctx, qpos_start, qpos_goal):
        try:
            flags = ctx.check_states(np.stack([qpos_start, qpos_goal]).astype(np.float32))
        except NativeError as ex:
            _logger().warning(f"MI355X planner error: {ex}")
            return
        if not flags[0]:
            _logger().warning("OMPL start state invalid")
            self.diagnose_valid_violation(qpos_start)
        if not flags[1]:
            _logger().warning("OMPL goal state invalid")
            self.diagnose_valid_violation(qpos_goal)

    # -- goal configurations (motion_primitives.py:131-134) ----------------------
    def inverse_kinematics(self, pos, quat, init_qpos=None, n_seeds=256, iters=64, attached_object=None):
        """Hand-link IK on the GPU (rp_ik): the drop-in for the Genesis
        robot.inverse_kinematics(link=hand, pos, quat) that _ik_for_pose calls.
        Restarts from init_qpos (default: current qpos) and seeded samples, keeps the
        fingers of init_qpos, prefers a collision-free solution in the current scene.
        Returns a float32 CPU tensor (9,), or None if no restart reached the pose."""
        init = np.asarray(tensor_to_array(init_qpos if init_qpos is not None else self.robot.get_qpos()),
                          dtype=np.float64)
        lo = np.asarray(tensor_to_array(self.robot.q_limit[0]), dtype=float)
        hi = np.asarray(tensor_to_array(self.robot.q_limit[1]), dtype=float)
        self.attached_object = attached_object
        ctx = self._context()
        self._sync_scene()
        p = _abi.make_ik_params(seed=_next_seed(), n_seeds=n_seeds, iters=iters)
        q, st = ctx.ik(np.asarray(tensor_to_array(pos), dtype=np.float64)[None, :],
                       np.asarray(tensor_to_array(quat), dtype=np.float64)[None, :], init[None, :], lo, hi, p)
        self.last_ik_status = int(st[0])
        if st[0] == _abi.IK_NOT_CONVERGED:
            _logger().warning("IK did not reach the target pose.")
            return None
        if st[0] == _abi.IK_COLLIDING:
            _logger().warning("IK solution is in collision.")
        return torch.tensor(q[0], dtype=torch.float32)

    # -- single-state validity (planning.py:209-219) ------------------------------
    def _is_ompl_state_valid(self, state):
        """planning.py:209-219: checked against the live scene (box poses and the
        attached object as they are now), like the reference's set_qpos +
        detect_collision on every call."""
        q = np.asarray([float(state[i]) for i in range(_abi.NQ)], dtype=np.float32)
        self._sync_scene()
        return bool(self._context().check_states(q)[0])

    def collision_with_attached_object(self, collision_pairs):
        """planning.py:221-230 on a Genesis contact-pair list (kept for callers that
        use it directly; the GPU path applies the same rule per capsule)."""
        finger_names = {"left_finger", "right_finger", "hand"}
        geoms = self.scene.rigid_solver.geoms
        for a, b in collision_pairs:
            name_a = geoms[a].link.name
            name_b = geoms[b].link.name
            if (name_a in finger_names and b == self.attached_object.idx) or \
                    (name_b in finger_names and a == self.attached_object.idx):
                continue
            return False
        return True

    @staticmethod
    def _states_to_tensor_list(path):
        """planning.py:232-242: one float32 CPU tensor (n_qs,) per waypoint. The
        rows are views of one (n, n_qs) tensor made with a single conversion (150
        torch.tensor constructions cost ~0.8 ms, the views ~0.2 ms)."""
        return list(torch.from_numpy(np.ascontiguousarray(path, dtype=np.float32)).unbind(0))

    def _ompl_state_to_tensor(self, state):
        return torch.tensor([float(state[i]) for i in range(self.robot.n_qs)], dtype=torch.float32)
