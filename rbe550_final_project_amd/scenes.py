"""Obstacle scenes of the planning path: boxes + ground plane + robot base.

Scene factories transcribe the obstacle constants of code/scenes.py (the reference
builds Genesis scenes; here only the geometry the collider sees is kept):

  goal1_scattered   create_scene_6blocks      scenes.py:41-99  (6 boxes, +-5 cm xy jitter)
  goal3_tallest     create_scene_10blocks2ln  scenes.py:150-223 (10 boxes, no jitter)
  goal4_pentagon    create_scene_10blocks     scenes.py:226-299 (10 boxes, no jitter)
  clutter64         SURVEY.md §8(d) C5 synthetic clutter (64 floating boxes)

Every scene adds the plane first, then the boxes, then the robot, so box k of a
scene is Genesis entity k+1 (planning.py:226 compares attached_object.idx with geom
indices). The robot base is raised by 1 cm (scenes.py:29-34).

`from_genesis()` ingests a live Genesis scene (box entities and their current
poses, upright or toppled) so the drop-in planning.py sees the blocks where the
simulation has them.
"""
from dataclasses import dataclass, field
import json
import math

import numpy as np

BLOCK = 0.04                 # gs.morphs.Box(size=(0.04, 0.04, 0.04)) (scenes.py:60)
HALF = (BLOCK / 2, BLOCK / 2, BLOCK / 2)
BASE = (0.0, 0.0, 0.01)


def _rot_copy(rot):
    """A box orientation: a yaw (float) or a quaternion (w, x, y, z) tuple."""
    if hasattr(rot, "__len__"):
        return tuple(float(v) for v in rot)
    return float(rot)


@dataclass
class Scene:
    # [(center(3), half(3), rot)]: rot is the yaw about world z, or a quaternion
    # (w, x, y, z) for a tilted (toppled, leaning) box
    boxes: list = field(default_factory=list)
    names: list = field(default_factory=list)
    plane_z: float = 0.0
    base: tuple = BASE
    entity_idx: list = field(default_factory=list)  # Genesis entity index per box (or None)

    def copy(self):
        return Scene([(tuple(c), tuple(h), _rot_copy(y)) for c, h, y in self.boxes], list(self.names), self.plane_z,
                     tuple(self.base), list(self.entity_idx))

    def index(self, name):
        return self.names.index(name)

    def move(self, name, center, yaw=None, quat=None):
        """Move box `name`; yaw (float) or quat (w, x, y, z) sets its orientation."""
        i = self.index(name)
        c, h, y = self.boxes[i]
        rot = quat if quat is not None else (yaw if yaw is not None else y)
        self.boxes[i] = (tuple(float(v) for v in center), h, _rot_copy(rot))

    def remove(self, name):
        i = self.index(name)
        del self.boxes[i]
        del self.names[i]
        if self.entity_idx:
            del self.entity_idx[i]

    def to_json(self):
        out = []
        for n, (c, h, y) in zip(self.names, self.boxes):
            rec = {"name": n, "center": list(c), "half": list(h)}
            if hasattr(y, "__len__"):
                rec["quat"] = list(y)
            else:
                rec["yaw"] = y
            out.append(rec)
        return {"boxes": out, "plane_z": self.plane_z, "base": list(self.base)}

    @staticmethod
    def from_json(d):
        s = Scene(plane_z=float(d.get("plane_z", 0.0)), base=tuple(d.get("base", BASE)))
        for b in d["boxes"]:
            rot = tuple(float(v) for v in b["quat"]) if "quat" in b else float(b.get("yaw", 0.0))
            s.boxes.append((tuple(b["center"]), tuple(b["half"]), rot))
            s.names.append(b.get("name", f"box{len(s.names)}"))
        s.entity_idx = [i + 1 for i in range(len(s.boxes))]
        return s


def _mk(named_centers):
    s = Scene()
    for i, (n, c) in enumerate(named_centers):
        s.boxes.append((tuple(float(v) for v in c), HALF, 0.0))
        s.names.append(n)
        s.entity_idx.append(i + 1)
    return s


def goal1_scattered(seed=0, noise=0.05):
    """create_scene_6blocks (scenes.py:41-99) with the jitter seeded instead of
    random.seed(time.time()) (scenes.py:9)."""
    rng = np.random.default_rng(seed)
    nominal = [("r", (0.65, 0.0)), ("g", (0.65, 0.2)), ("b", (0.65, 0.4)),
               ("y", (0.45, 0.0)), ("m", (0.45, 0.2)), ("c", (0.45, 0.4))]
    out = []
    for n, (x, y) in nominal:
        dx, dy = rng.uniform(-noise, noise, 2)
        out.append((n, (x + dx, y + dy, 0.02)))
    return _mk(out)


def goal3_tallest():
    """create_scene_10blocks2ln (scenes.py:150-223)."""
    pos = [("r", (0.45, -0.40)), ("g", (0.45, -0.20)), ("b", (0.45, 0.00)), ("y", (0.45, 0.20)),
           ("o", (0.45, 0.40)), ("r2", (0.65, -0.40)), ("g2", (0.65, -0.20)), ("b2", (0.65, 0.00)),
           ("y2", (0.65, 0.20)), ("o2", (0.65, 0.40))]
    return _mk([(n, (x, y, 0.02)) for n, (x, y) in pos])


def goal4_pentagon():
    """create_scene_10blocks (scenes.py:226-299)."""
    pos = [(0.35, -0.40), (0.35, -0.25), (0.45, -0.30), (0.6, -0.40), (0.6, -0.25),
           (0.35, 0.40), (0.35, 0.25), (0.45, 0.30), (0.6, 0.40), (0.6, 0.25)]
    return _mk([(f"b{i + 1}", (x, y, 0.02)) for i, (x, y) in enumerate(pos)])


def pentagon_slots(center=(0.50, 0.10), radius=0.06):
    """Base and top slot poses of goal4_task1.py:66-126: (x, y, yaw_deg)."""
    base, top = [], []
    for i in range(5):
        a = 0.0 + i * 72.0
        x = center[0] + radius * math.cos(math.radians(a)) + 0.0045
        y = center[1] + radius * math.sin(math.radians(a))
        base.append((x, y, _wrap180(a)))
        a = i * 72.0 + 36.0
        x = center[0] + radius * math.cos(math.radians(a)) + 0.0053
        y = center[1] + radius * math.sin(math.radians(a)) - 0.0005
        top.append((x, y, _wrap180(a)))
    return base, top


def _wrap180(a):
    while a < -180:
        a += 360
    while a > 180:
        a -= 360
    return a


def clutter64(seed=0x64B0, n=64, keep_clear=None):
    """n boxes, centres x~U[0.25,0.85], y~U[-0.6,0.6],
    z~U[0.02,0.6], half extents U[0.01,0.05], yaw 0. `keep_clear(scene_with_one_box)`
    returns False to reject a box (e.g. one that collides with start/goal)."""
    rng = np.random.default_rng(seed)
    s = Scene()
    tries = 0
    while len(s.boxes) < n and tries < 100 * n:
        tries += 1
        c = (rng.uniform(0.25, 0.85), rng.uniform(-0.6, 0.6), rng.uniform(0.02, 0.6))
        h = tuple(rng.uniform(0.01, 0.05, 3))
        cand = ((float(c[0]), float(c[1]), float(c[2])), tuple(float(v) for v in h), 0.0)
        if keep_clear is not None and not keep_clear(cand):
            continue
        s.boxes.append(cand)
        s.names.append(f"k{len(s.names)}")
        s.entity_idx.append(len(s.names))
    return s


# ---------------------------------------------------------------------------
# Genesis ingestion (drop-in path)
# ---------------------------------------------------------------------------

def _to_np(x):
    if hasattr(x, "detach"):
        x = x.detach()
    if hasattr(x, "cpu"):
        x = x.cpu()
    if hasattr(x, "numpy"):
        x = x.numpy()
    return np.asarray(x, dtype=float).reshape(-1)


def _floats(x, n):
    """The first n values of a pose vector as Python floats: one .tolist() for a
    torch tensor (one device read when it lives on the GPU), else via numpy."""
    if hasattr(x, "tolist") and not isinstance(x, np.ndarray):
        v = x.tolist()
        if len(v) >= n and not isinstance(v[0], list):
            return [float(a) for a in v[:n]]
    return [float(a) for a in _to_np(x)[:n]]


def quat_upright(q):
    """An upright (w, x, y, z) quaternion: |x|, |y| <= 1e-7 |q|, a rotation about z to
    within simulation noise (rp_lib.hip quat_upright, the oracle's rule)."""
    w, x, y, z = (float(v) for v in q)
    t = 1e-7 * math.sqrt(w * w + x * x + y * y + z * z)
    return abs(x) <= t and abs(y) <= t


def yaw_of_quat(q):
    """Rotation about world z of an upright (w, x, y, z) quaternion (normalised first
    when its norm is not 1, as rp_set_scene_poses does)."""
    w, x, y, z = (float(v) for v in q)
    n2 = w * w + x * x + y * y + z * z
    if abs(n2 - 1.0) > 1e-12:
        n = math.sqrt(n2)
        w, x, y, z = w / n, x / n, y / n, z / n
    return math.atan2(2.0 * (w * z + x * y), 1.0 - 2.0 * (y * y + z * z))


def rot_of_quat(q):
    """A box orientation from a (w, x, y, z) quaternion: its yaw when the box is
    upright (quat_upright: exactly the record rp_set_scene_poses makes), else the
    quaternion itself (a tilted box; rp_set_scene_rot)."""
    w, x, y, z = (float(v) for v in q)
    if quat_upright((w, x, y, z)):
        return yaw_of_quat((w, x, y, z))
    return (w, x, y, z)


def _entity_table(entities, raw_robot, robot):
    """Per-entity static data: ("robot" | "plane" | "box" | None, payload). The box
    payload is (half extents, entity index); the plane's is its height."""
    table = []
    for ent in entities:
        morph = getattr(ent, "morph", None)
        kind = type(morph).__name__ if morph is not None else ""
        if ent is raw_robot or ent is robot:
            table.append(("robot", None))
        elif kind == "Plane":
            table.append(("plane", float(_to_np(getattr(morph, "pos", (0.0, 0.0, 0.0)))[2])))
        elif kind == "Box":
            size = getattr(morph, "size", None)
            if size is None:
                lo, hi = np.asarray(morph.lower, float), np.asarray(morph.upper, float)
                size = hi - lo
            half = tuple(float(v) / 2.0 for v in _to_np(size)[:3])
            table.append(("box", (half, getattr(ent, "idx", None))))
        else:
            table.append((None, None))
    return table


def _entities(scene):
    entities = getattr(scene, "entities", None)
    if entities is None and hasattr(scene, "sim"):
        entities = scene.sim.entities
    return entities if entities is not None else []


def _rows(x, n, k):
    """An (n, k) pose block (torch tensor / array, possibly with a leading env axis of
    1) as a float64 array: one device read for a GPU tensor, no per-value Python
    objects (the drop-in reads the poses on every plan_path call)."""
    if hasattr(x, "detach"):
        x = x.detach()
    if hasattr(x, "cpu") and not isinstance(x, np.ndarray):
        x = x.cpu().numpy()
    a = np.asarray(x, dtype=np.float64)
    while a.ndim > 2 and a.shape[0] == 1:
        a = a[0]
    if a.ndim == 1:
        a = a[None]
    return a[:n, :k]


class GenesisReader:
    """Reads the collider-relevant state of a live Genesis scene: every Box entity's
    pose, the robot base and the ground height (code/scenes.py builds them; the
    reference's collider sees them through set_qpos + detect_collision,
    code/planning.py:209-219).

    The entities' static data (morph kind, box half extents, plane height) is read
    once while the scene's entity list is the same objects. Poses are read per query:
    when the scene's rigid solver offers `get_links_pos` / `get_links_quat` and every
    box has a `base_link_idx`, with one call each for all boxes and the robot base
    (Genesis serves each entity.get_pos() with its own solver read); otherwise per
    entity with `get_pos()` / `get_quat()`."""

    def __init__(self, scene, robot=None):
        self.scene = scene
        entities = _entities(scene)
        self._ents_obj = entities
        self._ents = list(entities)
        raw_robot = getattr(robot, "robot", robot)
        self._raw_robot = raw_robot
        self._robot = robot
        table = _entity_table(self._ents, raw_robot, robot)
        self.box_ents, self.halves, self.entity_idx = [], [], []
        self.robot_ent = None
        self.plane_z = 0.0
        for ent, (kind, data) in zip(self._ents, table):
            if kind == "box":
                self.box_ents.append(ent)
                self.halves.append(data[0])
                self.entity_idx.append(data[1])
            elif kind == "robot":
                self.robot_ent = ent
            elif kind == "plane":
                self.plane_z = data
        self.halves_f32 = np.array(self.halves, dtype=np.float32).reshape(-1, 3)
        self.box_of_entity = {e: k for k, e in enumerate(self.entity_idx) if e is not None}
        self.names = [str(e if e is not None else k) for k, e in enumerate(self.entity_idx)]
        self._links = None
        solver = getattr(scene, "rigid_solver", None)
        if solver is not None and hasattr(solver, "get_links_pos") and hasattr(solver, "get_links_quat"):
            rsrc = self._raw_robot if self._raw_robot is not None else self.robot_ent
            links = [getattr(e, "base_link_idx", None) for e in self.box_ents]
            if rsrc is not None:
                links.append(getattr(rsrc, "base_link_idx", None))
            if all(isinstance(x, (int, np.integer)) for x in links):
                self._solver = solver
                self._nb = len(self.box_ents)
                self._with_base = rsrc is not None
                self._links = [int(x) for x in links]

    def valid_for(self, scene, robot):
        """Same scene, robot and entity objects as when the static data was read."""
        if scene is not self.scene or getattr(robot, "robot", robot) is not self._raw_robot:
            return False
        ents = _entities(scene)
        if ents is self._ents_obj and len(ents) == len(self._ents):
            return True
        ents = list(ents)
        return len(ents) == len(self._ents) and all(a is b for a, b in zip(ents, self._ents))

    def poses(self):
        """(box poses: an (n, 7) float64 array of rows [x, y, z, qw, qx, qy, qz], robot
        base (x, y, z))."""
        if self._links is not None:
            n = len(self._links)
            P = _rows(self._solver.get_links_pos(self._links), n, 3)
            Q = _rows(self._solver.get_links_quat(self._links), n, 4)
            boxes = np.concatenate([P[:self._nb], Q[:self._nb]], axis=1)
            base = tuple(P[self._nb].tolist()) if self._with_base else BASE
            return boxes, base
        rows = []
        for ent in self.box_ents:
            pos = _floats(ent.get_pos(), 3)
            quat = _floats(ent.get_quat(), 4) if hasattr(ent, "get_quat") else [1.0, 0.0, 0.0, 0.0]
            rows.append(pos + quat)
        boxes = np.array(rows, dtype=np.float64).reshape(-1, 7)
        base = BASE
        if self.robot_ent is not None and hasattr(self.robot_ent, "get_pos"):
            base = tuple(_floats(self.robot_ent.get_pos(), 3))
        robot = self._robot
        if robot is not None and robot is not self.robot_ent and hasattr(robot, "get_pos"):
            try:
                base = tuple(_floats(robot.get_pos(), 3))
            except Exception:
                pass
        return boxes, base

    def boxes(self, poses):
        """Box records (center, half, yaw or quaternion) of box poses from poses()."""
        return [((float(p[0]), float(p[1]), float(p[2])), h, rot_of_quat(p[3:7])) for p, h in zip(poses, self.halves)]

    def read(self):
        """The scene as a Scene record."""
        poses, base = self.poses()
        return Scene(self.boxes(poses), list(self.names), self.plane_z, base, list(self.entity_idx))


def from_genesis(scene, robot=None, cache=None):
    """Boxes of a Genesis scene: every entity whose morph is a Box, at its current
    pose (GenesisReader). cache: a dict owned by the caller (one per
    PlannerInterface) that keeps the reader while the scene's entities stay the same."""
    rd = cache.get("reader") if cache is not None else None
    if rd is None or not rd.valid_for(scene, robot):
        rd = GenesisReader(scene, robot)
        if cache is not None:
            cache["reader"] = rd
    return rd.read()


def load_json(path):
    with open(path) as f:
        return Scene.from_json(json.load(f))
