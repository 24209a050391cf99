"""Genesis-free mock robot/scene exposing exactly what planning.py reads
(SURVEY.md §4 item 5): n_qs, n_dofs, q_limit, get_qpos/set_qpos, get_pos,
_solver.n_envs, and scene.entities with Box/Plane morphs and poses; with
`rigid_solver=True` also Genesis' batched link-pose reads
(scene.rigid_solver.get_links_pos / get_links_quat over entity.base_link_idx)."""
import math

import numpy as np
import torch

from rbe550_final_project_amd import model


class Box:
    def __init__(self, size, pos):
        self.size = tuple(size)
        self.pos = tuple(pos)


class Plane:
    def __init__(self):
        self.pos = (0.0, 0.0, 0.0)


class MJCF:
    def __init__(self, file):
        self.file = file


class Entity:
    def __init__(self, idx, morph, yaw=0.0):
        """yaw: a rotation about z, or a quaternion (w, x, y, z) (a tilted box)."""
        self.idx = idx
        self.base_link_idx = idx   # one link per entity here (the robot's base link)
        self.morph = morph
        self._pos = np.array(getattr(morph, "pos", (0, 0, 0)), dtype=float)
        if hasattr(yaw, "__len__"):
            self._quat = np.array([float(v) for v in yaw])
        else:
            self._quat = np.array([math.cos(yaw / 2), 0.0, 0.0, math.sin(yaw / 2)])

    def set_quat(self, q):
        self._quat = np.asarray(q, dtype=float)

    def get_pos(self):
        return torch.tensor(self._pos, dtype=torch.float32)

    def get_quat(self):
        return torch.tensor(self._quat, dtype=torch.float32)

    def set_pos(self, p):
        self._pos = np.asarray(p, dtype=float)


class Robot(Entity):
    def __init__(self, idx, n_envs=0, n_dofs=9):
        super().__init__(idx, MJCF("xml/franka_emika_panda/panda.xml"))
        self._pos = np.array(model.BASE_POS)
        self.n_qs = 9
        self.n_dofs = n_dofs
        self._solver = type("S", (), {"n_envs": n_envs})()
        self.q_limit = (model.Q_LO_SPEC.astype(np.float32), model.Q_HI_SPEC.astype(np.float32))
        self.q = torch.tensor(model.SAFE_HOME, dtype=torch.float32).clamp(max=float(np.float32(0.04)))
        self.set_calls = []

    def get_qpos(self):
        return self.q.clone()

    def set_qpos(self, q):
        self.set_calls.append(torch.as_tensor(q).clone())
        self.q = torch.as_tensor(q, dtype=torch.float32).clone()


class RigidSolver:
    """scene.rigid_solver's link-pose reads: one (n, 3) / (n, 4) float32 tensor per
    call, as Genesis returns for n links of an unbatched scene."""

    def __init__(self, scene):
        self._scene = scene

    def get_links_pos(self, links_idx=None):
        ents = self._scene.entities
        return torch.tensor(np.stack([ents[i]._pos for i in links_idx]), dtype=torch.float32)

    def get_links_quat(self, links_idx=None):
        ents = self._scene.entities
        return torch.tensor(np.stack([ents[i]._quat for i in links_idx]), dtype=torch.float32)


class Scene:
    """plane (entity 0), boxes (1..n), robot (n+1) — the order of code/scenes.py."""

    def __init__(self, boxes, rigid_solver=True, **robot_kw):
        self.entities = [Entity(0, Plane())]
        for i, (c, h, yaw) in enumerate(boxes):
            self.entities.append(Entity(i + 1, Box([2 * v for v in h], c), yaw))
        self.robot = Robot(len(self.entities), **robot_kw)
        self.entities.append(self.robot)
        if rigid_solver:
            self.rigid_solver = RigidSolver(self)
