"""Golden fixtures produced by running the REFERENCE's own code/planning.py.

    python tests/golden/make_reference_fixtures.py   (needs /root/reference; run here only)

genesis and ompl are absent from this container, so they are replaced by small
stubs (sys.modules) that record calls; the reference's Python control flow and its
pair-filter arithmetic (code/planning.py:209-230) then run unmodified. Outputs
(tests/golden/reference_fixtures.json):
  * exemption truth table: contact-pair lists -> _is_ompl_state_valid result
  * plan_path call order and return contract (waypoint count / dtype / shape)
  * bounds semantics: float32 limits vs a float64 finger value of 0.04
No reference source is copied; only inputs and outputs are stored.
"""
import itertools
import json
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference/code"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_fixtures.json")

CALLS = []


def _install_stubs():
    gs = types.ModuleType("genesis")
    gs.tc_float = torch.float32
    gs.device = torch.device("cpu")

    class _Log:
        def warning(self, m):
            CALLS.append(("warning", str(m)))

        def info(self, m):
            CALLS.append(("info", str(m)))

    gs.logger = _Log()

    class GenesisException(Exception):
        pass

    def raise_exception(msg):
        raise GenesisException(msg)

    gs.GenesisException = GenesisException
    gs.raise_exception = raise_exception
    utils = types.ModuleType("genesis.utils")
    misc = types.ModuleType("genesis.utils.misc")
    misc.tensor_to_array = lambda x: x.detach().cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x)
    utils.misc = misc
    gs.utils = utils
    sys.modules["genesis"] = gs
    sys.modules["genesis.utils"] = utils
    sys.modules["genesis.utils.misc"] = misc

    # recording OMPL stub: RRTConnect "solves" with a 2-state path
    ompl = types.ModuleType("ompl")
    ob = types.ModuleType("ompl.base")
    og = types.ModuleType("ompl.geometric")
    ou = types.ModuleType("ompl.util")
    ou.LOG_ERROR = 3
    ou.setLogLevel = lambda lvl: CALLS.append(("setLogLevel", lvl))

    class RealVectorBounds:
        def __init__(self, n):
            self.low = [0.0] * n
            self.high = [0.0] * n

        def setLow(self, i, v):
            self.low[i] = v

        def setHigh(self, i, v):
            self.high[i] = v

    class RealVectorStateSpace:
        def __init__(self, n):
            CALLS.append(("RealVectorStateSpace", n))
            self.n = n

        def setBounds(self, b):
            CALLS.append(("setBounds", list(b.low), list(b.high)))
            self.b = b

        def getBounds(self):
            return self.b

    class _Raw(list):
        pass

    class State:
        def __init__(self, space):
            self.v = _Raw([0.0] * space.n)

        def __setitem__(self, i, x):
            self.v[i] = x

        def __getitem__(self, i):
            return self.v[i]

        def get(self):
            return self.v

    class SpaceInformation:
        def __init__(self, space):
            self.space = space
            self.fn = None

        def satisfiesBounds(self, s):
            b = self.space.b
            eps = np.finfo(np.float64).eps
            r = all(not (s[i] - eps > b.high[i] or s[i] + eps < b.low[i]) for i in range(self.space.n))
            CALLS.append(("satisfiesBounds", r))
            return r

        def isValid(self, s):
            r = bool(self.fn(s))
            CALLS.append(("isValid", r))
            return r

        def getStateSpace(self):
            return self.space

    class Path:
        def __init__(self, a, b):
            self.states = [a, b]

        def interpolate(self, n):
            CALLS.append(("interpolate", n))
            a, b = np.array(self.states[0]), np.array(self.states[-1])
            self.states = [list(a + (b - a) * (i / (n - 1))) for i in range(n)]

        def getStateCount(self):
            return len(self.states)

        def getStates(self):
            return self.states

    class SimpleSetup:
        def __init__(self, space):
            CALLS.append(("SimpleSetup",))
            self.si = SpaceInformation(space)

        def setStateValidityChecker(self, fn):
            CALLS.append(("setStateValidityChecker",))
            self.si.fn = fn

        def setPlanner(self, p):
            CALLS.append(("setPlanner", type(p).__name__))

        def getSpaceInformation(self):
            return self.si

        def setStartAndGoalStates(self, s, g):
            CALLS.append(("setStartAndGoalStates",))
            self.s, self.g = list(s.get()), list(g.get())

        def setup(self):
            CALLS.append(("setup",))

        def solve(self, t):
            CALLS.append(("solve", t))
            return True

        def getSolutionPath(self):
            CALLS.append(("getSolutionPath",))
            self.path = Path(self.s, self.g)
            return self.path

        def simplifySolution(self):
            CALLS.append(("simplifySolution",))

    ob.StateValidityCheckerFn = lambda f: f
    ob.RealVectorStateSpace = RealVectorStateSpace
    ob.RealVectorBounds = RealVectorBounds
    ob.State = State
    og.SimpleSetup = SimpleSetup
    for name in ["PRM", "RRT", "RRTConnect", "RRTstar", "EST", "FMT", "BITstar", "ABITstar"]:
        setattr(og, name, type(name, (), {"__init__": lambda self, si: None}))
    ompl.base, ompl.geometric, ompl.util = ob, og, ou
    sys.modules.update({"ompl": ompl, "ompl.base": ob, "ompl.geometric": og, "ompl.util": ou})


LINK_OF_GEOM = {0: "plane", 1: "box_r", 2: "box_g", 3: "box_b", 4: "box_y", 5: "box_m", 6: "box_c",
                7: "link0", 8: "link1", 9: "link2", 10: "link3", 11: "link4", 12: "link5", 13: "link6",
                14: "link7", 15: "hand", 16: "left_finger", 17: "right_finger"}


class _Link:
    def __init__(self, n):
        self.name = n


class _Geom:
    def __init__(self, n):
        self.link = _Link(n)


class FakeScene:
    def __init__(self):
        self.rigid_solver = types.SimpleNamespace(geoms=[_Geom(LINK_OF_GEOM[i]) for i in range(18)])


class FakeRobot:
    """plane = entity/geom 0, boxes 1..6, robot geoms 7..17."""

    def __init__(self, q_limit):
        self.n_qs = 9
        self.n_dofs = 9
        self._solver = types.SimpleNamespace(n_envs=0)
        self.q_limit = q_limit
        self.q = torch.zeros(9)
        self.pairs = np.zeros((0, 2), dtype=np.int32)

    def get_qpos(self):
        return self.q.clone()

    def set_qpos(self, q):
        CALLS.append(("set_qpos",))
        self.q = torch.as_tensor(q, dtype=torch.float32).clone()

    def detect_collision(self):
        return self.pairs


def main():
    _install_stubs()
    sys.path.insert(0, REF)
    import planning  # the reference module

    lo = np.array([-2.8973, -1.7628, -2.8973, -3.0718, -2.8973, -0.0175, -2.8973, 0.0, 0.0], np.float32)
    hi = np.array([2.8973, 1.7628, 2.8973, -0.0698, 2.8973, 3.7525, 2.8973, 0.04, 0.04], np.float32)
    robot = FakeRobot((lo, hi))
    scene = FakeScene()
    pi = planning.PlannerInterface(robot, scene)

    # 1. exemption truth table over pair lists
    cases = []
    attached_idx = 3  # box_b
    singles = [(3, 17), (17, 3), (3, 15), (16, 3), (0, 17), (4, 16), (1, 7), (3, 14), (3, 10), (2, 15), (0, 7),
               (14, 16)]
    pair_lists = [[]] + [[p] for p in singles] + [list(c) for c in itertools.combinations(singles, 2)]
    for att in (None, attached_idx):
        pi.attached_object = types.SimpleNamespace(idx=att) if att is not None else None
        for pl in pair_lists:
            robot.pairs = np.array(pl, dtype=np.int32).reshape(-1, 2)
            v = pi._is_ompl_state_valid([0.0] * 9)
            cases.append({"attached": att, "pairs": [[LINK_OF_GEOM[a], a, LINK_OF_GEOM[b], b] for a, b in pl],
                          "valid": bool(v)})

    # 2. plan_path control flow + return contract (stub OMPL)
    robot.pairs = np.zeros((0, 2), dtype=np.int32)
    CALLS.clear()
    start = np.array([0.0, -0.785, 0.0, -2.356, 0.0, 1.571, 0.785, 0.039, 0.039])
    goal = start.copy()
    goal[0] = 0.5
    wps = pi.plan_path(qpos_goal=goal, qpos_start=start, num_waypoints=150, timeout=10.0)
    flow = [c[0] for c in CALLS if c[0] not in ("info",)]
    contract = {"n": len(wps), "dtype": str(wps[0].dtype), "shape": list(wps[0].shape),
                "first": [float(v) for v in wps[0]], "last": [float(v) for v in wps[-1]]}

    # 3. bounds: float32 q_limit vs finger 0.04
    CALLS.clear()
    start2 = start.copy()
    start2[7:] = 0.04
    pi.plan_path(qpos_goal=goal, qpos_start=start2, num_waypoints=150)
    bounds_calls = [list(c) for c in CALLS if c[0] in ("satisfiesBounds", "warning")]

    # 4. errors
    errors = {}
    for kw, label in [({"planner": "Foo"}, "bad_planner")]:
        try:
            pi.plan_path(qpos_goal=goal, qpos_start=start, **kw)
            errors[label] = None
        except Exception as e:  # noqa: BLE001
            errors[label] = str(e)
    try:
        pi.plan_path(qpos_goal=goal[:7], qpos_start=start)
        errors["bad_shape"] = None
    except Exception as e:  # noqa: BLE001
        errors["bad_shape"] = str(e)

    out = {"about": __doc__.strip().splitlines()[0], "exemption_cases": cases, "plan_flow": flow,
           "return_contract": contract, "bounds_f32_finger_004": bounds_calls, "errors": errors,
           "q_limit_f32": [lo.astype(float).tolist(), hi.astype(float).tolist()]}
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {OUT}: {len(cases)} exemption cases, flow {flow}")


if __name__ == "__main__":
    main()
