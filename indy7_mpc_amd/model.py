"""Robot model for the Indy7 SQP-MPC path: URDF parser + the pinocchio-like model surface.

The reference builds its model with ``pin.buildModelsFromUrdf(urdf_path, mesh_dir)``
(reference ``src/utils.py:20-21``) and then only touches ``model.nq``, ``model.nv``,
``len(model.joints)``, ``model.gravity.linear`` and ``model.createData()``
(``src/osqp_solver.py:9-20``, ``src/osqp_mpc.py:8-9``).  This module provides exactly that
surface without pinocchio, plus the packed parameter block the HIP kernels consume.

Conventions reproduced from pinocchio's URDF parser (semantics, not code):
  * the root link is the URDF root (``world``); fixed joints are merged into their parent
    body (their inertia is folded into the parent via the parallel-axis theorem);
  * each revolute joint becomes one joint frame whose placement in the parent joint frame
    is the composition of every fixed-joint origin on the way plus its own ``<origin>``;
  * URDF ``rpy`` -> R = Rz(yaw) @ Ry(pitch) @ Rx(roll);
  * a link's ``<inertial>`` gives mass, COM (in the link = joint frame) and the rotational
    inertia about the COM, rotated by the inertial ``rpy``.
The kernels assume every actuated joint rotates about its local +z axis (true for Indy7,
``description/indy7.urdf:201,208,215,222,229,236``); anything else is rejected loudly.
"""
from __future__ import annotations

import json
import math
import os
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

NJ = 6  # the kernels are specialised for a 6-DOF serial chain (Indy7)

_DEFAULT_PARAMS = os.path.join(os.path.dirname(__file__), "params", "indy7.json")


def rpy_to_matrix(r: float, p: float, y: float) -> np.ndarray:
    """URDF roll-pitch-yaw -> rotation, R = Rz(y) Ry(p) Rx(r)."""
    cr, sr = math.cos(r), math.sin(r)
    cp, sp = math.cos(p), math.sin(p)
    cy, sy = math.cos(y), math.sin(y)
    return np.array(
        [
            [cy * cp, cy * sp * sr - sy * cr, cy * sp * cr + sy * sr],
            [sy * cp, sy * sp * sr + cy * cr, sy * sp * cr - cy * sr],
            [-sp, cp * sr, cp * cr],
        ]
    )


def _floats(s: Optional[str], n: int = 3) -> List[float]:
    if s is None:
        return [0.0] * n
    v = [float(x) for x in s.split()]
    if len(v) != n:
        raise ValueError(f"expected {n} numbers, got {s!r}")
    return v


@dataclass
class _Inertia:
    mass: float = 0.0
    com: np.ndarray = field(default_factory=lambda: np.zeros(3))
    Ic: np.ndarray = field(default_factory=lambda: np.zeros((3, 3)))  # about COM

    def transformed(self, R: np.ndarray, t: np.ndarray) -> "_Inertia":
        return _Inertia(self.mass, R @ self.com + t, R @ self.Ic @ R.T)

    def __add__(self, o: "_Inertia") -> "_Inertia":
        m = self.mass + o.mass
        if m == 0.0:
            return _Inertia()
        c = (self.mass * self.com + o.mass * o.com) / m

        def shift(I: _Inertia) -> np.ndarray:
            d = I.com - c
            return I.Ic + I.mass * (np.dot(d, d) * np.eye(3) - np.outer(d, d))

        return _Inertia(m, c, shift(self) + shift(o))


class Motion:
    """Minimal stand-in for ``pin.Motion`` (only ``.linear``/``.angular`` are used)."""

    def __init__(self, linear=None, angular=None):
        self.linear = np.zeros(3) if linear is None else np.asarray(linear, dtype=float)
        self.angular = np.zeros(3) if angular is None else np.asarray(angular, dtype=float)

    @staticmethod
    def Zero() -> "Motion":
        return Motion()


class Data:
    """Stand-in for ``pin.Data``: holds the last kinematics evaluated on the host."""

    def __init__(self, model: "RobotModel"):
        self.oMi = [None] * model.njoints
        self.ddq = np.zeros(model.nv)


class RobotModel:
    """pinocchio-``Model``-like view of a 6-DOF revolute-z serial chain."""

    def __init__(self, params: dict):
        self.params = params
        self.name = params.get("name", "robot")
        self.names = ["universe"] + list(params["joint_names"])
        self.njoints = len(self.names)
        self.joints = list(range(self.njoints))  # len(model.joints) - 1 == nu (osqp_solver.py:20)
        self.nq = len(params["joint_names"])
        self.nv = self.nq
        g = params.get("gravity", [0.0, 0.0, -9.81])
        self.gravity = Motion(linear=g)
        self.lowerPositionLimit = np.array(params["q_lower"])
        self.upperPositionLimit = np.array(params["q_upper"])
        self.velocityLimit = np.array(params["v_limit"])
        self.effortLimit = np.array(params["effort_limit"])
        if self.nq != NJ:
            raise ValueError(f"the HIP kernels are specialised for {NJ} joints, model has {self.nq}")

    def createData(self) -> Data:
        return Data(self)

    # ---- packed block for the C-ABI (i7m_model in include/indy7_mpc.h) ----------------
    def packed(self) -> np.ndarray:
        """Flat float64 block laid out exactly like ``i7m_model`` (include/indy7_mpc.h)."""
        p = self.params
        out = []
        for j in range(NJ):
            out += list(np.asarray(p["placement_R"][j], dtype=float).reshape(9))
        for j in range(NJ):
            out += list(p["placement_t"][j])
        out += list(p["mass"])
        for j in range(NJ):
            out += list(p["com"][j])
        for j in range(NJ):
            I = np.asarray(p["inertia_com"][j], dtype=float)
            out += [I[0, 0], I[0, 1], I[0, 2], I[1, 1], I[1, 2], I[2, 2]]
        out += list(self.gravity.linear)
        out += list(self.lowerPositionLimit) + list(self.upperPositionLimit)
        out += list(self.velocityLimit) + list(self.effortLimit)
        return np.asarray(out, dtype=np.float64)


def parse_urdf(urdf_path: str) -> dict:
    """Parse a URDF into the parameter dict used by :class:`RobotModel`."""
    root = ET.parse(urdf_path).getroot()
    links = {}
    for ln in root.findall("link"):
        inert = _Inertia()
        el = ln.find("inertial")
        if el is not None:
            o = el.find("origin")
            xyz = _floats(o.get("xyz") if o is not None else None)
            rpy = _floats(o.get("rpy") if o is not None else None)
            m = float(el.find("mass").get("value"))
            ie = el.find("inertia")
            ixx, ixy, ixz, iyy, iyz, izz = (float(ie.get(k)) for k in ("ixx", "ixy", "ixz", "iyy", "iyz", "izz"))
            Ic = np.array([[ixx, ixy, ixz], [ixy, iyy, iyz], [ixz, iyz, izz]])
            R = rpy_to_matrix(*rpy)
            inert = _Inertia(m, np.array(xyz), R @ Ic @ R.T)
        links[ln.get("name")] = inert

    joints = []
    for jn in root.findall("joint"):
        o = jn.find("origin")
        ax = jn.find("axis")
        lim = jn.find("limit")
        joints.append(
            dict(
                name=jn.get("name"),
                type=jn.get("type"),
                parent=jn.find("parent").get("link"),
                child=jn.find("child").get("link"),
                xyz=np.array(_floats(o.get("xyz") if o is not None else None)),
                R=rpy_to_matrix(*_floats(o.get("rpy") if o is not None else None)),
                axis=np.array(_floats(ax.get("xyz") if ax is not None else "1 0 0")),
                lower=float(lim.get("lower", "0")) if lim is not None else 0.0,
                upper=float(lim.get("upper", "0")) if lim is not None else 0.0,
                velocity=float(lim.get("velocity", "0")) if lim is not None else 0.0,
                effort=float(lim.get("effort", "0")) if lim is not None else 0.0,
            )
        )
    children = {}
    child_links = set()
    for j in joints:
        children.setdefault(j["parent"], []).append(j)
        child_links.add(j["child"])
    roots = [n for n in links if n not in child_links]
    if len(roots) != 1:
        raise ValueError(f"URDF must have exactly one root link, found {roots}")

    # Walk the tree: each movable joint opens a new body; fixed joints merge into the
    # current body with the accumulated placement (R_acc, t_acc) from that body's frame.
    out = dict(joint_names=[], placement_R=[], placement_t=[], mass=[], com=[], inertia_com=[],
               q_lower=[], q_upper=[], v_limit=[], effort_limit=[])
    bodies: List[_Inertia] = []

    def walk(link: str, body: int, R_acc: np.ndarray, t_acc: np.ndarray):
        if body >= 0:
            bodies[body] = bodies[body] + links[link].transformed(R_acc, t_acc)
        for j in children.get(link, []):
            Rj = R_acc @ j["R"]
            tj = R_acc @ j["xyz"] + t_acc
            if j["type"] == "fixed":
                walk(j["child"], body, Rj, tj)
            elif j["type"] in ("revolute", "continuous"):
                if not np.allclose(j["axis"], [0.0, 0.0, 1.0]):
                    raise ValueError(f"joint {j['name']}: kernels need axis +z, got {j['axis']}")
                out["joint_names"].append(j["name"])
                out["placement_R"].append(Rj.tolist())
                out["placement_t"].append(tj.tolist())
                out["q_lower"].append(j["lower"])
                out["q_upper"].append(j["upper"])
                out["v_limit"].append(j["velocity"])
                out["effort_limit"].append(j["effort"])
                bodies.append(_Inertia())
                if len(children.get(link, [])) > 1:
                    raise ValueError("only serial chains are supported")
                walk(j["child"], len(bodies) - 1, np.eye(3), np.zeros(3))
            else:
                raise ValueError(f"unsupported joint type {j['type']}")

    walk(roots[0], -1, np.eye(3), np.zeros(3))
    for b in bodies:
        out["mass"].append(b.mass)
        out["com"].append(b.com.tolist())
        out["inertia_com"].append(b.Ic.tolist())
    out["gravity"] = [0.0, 0.0, -9.81]
    out["name"] = root.get("name", "robot")
    return out


def load_params(path: str = _DEFAULT_PARAMS) -> dict:
    with open(path) as f:
        return json.load(f)


def default_model() -> RobotModel:
    """The Indy7 model from the committed parameter block (generated from the URDF)."""
    return RobotModel(load_params())
