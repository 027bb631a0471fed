"""Drop-in for reference src/utils.py: ``load_robot_model``, ``rk4``, ``print_stats``.

``rk4`` runs on the GPU (i7m_rk4, 4 ABA evaluations per step) — there is no host dynamics.
"""
from __future__ import annotations

import threading

import numpy as np

from . import _lib
from .model import RobotModel, parse_urdf

_query_handles = {}
_qlock = threading.Lock()


class GeometryModel:
    """Placeholder for pinocchio's collision/visual GeometryModel (meshes are not used by the
    solver; the reference only hands them to the meshcat visualiser)."""

    def __init__(self, urdf_path: str = "", mesh_dir: str = ""):
        self.urdf_path, self.mesh_dir = urdf_path, mesh_dir
        self.ngeoms = 0


def load_robot_model(urdf_path, mesh_dir):
    """reference src/utils.py:20-21 -> ``pin.buildModelsFromUrdf(urdf_path, mesh_dir)``, which
    returns (model, collision_model, visual_model)."""
    model = RobotModel(parse_urdf(urdf_path))
    return model, GeometryModel(urdf_path, mesh_dir), GeometryModel(urdf_path, mesh_dir)


def query_handle(model) -> "_lib.Handle":
    """A small device handle for per-call kinematics/dynamics queries on ``model``."""
    key = id(model)
    with _qlock:
        h = _query_handles.get(key)
        if h is None:
            h = _lib.Handle(model, N=2, max_batch=256)
            _query_handles[key] = (h, model)  # keep model alive with its handle
            return h
        return h[0]


def fext_last_joint(f_ext):
    """Accept the f_ext forms of the reference (a pin.StdVec_Force of per-joint local forces,
    src/gato_mpc_batch_sample.py:143-161) or a (6,) / (B, 6) array for joint 6.  Only a wrench
    on the last joint is supported (the only one the reference ever sets)."""
    if f_ext is None:
        return None
    if isinstance(f_ext, np.ndarray) and f_ext.dtype != object:
        return np.asarray(f_ext, dtype=float).reshape(-1, 6)
    forces = list(f_ext)

    def as6(f):
        if hasattr(f, "linear") and hasattr(f, "angular"):
            return np.concatenate([np.asarray(f.linear, float), np.asarray(f.angular, float)])
        return np.asarray(f, dtype=float).reshape(6)

    vecs = [as6(f) for f in forces]
    if any(np.any(v != 0.0) for v in vecs[:-1]):
        raise NotImplementedError("external forces are supported on the last joint only")
    return vecs[-1].reshape(1, 6)


def rk4(model, data, q, v, u, dt, f_ext=None):
    """reference src/utils.py:3-18 (4 x pin.aba, pin.integrate = q + v dt), on the GPU."""
    h = query_handle(model)
    qo, vo = h.rk4(q, v, u, dt, fext=fext_last_joint(f_ext))
    return qo[0], vo[0]


def print_stats(stats):
    """reference src/utils.py:23-39."""
    for task, stat in stats.items():
        stat_list = stat["values"]
        stat_unit = stat["unit"]
        stat_mult = stat["multiplier"]
        if not stat_list:
            continue
        avg_stat = stat_mult * sum(stat_list) / len(stat_list)
        min_stat, max_stat = stat_mult * min(stat_list), stat_mult * max(stat_list)
        print(f"{task}:")
        print(f"  avg: {avg_stat:.2f} {stat_unit}")
        print(f"  min: {min_stat:.2f} {stat_unit}")
        print(f"  max: {max_stat:.2f} {stat_unit}")
        print()
