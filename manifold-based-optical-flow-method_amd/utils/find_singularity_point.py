"""Drop-in for the reference's ``utils/find_singularity_point.py``.

Replaced on the GPU: ``process_V_k`` (find_singularity_point.py:28-69, the
S3 epilogue on the hot path's output, ``mofhip.epilogue``) and the critical
point search ``find_singularity_points`` / ``find_singularity_points_for_all_Vk``
(:140-189, :530-558, ``mofhip.singular``). Every other name (classification,
error metrics -- out of scope) is taken unchanged from the
reference's module when that module is reachable through the extended
``utils`` package path.
"""
from __future__ import annotations

import importlib.util as _ilu
import os as _os

from mofhip.epilogue import velocity_vectors as _velocity_vectors
from mofhip import singular as _singular


def _load_reference_module():
    here = _os.path.dirname(_os.path.abspath(__file__))
    from . import __path__ as pkg_path
    for d in pkg_path:
        if _os.path.abspath(d) == here:
            continue
        cand = _os.path.join(d, "find_singularity_point.py")
        if _os.path.exists(cand):
            spec = _ilu.spec_from_file_location("_reference_find_singularity_point", cand)
            mod = _ilu.module_from_spec(spec)
            try:
                spec.loader.exec_module(mod)
            except ImportError:  # its optional plotting/mesh deps are absent
                return None
            return mod
    return None


_REPLACED = ("process_V_k", "find_singularity_points", "find_singularity_points_for_all_Vk")
_ref = _load_reference_module()
if _ref is not None:
    globals().update({k: v for k, v in vars(_ref).items()
                      if not k.startswith("__") and k not in _REPLACED})


def process_V_k(V_k, e):
    """3-D tangent velocity vectors ``V^0 e^0 + V^1 e^1`` per vertex and
    timestep: array (K, N, 3), bit-identical to the reference's list."""
    coord, _ = _velocity_vectors(V_k, e, want_speed=False)
    return coord


def find_singularity_points(coordinates, triangles, V_now, eps):
    """Zero-velocity vertices and triangle interiors of one field (reference
    :140-189): ``(singularity_vertices, singularity_interiors, v_length_max)``."""
    return _singular.find_singularity_points(coordinates, triangles, V_now, eps)


def find_singularity_points_for_all_Vk(V_k_coord, coordinates, triangles, eps):
    """Critical point coordinates per timestep (reference :530-558), all
    timesteps in one GPU launch sequence."""
    return _singular.find_singularity_points_for_all_Vk(V_k_coord, coordinates, triangles, eps)
