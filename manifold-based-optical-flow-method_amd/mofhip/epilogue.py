"""S3's post-solve epilogue on the GPU.

``process_V_k(V_k, e)`` (find_singularity_point.py:28-69) turns the planar
velocity components into 3-D tangent vectors ``V^0 e^0 + V^1 e^1`` and S3
then takes their lengths, ``V_c = sqrt(sum(V_k_coord**2, axis=2))``
(S3…py:130-132). Both are one elementwise kernel (``mof_velocity_vectors``),
bit-identical to numpy.
"""
from __future__ import annotations

import numpy as np

from . import _lib as L


def velocity_vectors(V_k, e, device: int = 0, want_coord: bool = True, want_speed: bool = True):
    """``(V_k_coord (K,N,3), V_c (K,N))`` from V_k (K,2N) and e (N,2,3)."""
    V = np.ascontiguousarray(np.asarray(V_k, dtype=np.float64))
    E = np.ascontiguousarray(np.asarray(e, dtype=np.float64))
    if V.ndim == 1:
        V = V[None, :]
    N = E.shape[0]
    if E.shape != (N, 2, 3) or V.ndim != 2 or V.shape[1] != 2 * N:
        raise ValueError("need V_k (K, 2N) and e (N, 2, 3)")
    K = V.shape[0]
    coord = np.empty((K, N, 3)) if want_coord else None
    speed = np.empty((K, N)) if want_speed else None
    L.check(L.lib().mof_velocity_vectors(
        int(device), L.ptr(E), L.ptr(V), N, K,
        L.ptr(coord) if want_coord else None, L.ptr(speed) if want_speed else None, 0, None))
    return coord, speed


def velocity_vectors_device(e_ptr: int, V_ptr: int, N: int, K: int, coord_ptr: int | None,
                            speed_ptr: int | None, device: int = 0, stream: int | None = None):
    """Device-pointer form (all buffers already in HBM)."""
    L.check(L.lib().mof_velocity_vectors(int(device), e_ptr, V_ptr, int(N), int(K), coord_ptr,
                                         speed_ptr, L.MOF_IO_DEVICE, stream))
