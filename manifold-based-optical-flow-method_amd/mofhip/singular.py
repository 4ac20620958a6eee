"""Critical points of the velocity fields on the GPU (SURVEY.md §8(f)4;
C ABI ``mof_singularities``).

``find_singularity_points(coordinates, triangles, V_now, eps)`` returns the
reference's structure (find_singularity_point.py:140-189):
``(singularity_vertices, singularity_interiors, v_length_max)`` with
``[i, coordinates[i]]`` per zero vertex and ``[i, P_coord, triangle, [lam,
mu, 1 - lam - mu], [A, B, C coordinates]]`` per triangle holding a zero;
``find_singularity_points_for_all_Vk`` (:530-558) runs all K fields in one
launch sequence. v_length_max and the vertex test are bit-identical to the
reference; (lam, mu) come from a QR/SVD restatement of np.linalg.lstsq and
agree to rounding.
"""
from __future__ import annotations

import numpy as np

from . import _lib as L


def singularity_flags(coordinates, triangles, V_k_coord, eps, device: int = 0):
    """Raw per-field results for V_k_coord (K,N,3):
    ``(vmax (K,), vertex_flag (K,N) bool, triangle_flag (K,M) bool, lam_mu (K,M,2))``."""
    P = np.asarray(coordinates)
    f32 = P.dtype == np.float32
    P = np.ascontiguousarray(P, dtype=np.float32 if f32 else np.float64)
    T = np.ascontiguousarray(np.asarray(triangles).reshape(-1, 3), dtype=np.int32)
    V = np.ascontiguousarray(np.asarray(V_k_coord, dtype=np.float64))
    if V.ndim == 2:
        V = V[None]
    N, M, K = P.shape[0], T.shape[0], V.shape[0]
    if P.shape != (N, 3) or V.shape[1:] != (N, 3):
        raise ValueError("need coordinates (N,3) and V (K,N,3)")
    vmax = np.empty(K)
    vf = np.empty((K, N), dtype=np.uint8)
    tf = np.empty((K, M), dtype=np.uint8)
    lm = np.empty((K, M, 2))
    L.check(L.lib().mof_singularities(int(device), L.ptr(P), L.ptr(T), N, M, L.ptr(V), K, float(eps),
                                      L.MOF_COORDS_F32 if f32 else 0, None, L.ptr(vmax),
                                      L.ptr(vf), L.ptr(tf), L.ptr(lm)))
    return vmax, vf.astype(bool), tf.astype(bool), lm


def singularity_lists(coordinates, triangles, V_k_coord, eps, device: int = 0, cap: int = 0):
    """Per field, only what the reference returns: ``(vmax (K,), [zero vertex
    ids (n_k,)] * K, [(zero triangle ids (m_k,), lam_mu (m_k, 2))] * K)``,
    compacted on the device (``mof_singularities_compact``)."""
    P = np.asarray(coordinates)
    f32 = P.dtype == np.float32
    P = np.ascontiguousarray(P, dtype=np.float32 if f32 else np.float64)
    T = np.ascontiguousarray(np.asarray(triangles).reshape(-1, 3), dtype=np.int32)
    V = np.ascontiguousarray(np.asarray(V_k_coord, dtype=np.float64))
    if V.ndim == 2:
        V = V[None]
    N, M, K = P.shape[0], T.shape[0], V.shape[0]
    if P.shape != (N, 3) or V.shape[1:] != (N, 3):
        raise ValueError("need coordinates (N,3) and V (K,N,3)")
    cap = int(cap) or max(4096, 256 * K)
    while True:
        totals = np.zeros(2, np.int64)
        vmax = np.empty(K)
        nv = np.empty(K, np.int64)
        nt = np.empty(K, np.int64)
        vi = np.empty(cap, np.int32)
        ti = np.empty(cap, np.int32)
        lm = np.empty((cap, 2))
        rc = L.lib().mof_singularities_compact(
            int(device), L.ptr(P), L.ptr(T), N, M, L.ptr(V), K, float(eps),
            L.MOF_COORDS_F32 if f32 else 0, None, cap, L.ptr(totals), L.ptr(vmax), L.ptr(nv),
            L.ptr(vi), L.ptr(nt), L.ptr(ti), L.ptr(lm))
        if rc == L.MOF_E_ARG and int(totals.max()) > cap:
            cap = int(totals.max())  # the device counted what it needs: once more, sized
            continue
        L.check(rc)
        break
    ov = np.concatenate([[0], np.cumsum(nv)])
    ot = np.concatenate([[0], np.cumsum(nt)])
    verts = [vi[ov[k]:ov[k + 1]].copy() for k in range(K)]
    tris = [(ti[ot[k]:ot[k + 1]].copy(), lm[ot[k]:ot[k + 1]].copy()) for k in range(K)]
    return vmax, verts, tris


def _lists(coordinates, triangles, vids, tids, lms):
    verts = [[int(i), coordinates[i]] for i in vids]
    inter = []
    for i, (lam, mu) in zip(tids, lms):
        tri = triangles[i]
        A, B, C = tri
        P = lam * coordinates[A] + mu * coordinates[B] + (1 - lam - mu) * coordinates[C]
        inter.append([int(i), P, tri, [lam, mu, 1 - lam - mu],
                      [coordinates[A], coordinates[B], coordinates[C]]])
    return verts, inter


def find_singularity_points(coordinates, triangles, V_now, eps, device: int = 0):
    vmax, verts, tris = singularity_lists(coordinates, triangles, V_now, eps, device)
    verts, inter = _lists(np.asarray(coordinates), np.asarray(triangles), verts[0], *tris[0])
    return verts, inter, np.float64(vmax[0])


def find_singularity_points_for_all_Vk(V_k_coord, coordinates, triangles, eps, device: int = 0):
    vmax, vlist, tlist = singularity_lists(coordinates, triangles, V_k_coord, eps, device)
    C, T = np.asarray(coordinates), np.asarray(triangles)
    out = []
    for k in range(len(vmax)):
        verts, inter = _lists(C, T, vlist[k], *tlist[k])
        print(f"第{k}个时刻临界点个数为{len(verts) + len(inter)}")
        out.append([v[1] for v in verts] + [s[1] for s in inter])
    return out
