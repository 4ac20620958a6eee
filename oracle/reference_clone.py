"""CPU baseline: the reference's own algorithm, re-stated to be timed on the
GPU box (where /root/reference does not exist).

TEST / BENCH INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg, tests).

What the reference does per timestep (compute_optical_flow.py:100-149) and
what this clone repeats, operation class for operation class:
  * a Python loop over triangles; per triangle grad_M I from three scaled
    grad_w rows (:116-117);
  * per corner and alpha, the f term with a set difference, a list
    comprehension, np.sum and np.dot (:123-126, :288-311);
  * per (i <= j, alpha, beta) pair the a1 term (two np.dot) accumulated with a
    scalar ``lil_matrix.__getitem__`` + ``__setitem__``, plus the mirrored
    assignment (:127-141, :273-285);
  * ``a1 + lambda * a2`` -> ``csr_matrix`` -> ``spsolve`` (:144-147);
  * timesteps farmed out with ``multiprocessing.Pool.apply_async``, each task
    pickling a2 (lil), grad_w, e, ... as the reference does (:157-191).

Calibrated against the real reference in the build container
(tests/golden/cpu_clone_calibration.json): the clone is not slower.

``sample_tris`` restricts the triangle loop to the first ``sample_tris``
triangles (the bounded sample bench.py times at 160k; the per-triangle cost
is linear in M) while spsolve still runs on the full-size
system.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import time
import warnings

import numpy as np
from scipy.sparse import csr_matrix, lil_matrix
from scipy.sparse.linalg import spsolve


def _f_term(g, e_ia, I1, I0, dt, i, tri, area):
    rest = set(tri) - {i}
    d_i = (I1[i] - I0[i]) / dt
    d_rest = np.sum([(I1[x] - I0[x]) / dt for x in rest])
    return np.dot(e_ia, g) * (2 * d_i + d_rest) * area / 12


def timestep(k, a2, grad_w, e, iw, triangles, t_k, areas, lam, I0, I1, sample_tris=None):
    """One reference ``worker``: returns (V, seconds in the triangle loop,
    seconds in csr + spsolve)."""
    N = len(e)
    a1 = lil_matrix((2 * N, 2 * N))
    f = np.zeros(2 * N)
    dt = t_k[k + 1] - t_k[k]
    M = len(triangles) if sample_tris is None else min(int(sample_tris), len(triangles))
    t0 = time.perf_counter()
    for t in range(M):
        tri = triangles[t]
        gw = grad_w[t]
        g = I0[tri[0]] * gw[0] + I0[tri[1]] * gw[1] + I0[tri[2]] * gw[2]
        for i in tri:
            for al in range(2):
                row = i + N * al
                f[row] += _f_term(g, e[i][al], I1, I0, dt, i, tri, areas[t])
                for j in tri:
                    if i > j:
                        continue
                    w = iw[t][0] if i == j else iw[t][1]
                    for be in range(2):
                        col = j + N * be
                        a1[row, col] += np.dot(g, e[i][al]) * np.dot(g, e[j][be]) * w
                        if i != j:
                            a1[col, row] = a1[row, col]
    t1 = time.perf_counter()
    A = csr_matrix(a1 + lam * a2)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        V = spsolve(A, f)
    t2 = time.perf_counter()
    return V, t1 - t0, t2 - t1


def _task(args):
    return timestep(*args)


def pool_timesteps(ks, a2, grad_w, e, iw, triangles, t_k, areas, lam, I, I2, processes,
                   sample_tris=None):
    """Run ``timestep`` for every k in ``ks`` on ``Pool(processes)`` with one
    ``apply_async`` per timestep, like compute_velocity_field. Returns
    (list of (V, t_loop, t_solve) in k order, wall seconds submit->join)."""
    ctx = mp.get_context("fork")
    pool = ctx.Pool(processes)
    try:
        t0 = time.perf_counter()
        handles = [pool.apply_async(timestep, (k, a2, grad_w, e, iw, triangles, t_k, areas, lam,
                                               I[k], I2[k + 1], sample_tris)) for k in ks]
        pool.close()
        pool.join()
        wall = time.perf_counter() - t0
        return [h.get() for h in handles], wall
    finally:
        pool.terminate()


def as_lil(a2_csr):
    """The reference hands workers an a2 lil_matrix (compute_optical_flow.py:49)."""
    return lil_matrix(a2_csr)


def default_cores() -> int:
    """Host cores to use on the GPU box: its CPU share is 16 per GPU."""
    return max(1, min(16, os.cpu_count() or 1))
