"""Drop-in replacement for the reference's ``utils/compute_optical_flow.py``
(SEU-dynamical-models/Manifold-based-optical-flow-method), backed by
libmofhip on MI355X.

Same public names, positional order and return tuples, so the reference's
S3 driver (``from utils import compute_optical_flow``, S3…py:11,97-123) runs
unchanged with this directory on ``sys.path``:

=============================  ============================================
reference (file:line)          here
=============================  ============================================
compute_geometrical_quantities  mesh build on the GPU; ``a2`` is a
  (:27-97)                       :class:`mofhip.DeviceMesh` (opaque; S3 only
                                 passes it back) with ``.tocsr()``
worker (:100-149)              one timestep: GPU assembly + PCG
compute_velocity_field         timesteps batched per GPU, contiguous
  (:152-194)                     k-shards over ``min(processes_num, #GPUs)``
load_potentials (:203-207)     threaded native reader, pandas' parser
                                 restated (bit-identical values)
reshape_and_save_data          threaded native writer, pandas' bytes
  (:314-320)
compute_orthonormal_basis,     host helpers with the reference's formulas;
compute_gradient_w, compute_a2,  not on the hot path (the GPU kernels
compute_a1, compute_f            restate them, csrc/mof_assemble.hip)
  (:210-311)
=============================  ============================================

Solver semantics: ``scipy.sparse.linalg.spsolve`` (direct) becomes a
preconditioned CG stopped at ``||f - A V||_2 <= rtol ||f||_2`` (rtol 1e-8
by default: |V - V_spsolve|_max ~ 1e-8 on the parity meshes). A system that
does not converge is returned NaN-filled with a ``MatrixRankWarning``, as
spsolve does for a singular matrix (scipy linsolve.py:287-289).
"""
from __future__ import annotations

import os
import time
import warnings

import numpy as np

from mofhip import DeviceMesh, device_count, velocity_field_sharded

try:  # the warning class spsolve uses
    from scipy.sparse.linalg import MatrixRankWarning
except Exception:  # pragma: no cover
    class MatrixRankWarning(UserWarning):
        pass

# Solver options used by worker / compute_velocity_field. Override with
# set_solver_options() or the environment. Default ("auto"): fp32 inner PCG
# with the multigrid preconditioner and fp64 iterative refinement to
# ||f - A V|| <= 1e-8 ||f|| in fp64; on meshes of at most SMALL_MESH vertices
# fp64 block-Jacobi PCG, which the library runs as one fused launch per batch
# (round 4, 642 vertices x 15 timesteps: 0.55 vs 1.1 ms; at 3,249 vertices the
# multigrid is 2x faster). MOF_PRECISION=f64 / mixed forces either;
# MOF_PRECOND=jacobi: block Jacobi in the mixed inner solve.
SMALL_MESH = 1024
SOLVER_OPTIONS = {
    "precision": os.environ.get("MOF_PRECISION", "auto"),
    "precond": os.environ.get("MOF_PRECOND", ""),
    "rtol": 1e-8,
    "batch": 0,
}
# compute_velocity_field checkpoint / resume: a directory for shard-granular
# V chunks (mofhip.solve.Checkpoint; MOF_CHECKPOINT_DIR), "" for none
RUN_OPTIONS = {
    "checkpoint_dir": os.environ.get("MOF_CHECKPOINT_DIR", ""),
    "checkpoint_chunk": int(os.environ.get("MOF_CHECKPOINT_CHUNK", "0") or 0),
}


def set_solver_options(**kw):
    """Update the PCG options (precision 'auto'|'f64'|'mixed', precond
    'amg'|'jacobi' (default: amg for mixed, jacobi for f64), rtol, batch, ...)
    and the run options (checkpoint_dir, checkpoint_chunk)."""
    for k, v in kw.items():
        (RUN_OPTIONS if k in RUN_OPTIONS else SOLVER_OPTIONS)[k] = v
    return dict(SOLVER_OPTIONS, **RUN_OPTIONS)


def _solver_options(mesh=None):
    o = dict(SOLVER_OPTIONS)
    if o.get("precision") in (None, "", "auto"):
        o["precision"] = "f64" if mesh is not None and mesh.N <= SMALL_MESH else "mixed"
    if not o.get("precond"):
        o["precond"] = "amg" if o.get("precision") == "mixed" else "jacobi"
    return o


def _mesh_of(a2) -> DeviceMesh:
    if isinstance(a2, DeviceMesh):
        return a2
    raise TypeError(
        "a2 must be the DeviceMesh returned by this module's "
        "compute_geometrical_quantities (got %s)" % type(a2).__name__)


def _warn_failed(n_failed: int):
    if n_failed:
        warnings.warn("%d system(s) did not converge (singular or not SPD); "
                      "their velocity field is NaN" % n_failed, MatrixRankWarning, stacklevel=3)


def compute_geometrical_quantities(coordinates, normals, triangles, areas):
    """Mesh constants on the GPU (reference :27-97).

    Returns ``(a2, grad_w, e, integral_wi_wj, execution_time)``: ``a2`` is a
    :class:`mofhip.DeviceMesh`; ``grad_w`` (M,3,3), ``e`` (N,2,3) and
    ``integral_wi_wj`` (M,2) are host float64 arrays, bit-identical to the
    reference's."""
    start = time.time()
    mesh = DeviceMesh(coordinates, normals, triangles, areas, device=0)
    # the per-mesh solver setup (the multigrid hierarchy of a2) belongs to
    # this per-mesh call, as a2 itself does in the reference: built on a host
    # thread of the handle beside the geometry export, finished before return
    mesh.prepare_solver(**_solver_options(mesh))
    e, grad_w, iw = mesh.geometry()
    mesh.sync_solver()
    return mesh, grad_w, e, iw, time.time() - start


def worker(k, a2, grad_w, e, integral_wi_wj, triangles, t_k, areas, lambda_, I_k_k, I_k_kplus1):
    """Velocity field of timestep ``k`` (reference :100-149): (2N,) float64."""
    mesh = _mesh_of(a2)
    I = np.stack([np.asarray(I_k_k, dtype=np.float64), np.asarray(I_k_kplus1, dtype=np.float64)])
    tk = np.array([t_k[k], t_k[k + 1]], dtype=np.float64)
    V, st = mesh.solve_range(I, tk, 0, 1, lambda_, **_solver_options(mesh))
    _warn_failed(st["failed"])
    return V[0]


def compute_velocity_field(processes_num, time_steps, a2, grad_w, e, integral_wi_wj, triangles,
                           t_k, areas, lambda_, I_k, I_k_2):
    """All ``time_steps - 1`` velocity fields (reference :152-194).

    Timestep k uses ``I_k[k]`` and ``I_k_2[k+1]``. Returns
    ``(V_k: list of (2N,) arrays in k order, execution_time)``; the GPUs
    used are the first ``min(processes_num, device count)``."""
    mesh = _mesh_of(a2)
    ndev = max(1, min(int(processes_num), device_count()))
    K = int(time_steps) - 1
    I = np.ascontiguousarray(np.asarray(I_k, dtype=np.float64)[:time_steps])
    I2 = np.ascontiguousarray(np.asarray(I_k_2, dtype=np.float64)[:time_steps])
    tk = np.asarray(t_k, dtype=np.float64)
    # one handle per GPU, built concurrently before the clock starts -- as the
    # reference creates its Pool(processes_num) before start_time (:155-158)
    mesh.prepare(range(ndev))
    start = time.time()
    V, stats = velocity_field_sharded(mesh, I, tk, 0, max(K, 0), lambda_, I2=I2, devices=range(ndev),
                                      checkpoint=RUN_OPTIONS["checkpoint_dir"] or None,
                                      chunk=RUN_OPTIONS["checkpoint_chunk"], **_solver_options(mesh))
    execution_time = time.time() - start
    _warn_failed(sum(s["failed"] for s in stats))
    return [V[k] for k in range(V.shape[0])], execution_time


def load_surface(surface_path):
    """The surface (reference :197-200, ``pv.read``): pyvista when it is
    installed, else libmofhip's PLY reader with the attributes S3 uses
    (``points``, ``faces``, ``point_normals``, ``compute_cell_sizes``)."""
    try:
        import pyvista as pv  # noqa: WPS433 (optional)
    except ImportError:
        from mofhip.surface import read_surface
        return read_surface(surface_path)
    return pv.read(surface_path)


def load_potentials(csv_path):
    """(T, N) potentials from the S2 CSV (reference :203-207,
    ``pd.read_csv(path, sep=',', header='infer', index_col=0).values``):
    parsed by libmofhip's threaded reader with pandas' own float parser
    restated (bit-identical values); a file it cannot read as a numeric
    table goes to pandas itself."""
    from mofhip import csvio
    from mofhip._lib import MofError
    try:
        return csvio.read_csv(csv_path)
    except MofError:
        import pandas as pd
        return pd.read_csv(csv_path, sep=",", header="infer", index_col=0).values


def reshape_and_save_data(data, file_path):
    """Flatten to (rows, -1) and write the CSV (reference :314-320; e: (N,6),
    V_k: (T-1, 2N)): float data through libmofhip's threaded writer, the
    same bytes as ``pd.DataFrame(...).to_csv(file_path)``."""
    arr = np.asarray(data)
    reshaped = arr.reshape(arr.shape[0], -1)
    if reshaped.dtype.kind == "f":
        from mofhip import csvio
        csvio.write_csv(file_path, reshaped)
    else:
        import pandas as pd
        pd.DataFrame(reshaped).to_csv(file_path)
    print(f"{file_path}文件保存成功。")


# ---- per-element helpers (host; the GPU kernels restate these) -----------

def compute_orthonormal_basis(n_i):
    """Tangent basis (e1, e2) of a vertex normal (reference :210-235)."""
    n = np.asarray(n_i)
    if n[0] != 0 or n[1] != 0:
        t = np.array([-n[1], n[0], 0.0])
    else:
        t = np.array([0.0, -n[2], n[1]])
    c = np.cross(n, t)
    return t / np.linalg.norm(t), c / np.linalg.norm(c)


def compute_gradient_w(p_i, p_j, p_k):
    """Gradient of the P1 hat function of p_i on triangle (p_i, p_j, p_k)
    (reference :238-255)."""
    jk = p_k - p_j
    h = (p_j - p_i) + np.dot(p_i - p_j, jk) * jk / np.dot(jk, jk)
    return h / np.dot(h, h)


def compute_a2(T_area, e_i, e_j, grad_i, grad_j):
    """Smoothness term of one (i, alpha; j, beta) pair (reference :258-270)."""
    return np.dot(e_i, e_j) * np.dot(grad_i, grad_j) * T_area


def compute_a1(integral, grad_M_I, e_i, e_j):
    """Data term of one (i, alpha; j, beta) pair (reference :273-285)."""
    return np.dot(grad_M_I, e_i) * np.dot(grad_M_I, e_j) * integral


def compute_f(grad_M_I, e_i, I_kplus1, I_k, t, i, T, T_area):
    """Right-hand side term of vertex i on triangle T (reference :288-311)."""
    others = set(T) - {i}
    d_i = (I_kplus1[i] - I_k[i]) / t
    d_o = np.sum([(I_kplus1[x] - I_k[x]) / t for x in others])
    return np.dot(e_i, grad_M_I) * (2 * d_i + d_o) * T_area / 12
