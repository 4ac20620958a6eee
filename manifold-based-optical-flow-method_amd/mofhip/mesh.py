"""Device-resident mesh handle: the object the drop-in
``compute_geometrical_quantities`` returns where the reference returns its
``a2`` lil_matrix (compute_optical_flow.py:49,97).

S3 never looks inside ``a2``; it only hands it back to
``compute_velocity_field`` (S3…py:97-117). :class:`DeviceMesh` therefore
keeps a2 (and the rest of the mesh constants) in HBM and offers ``tocsr()``
for inspection and parity checks.
"""
from __future__ import annotations

import ctypes
import threading
import time

import numpy as np

from . import _lib as L


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


class DeviceMesh:
    """One triangle mesh, resident on one or more GPUs (one handle each)."""

    def __init__(self, coordinates, normals, triangles, areas, device: int = 0,
                 reorder: bool = True):
        coords = np.asarray(coordinates)
        tri = np.asarray(triangles)
        if coords.ndim != 2 or coords.shape[1] != 3:
            raise ValueError("coordinates must be (N, 3)")
        if tri.ndim != 2 or tri.shape[1] != 3:
            raise ValueError("triangles must be (M, 3)")
        self.f32_points = coords.dtype == np.float32
        self._xyz = _f64(coords)
        self._nrm = _f64(normals)
        self._tri = np.ascontiguousarray(tri, dtype=np.int32)
        self._area = _f64(np.asarray(areas).reshape(-1))
        self.N = len(self._xyz)
        self.M = len(self._tri)
        if self._nrm.shape != (self.N, 3) or len(self._area) != self.M:
            raise ValueError("normals must be (N, 3) and areas (M,)")
        self.reorder = bool(reorder)  # RCM vertex order on the device (results unaffected)
        self._handles = {}
        self._locks = {}
        self._build_locks = {}
        self._glock = threading.Lock()  # guards the dicts only; builds run outside it
        self.build_seconds = {}  # wall seconds of each handle's build (per device)
        self.device = int(device)
        self.handle(self.device)

    # -- handles ---------------------------------------------------------
    def handle(self, device: int | None = None) -> ctypes.c_void_p:
        """The handle on ``device``, built on first use: the primary device's
        with ``mof_mesh_create`` (host pattern, orders, the per-mesh kernels),
        every other device's with ``mof_mesh_clone`` of it (the host state
        and multigrid hierarchy are shared, only uploads and the per-mesh
        kernels run). Builds of different devices run concurrently; only the
        same device's build is serialised."""
        device = self.device if device is None else int(device)
        h = self._handles.get(device)
        if h is not None:
            return h
        with self._glock:
            blk = self._build_locks.setdefault(device, threading.Lock())
        with blk:
            h = self._handles.get(device)
            if h is not None:
                return h
            t0 = time.perf_counter()
            h = ctypes.c_void_p()
            if device != self.device:
                src = self.handle(self.device)
                L.check(L.lib().mof_mesh_clone(src, device, ctypes.byref(h)))
            else:
                flags = ((L.MOF_GEOM_F32_POINTS if self.f32_points else 0)
                         | (0 if self.reorder else L.MOF_NO_REORDER))
                L.check(L.lib().mof_mesh_create(
                    L.ptr(self._xyz), L.ptr(self._nrm), L.ptr(self._tri), L.ptr(self._area),
                    self.N, self.M, device, flags, ctypes.byref(h)))
            with self._glock:
                self.build_seconds[device] = time.perf_counter() - t0
                self._locks[device] = threading.Lock()
                self._handles[device] = h
        return h

    def prepare(self, devices) -> dict:
        """Build the handles of ``devices`` that do not exist yet, concurrently
        (one host thread per device; ctypes releases the GIL). Returns the
        build seconds per device."""
        todo = [int(d) for d in dict.fromkeys(devices) if int(d) not in self._handles]
        if self.device in todo:  # the clones need the primary handle
            self.handle(self.device)
            todo.remove(self.device)
        errors = []

        def run(d):
            try:
                self.handle(d)
            except BaseException as exc:  # re-raised below
                errors.append(exc)

        threads = [threading.Thread(target=run, args=(d,)) for d in todo]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        if errors:
            raise errors[0]
        return dict(self.build_seconds)

    def prepare_solver(self, device: int | None = None, **opts):
        """Start the per-mesh setup the solves with ``opts`` need (the
        multigrid hierarchy, mof_mesh_prepare) on a host thread of the
        handle; returns at once, the next solve waits for it."""
        o = self.make_opts(**{k: v for k, v in opts.items() if k != "batch"})
        with self.lock(device):
            L.check(L.lib().mof_mesh_prepare(self.handle(device), ctypes.byref(o)))

    def sync_solver(self, device: int | None = None):
        """Wait for the setup prepare_solver started (raises its error)."""
        with self.lock(device):
            L.check(L.lib().mof_mesh_sync(self.handle(device)))

    def lock(self, device: int | None = None) -> threading.Lock:
        device = self.device if device is None else int(device)
        self.handle(device)
        return self._locks[device]

    def close(self):
        with self._glock:
            hs = list(self._handles.values())
            self._handles.clear()
        for h in hs:
            L.lib().mof_mesh_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- matrix-like view of a2 -------------------------------------------
    @property
    def shape(self):
        return (2 * self.N, 2 * self.N)

    def info(self, device: int | None = None) -> dict:
        inf = L.MofMeshInfo()
        L.check(L.lib().mof_mesh_get_info(self.handle(device), ctypes.byref(inf)))
        return {k: getattr(inf, k) for k, _ in inf._fields_}

    @property
    def nnz(self) -> int:
        return int(self.info()["nnz_struct"])

    def geometry(self):
        """``(e (N,2,3), grad_w (M,3,3), integral_wi_wj (M,2))`` host copies."""
        e = np.empty((self.N, 2, 3))
        gw = np.empty((self.M, 3, 3))
        iw = np.empty((self.M, 2))
        with self.lock():
            L.check(L.lib().mof_geometry_export(self.handle(), L.ptr(e), L.ptr(gw), L.ptr(iw)))
        return e, gw, iw

    def _csr(self, which: int, drop_zeros: bool):
        with self.lock():
            return self._csr_locked(which, drop_zeros)

    def tocsr(self, drop_zeros: bool = True):
        """a2 as scipy CSR; ``drop_zeros`` mirrors lil's zero removal."""
        return self._csr(L.MOF_CSR_A2, drop_zeros)

    def assemble(self, I0, I1, dt, lambda_, drop_zeros: bool = True):
        """One timestep's ``(A = a1 + lambda*a2 as CSR, f)`` (worker :113-146)."""
        I0 = _f64(I0)
        I1 = _f64(I1)
        if I0.shape != (self.N,) or I1.shape != (self.N,):
            raise ValueError("I0 and I1 must be (N,)")
        f = np.empty(2 * self.N)
        with self.lock():
            L.check(L.lib().mof_assemble(self.handle(), L.ptr(I0), L.ptr(I1), float(dt),
                                         float(lambda_), L.ptr(f)))
            A = self._csr_locked(L.MOF_CSR_A_LAST, drop_zeros)
        return A, f

    def _csr_locked(self, which, drop_zeros):
        import scipy.sparse as sp
        cap = self.nnz
        indptr = np.empty(2 * self.N + 1, np.int32)
        indices = np.empty(cap, np.int32)
        data = np.empty(cap)
        nnz = ctypes.c_int64(0)
        L.check(L.lib().mof_csr_export(self.handle(), which, int(bool(drop_zeros)),
                                       L.ptr(indptr), L.ptr(indices), L.ptr(data),
                                       ctypes.byref(nnz)))
        n = nnz.value
        return sp.csr_matrix((data[:n].copy(), indices[:n].copy(), indptr), shape=self.shape)

    # -- solves ------------------------------------------------------------
    @staticmethod
    def make_opts(precision="f64", batch=0, rtol=0.0, inner_rtol=0.0, max_iter=0, max_outer=0,
                  block_jacobi=True, device_io=False, time_spmv=False, stream=None,
                  precond="jacobi", recovery=True, fused=None, etol=0.0) -> L.MofOpts:
        """precond: "jacobi" (2x2 block Jacobi) or "amg" (aggregation-multigrid
        V-cycle; precision="mixed" only). recovery=False: a failed system is
        NaN-filled at once (MOF_NO_RECOVERY) instead of re-solved with block
        Jacobi and then fp64. fused (precision="f64"): True -- each batch's
        solve in one launch (MOF_SOLVE_FUSED), False -- never, None -- the
        library's choice (small meshes). etol: the refinement's error
        control -- a system also needs its estimated error below etol max|V|
        (0: the library's 1e-7, < 0: the residual test alone)."""
        o = L.MofOpts()
        o.struct_size = ctypes.sizeof(L.MofOpts)
        o.precision = {"f64": L.MOF_PREC_F64, "mixed": L.MOF_PREC_MIXED}[precision]
        o.flags = ((L.MOF_IO_DEVICE if device_io else 0)
                   | (0 if block_jacobi else L.MOF_NO_BLOCK_JACOBI)
                   | (L.MOF_TIME_SPMV if time_spmv else 0)
                   | {"jacobi": 0, "amg": L.MOF_PRECOND_AMG}[precond]
                   | (0 if recovery else L.MOF_NO_RECOVERY)
                   | {None: 0, True: L.MOF_SOLVE_FUSED, False: L.MOF_SOLVE_EAGER}[fused])
        o.batch = int(batch)
        o.max_iter = int(max_iter)
        o.max_outer = int(max_outer)
        o.rtol = float(rtol)
        o.inner_rtol = float(inner_rtol)
        o.stream = stream
        o.etol = float(etol)
        return o

    def fingerprint(self) -> str:
        """Digest of the mesh inputs (checkpoint keys, mofhip.solve)."""
        fp = getattr(self, "_fp", None)
        if fp is None:
            from .solve import _digest
            fp = self._fp = _digest(self._xyz, self._nrm, self._tri, self._area, self.f32_points)
        return fp

    def solve_range(self, I, t_k, k0, k1, lambda_, I2=None, device=None, raise_on_noconv=False, out=None,
                    **opts):
        """V for k in [k0, k1): (k1-k0, 2N) float64 host array, plus stats.
        ``out``: a C-contiguous float64 (k1-k0, 2N) array to write V into."""
        I = _f64(I)
        I2a = I if I2 is None else _f64(I2)
        tk = _f64(t_k)
        T = I.shape[0]
        if I.ndim != 2 or I.shape[1] != self.N or I2a.shape != I.shape:
            raise ValueError("I and I_2 must be (T, N)")
        if len(tk) < T:
            raise ValueError("t_k needs at least T entries")
        shape = (max(k1 - k0, 0), 2 * self.N)
        if out is None:
            V = np.empty(shape)
        else:
            if out.shape != shape or out.dtype != np.float64 or not out.flags.c_contiguous:
                raise ValueError("out must be a C-contiguous float64 %s array" % (shape,))
            V = out
        st = L.MofStats()
        o = self.make_opts(**opts)
        h = self.handle(device)
        with self.lock(device):
            rc = L.lib().mof_solve_range(h, L.ptr(I), L.ptr(I2a), L.ptr(tk), T, int(k0), int(k1),
                                         float(lambda_), ctypes.byref(o), L.ptr(V),
                                         ctypes.byref(st))
        if rc == L.MOF_E_NOCONV and not raise_on_noconv:
            return V, st.as_dict()
        L.check(rc)
        return V, st.as_dict()

    def solve_range_device(self, I_ptr: int, I2_ptr: int, T: int, t_k, k0: int, k1: int,
                           lambda_, V_ptr: int, device=None, **opts):
        """Device-pointer form (inputs resident in HBM; used by bench.py)."""
        tk = _f64(t_k)
        st = L.MofStats()
        o = self.make_opts(device_io=True, **opts)
        h = self.handle(device)
        with self.lock(device):
            rc = L.lib().mof_solve_range(h, ctypes.c_void_p(I_ptr), ctypes.c_void_p(I2_ptr),
                                         L.ptr(tk), int(T), int(k0), int(k1), float(lambda_),
                                         ctypes.byref(o), ctypes.c_void_p(V_ptr),
                                         ctypes.byref(st))
        if rc != L.MOF_E_NOCONV:
            L.check(rc)
        return st.as_dict()

    def bench_spmv(self, precision="mixed", batch=1, reps=50, device=None):
        ms = ctypes.c_double(0)
        by = ctypes.c_double(0)
        prec = {"f64": L.MOF_PREC_F64, "mixed": L.MOF_PREC_MIXED}[precision]
        with self.lock(device):
            L.check(L.lib().mof_bench_spmv(self.handle(device), prec, int(batch), int(reps),
                                           ctypes.byref(ms), ctypes.byref(by)))
        return ms.value, by.value
