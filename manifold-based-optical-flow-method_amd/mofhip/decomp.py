"""Domain-decomposed solve: one timestep's system
split over P vertex parts, PCG iterations in lockstep with a halo exchange.

Timestep shards (:mod:`mofhip.solve`) stay the throughput path; this is the
path for a mesh one GPU should not hold alone, or for the latency of a single
timestep. Two transports (include/mof.h, ``mof_dd_*``):

* :class:`DecomposedMesh` -- all P parts in this process on one device
  (in-process halo gather, shared partial sums);
* :class:`DecomposedMesh` with ``group=`` -- one part per rank of a
  ``torch.distributed`` job (one process per GPU), halo and scalar reductions
  over RCCL; rank 0 makes the RCCL id and ``group`` broadcasts it;
* the same with ``transport="host"`` -- the per-rank plans and pack / unpack
  kernels of the RCCL transport, every exchange staged through host memory
  and carried by ``group`` itself (gloo): no RCCL, and ranks may share a GPU.

Both return V in the reference's planar layout and caller order, like
:meth:`DeviceMesh.solve_range` (compute_optical_flow.py:147, :190-191).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L
from .mesh import DeviceMesh, _f64


def partition_rcb(coordinates, nparts: int) -> np.ndarray:
    """Recursive coordinate bisection: (N,) part id per vertex (host)."""
    xyz = _f64(coordinates)
    part = np.empty(len(xyz), np.int32)
    L.check(L.lib().mof_partition_rcb(L.ptr(xyz), len(xyz), int(nparts), L.ptr(part)))
    return part


def plan_info(triangles, N: int, part) -> dict:
    """Per-part halo plan of a vertex partition (host): owned, ghost,
    neighbour, local-triangle and send-row counts."""
    tri = np.ascontiguousarray(triangles, dtype=np.int32)
    part = np.ascontiguousarray(part, dtype=np.int32)
    P = int(part.max()) + 1 if len(part) else 0
    out = {k: np.empty(P, np.int32) for k in ("n_own", "n_ghost", "n_nbr", "n_tri")}
    out["n_send"] = np.empty(P, np.int64)
    L.check(L.lib().mof_dd_plan_info(L.ptr(tri), int(N), len(tri), P, L.ptr(part),
                                     L.ptr(out["n_own"]), L.ptr(out["n_ghost"]),
                                     L.ptr(out["n_nbr"]), L.ptr(out["n_tri"]),
                                     L.ptr(out["n_send"])))
    return out


class HostTransport:
    """mof_dd_transport over a torch.distributed group (gloo, CPU tensors):
    the all-gather of partial records / owned V and the neighbour exchange of
    packed halo segments, called from inside the solver loop.

    Errors end the solve on every rank, not only on the rank that saw them:
    a local failure inside an exchange (copying a segment in or out) still
    completes that exchange's sends and receives with placeholder bytes, and
    every all-gather carries a status byte, so the next all-gather (the solver
    runs one after every exchange) returns failure on all ranks at the same
    call. A failure of the transport itself (a peer gone) can only end at the
    process group's timeout: create the group with a short ``timeout`` for
    this transport."""

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist
        self._dist, self._torch, self.group = dist, torch, group
        self.world = dist.get_world_size(group)
        self._failed = False  # a local error waiting to be reported to every rank
        self._ag = L.ALLGATHER_FN(self._allgather)
        self._ex = L.EXCHANGE_FN(self._exchange)
        self.struct = L.MofDdTransport(None, self._ag, self._ex)

    def _peer(self, r):
        g = self.group
        if g is None or not hasattr(self._dist, "get_global_rank"):
            return int(r)
        return self._dist.get_global_rank(g, int(r))

    def _allgather(self, ctx, send, recv, nbytes):
        t = self._torch
        try:
            src = t.zeros(nbytes + 1, dtype=t.uint8)
            try:
                src[1:] = t.frombuffer(bytearray(ctypes.string_at(send, nbytes)), dtype=t.uint8)
            except Exception:
                self._failed = True
            src[0] = 1 if self._failed else 0
            out = [t.empty(nbytes + 1, dtype=t.uint8) for _ in range(self.world)]
            self._dist.all_gather(out, src, group=self.group)
        except Exception:  # the transport itself failed
            return 1
        if any(int(o[0]) for o in out):
            self._failed = False
            return 1  # some rank failed: every rank reports it at this call
        try:
            for r, o in enumerate(out):
                ctypes.memmove(recv + r * nbytes, o.data_ptr() + 1, nbytes)
        except Exception:
            return 1  # local only, after the collective: the peers are not blocked
        return 0

    def _exchange(self, ctx, n, peers, send, sbytes, recv, rbytes):
        t = self._torch
        try:
            reqs, bufs = [], []
            for k in range(n):
                if sbytes[k]:
                    try:
                        st = t.frombuffer(bytearray(ctypes.string_at(send[k], sbytes[k])), dtype=t.uint8)
                    except Exception:
                        self._failed = True
                        st = t.zeros(sbytes[k], dtype=t.uint8)
                    reqs.append(self._dist.isend(st, self._peer(peers[k]), group=self.group))
                if rbytes[k]:
                    rt = t.empty(rbytes[k], dtype=t.uint8)
                    bufs.append((k, rt))
                    reqs.append(self._dist.irecv(rt, self._peer(peers[k]), group=self.group))
            for q in reqs:
                q.wait()
        except Exception:  # the transport itself failed
            return 1
        try:
            for k, rt in bufs:
                ctypes.memmove(recv[k], rt.data_ptr(), rbytes[k])
        except Exception:
            self._failed = True
        return 0


class DecomposedMesh:
    """One mesh decomposed into ``nparts`` vertex parts (RCB unless ``part``
    is given). Without ``group`` every part lives in this process on
    ``device``; with a torch.distributed ``group`` this rank drives part
    ``group.rank()`` on ``device`` and ``nparts`` must equal the group size.
    ``staged`` (in-process only): exchange through the pack / copy / unpack
    kernels of the RCCL transport (a one-GPU rehearsal of that path).
    ``transport`` (with ``group``): "rccl" (default) or "host" (host-staged
    exchanges over ``group``, see :class:`HostTransport`)."""

    def __init__(self, coordinates, normals, triangles, areas, nparts: int, device: int = 0,
                 part=None, group=None, rank=None, staged: bool = False, transport: str = "rccl"):
        coords = np.asarray(coordinates)
        tri = np.asarray(triangles)
        if coords.ndim != 2 or coords.shape[1] != 3 or tri.ndim != 2 or tri.shape[1] != 3:
            raise ValueError("coordinates must be (N, 3) and triangles (M, 3)")
        self.f32_points = coords.dtype == np.float32
        self._xyz = _f64(coords)
        self._nrm = _f64(normals)
        self._tri = np.ascontiguousarray(tri, dtype=np.int32)
        self._area = _f64(np.asarray(areas).reshape(-1))
        self.N = len(self._xyz)
        self.M = len(self._tri)
        if self._nrm.shape != (self.N, 3) or len(self._area) != self.M:
            raise ValueError("normals must be (N, 3) and areas (M,)")
        self.nparts = int(nparts)
        self._part = None if part is None else np.ascontiguousarray(part, dtype=np.int32)
        if self._part is not None and self._part.shape != (self.N,):
            raise ValueError("part must be (N,)")
        self.device = int(device)
        flags = ((L.MOF_GEOM_F32_POINTS if self.f32_points else 0)
                 | (L.MOF_DD_STAGED if staged else 0))
        h = ctypes.c_void_p()
        pp = L.ptr(self._part) if self._part is not None else None
        if group is None:
            L.check(L.lib().mof_dd_create(L.ptr(self._xyz), L.ptr(self._nrm), L.ptr(self._tri),
                                          L.ptr(self._area), self.N, self.M, self.nparts, pp,
                                          self.device, flags, ctypes.byref(h)))
        else:
            import torch.distributed as dist
            r = dist.get_rank(group) if rank is None else int(rank)
            if dist.get_world_size(group) != self.nparts:
                raise ValueError("nparts must equal the group size (one part per rank)")
            if transport == "host":
                self._transport = HostTransport(group)
                L.check(L.lib().mof_dd_create_rank_host(
                    L.ptr(self._xyz), L.ptr(self._nrm), L.ptr(self._tri), L.ptr(self._area), self.N, self.M,
                    self.nparts, pp, r, ctypes.byref(self._transport.struct), self.device, flags,
                    ctypes.byref(h)))
                self._h = h
                return
            if transport != "rccl":
                raise ValueError("transport must be 'rccl' or 'host'")
            ident = np.zeros(L.MOF_DD_ID_BYTES, np.uint8)
            if r == 0:
                L.check(L.lib().mof_dd_unique_id(L.ptr(ident)))
            box = [ident.tobytes()]
            dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if hasattr(
                dist, "get_global_rank") else 0, group=group)
            ident = np.frombuffer(box[0], np.uint8).copy()
            L.check(L.lib().mof_dd_create_rank(L.ptr(self._xyz), L.ptr(self._nrm),
                                               L.ptr(self._tri), L.ptr(self._area), self.N,
                                               self.M, self.nparts, pp, r, L.ptr(ident),
                                               self.device, flags, ctypes.byref(h)))
        self._h = h

    def info(self) -> dict:
        inf = L.MofDdInfo()
        L.check(L.lib().mof_dd_get_info(self._h, ctypes.byref(inf)))
        return {k: getattr(inf, k) for k, _ in inf._fields_ if k != "pad_"}

    def close(self):
        if getattr(self, "_h", None):
            L.lib().mof_dd_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def solve_range(self, I, t_k, k0, k1, lambda_, I2=None, raise_on_noconv=False, **opts):
        """V for k in [k0, k1): (k1-k0, 2N) float64 host array, plus stats
        (options as :meth:`DeviceMesh.make_opts`; precond "amg" = a multigrid
        V-cycle per part on its owned rows, block Jacobi across the parts)."""
        I = _f64(I)
        I2a = I if I2 is None else _f64(I2)
        tk = _f64(t_k)
        T = I.shape[0]
        if I.ndim != 2 or I.shape[1] != self.N or I2a.shape != I.shape:
            raise ValueError("I and I_2 must be (T, N)")
        if len(tk) < T:
            raise ValueError("t_k needs at least T entries")
        V = np.empty((max(k1 - k0, 0), 2 * self.N))
        st = L.MofStats()
        o = DeviceMesh.make_opts(**opts)
        rc = L.lib().mof_dd_solve_range(self._h, L.ptr(I), L.ptr(I2a), L.ptr(tk), T, int(k0),
                                        int(k1), float(lambda_), ctypes.byref(o), L.ptr(V),
                                        ctypes.byref(st))
        if rc == L.MOF_E_NOCONV and not raise_on_noconv:
            return V, st.as_dict()
        L.check(rc)
        return V, st.as_dict()

    def solve_range_device(self, I_ptr: int, I2_ptr: int, T: int, t_k, k0: int, k1: int,
                           lambda_, V_ptr: int, **opts):
        """Device-pointer form (inputs resident in HBM; bench.py)."""
        tk = _f64(t_k)
        st = L.MofStats()
        o = DeviceMesh.make_opts(device_io=True, **opts)
        rc = L.lib().mof_dd_solve_range(self._h, ctypes.c_void_p(I_ptr), ctypes.c_void_p(I2_ptr),
                                        L.ptr(tk), int(T), int(k0), int(k1), float(lambda_),
                                        ctypes.byref(o), ctypes.c_void_p(V_ptr),
                                        ctypes.byref(st))
        if rc != L.MOF_E_NOCONV:
            L.check(rc)
        return st.as_dict()
