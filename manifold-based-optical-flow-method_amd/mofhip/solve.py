"""Timestep sharding across the GPUs of one node.

The reference runs one ``worker`` per timestep on a
``multiprocessing.Pool(processes_num)`` (compute_optical_flow.py:157-177);
timesteps are independent, so here each GPU takes one contiguous k-range
(one host thread per device; ctypes releases the GIL) and results are
concatenated in k order (:190-191). No collective is involved.

Checkpoint / resume (``checkpoint=`` a directory): each device's range is
solved in chunks of ``chunk`` timesteps, every finished chunk is written as
``V_<k0>_<k1>.npy`` (atomically, with a fingerprint of the mesh, the
chunk's I rows, t_k, lambda, the solver options, the library version and
the MOF_* environment switches that change V or convergence), and a rerun
loads the chunks whose fingerprint matches instead of solving them again --
the shard-granular counterpart of S3's stage outputs (S3…py:122-137). A
chunk with failed (NaN-filled) systems is written but never reused: a rerun
solves it again, so a resume cannot hide a failure.
"""
from __future__ import annotations

import hashlib
import json
import os
import threading

import numpy as np


def shard_ranges(k0: int, k1: int, parts: int):
    """Split [k0, k1) into ``parts`` contiguous, balanced ranges."""
    parts = max(1, int(parts))
    n = max(0, k1 - k0)
    base, extra = divmod(n, parts)
    out, start = [], k0
    for p in range(parts):
        size = base + (1 if p < extra else 0)
        out.append((start, start + size))
        start += size
    return out


def _hasher():
    try:
        import xxhash
        return xxhash.xxh3_128()
    except ImportError:  # pragma: no cover
        return hashlib.blake2b(digest_size=16)


def _digest(*parts) -> str:
    h = _hasher()
    for p in parts:
        if isinstance(p, np.ndarray):
            h.update(np.ascontiguousarray(p).view(np.uint8).reshape(-1).data)
        else:
            h.update(repr(p).encode())
    return h.hexdigest()


# MOF_* switches that cannot change a saved V: logging, the host staging
# size, host threads, the RCCL library path (csrc/mof_knobs.h), and the
# checkpoint's own settings. The library's other switches (MOF_SYM_READS,
# MOF_AMG_SMOOTH, MOF_AMG_OMEGA, MOF_AMG_BSW) change V bits and key the chunk.
_KEY_NEUTRAL = frozenset((
    "MOF_CHECKPOINT_DIR", "MOF_CHECKPOINT_CHUNK", "MOF_VERBOSE", "MOF_STAGE_MB", "MOF_IO_THREADS", "MOF_RCCL_LIB",
))


def _library_key() -> tuple:
    """Library version and ABI, and the MOF_* environment switches that may
    change V (sorted; _KEY_NEUTRAL excluded): a rebuilt library or another
    solver setting must not reuse old chunks, a log switch must not discard
    them."""
    try:
        from . import _lib as L
        lib = L.lib()
        ver = (lib.mof_version().decode(), int(lib.mof_abi_version()))
    except Exception:  # no library (CPU tests with a stand-in mesh)
        ver = ("", 0)
    env = tuple(sorted((k, v) for k, v in os.environ.items() if k.startswith("MOF_")
                       and k not in _KEY_NEUTRAL))
    return ver, env


def chunk_fingerprint(mesh, I, I2, t_k, a, b, lambda_, opts) -> str:
    """What a saved chunk's V depends on: the mesh (and its device vertex
    order), timesteps [a, b)'s I rows (I[a:b] and I2[a+1:b+1]), t_k[a:b+1],
    lambda, the solver options and the library / environment key."""
    I2 = I if I2 is None else I2
    return _digest(mesh.fingerprint(), bool(getattr(mesh, "reorder", True)), np.asarray(I[a:b]),
                   np.asarray(I2[a + 1:b + 1]), np.asarray(t_k[a:b + 1], dtype=np.float64), float(lambda_),
                   sorted(opts.items()), _library_key())


class Checkpoint:
    """Shard-granular V chunks in a directory (see the module docstring)."""

    def __init__(self, path: str):
        self.path = path
        os.makedirs(path, exist_ok=True)

    def _files(self, a, b):
        stem = os.path.join(self.path, "V_%09d_%09d" % (a, b))
        return stem + ".npy", stem + ".json"

    def load(self, a, b, fp, out):
        """The saved chunk's stats (its V copied into ``out``), or None when
        there is no usable chunk: missing, another fingerprint, another shape,
        or one with failed systems (those are solved again)."""
        vf, mf = self._files(a, b)
        try:
            with open(mf) as f:
                meta = json.load(f)
            if meta.get("fingerprint") != fp:
                return None
            stats = dict(meta.get("stats") or {})
            if int(stats.get("failed", 0)) > 0:
                return None
            arr = np.load(vf, mmap_mode="r", allow_pickle=False)
            if arr.shape != out.shape:
                return None
            out[...] = arr
            return stats
        except (OSError, ValueError, TypeError):
            return None

    def save(self, a, b, fp, V, stats):
        vf, mf = self._files(a, b)
        tmp = vf + ".tmp%d" % threading.get_ident()
        with open(tmp, "wb") as f:
            np.save(f, V, allow_pickle=False)
        os.replace(tmp, vf)
        meta = {"k0": a, "k1": b, "fingerprint": fp,
                "stats": {k: v for k, v in stats.items() if isinstance(v, (int, float))}}
        tmpm = mf + ".tmp%d" % threading.get_ident()
        with open(tmpm, "w") as f:
            json.dump(meta, f)
        os.replace(tmpm, mf)  # the manifest last: a chunk counts once both are complete


def velocity_field_sharded(mesh, I, t_k, k0, k1, lambda_, I2=None, devices=(0,), checkpoint=None, chunk=0,
                           **opts):
    """Solve k in [k0, k1) on ``devices``; returns (V (k1-k0, 2N), [stats per
    device]). ``checkpoint``: a directory for shard-granular resume, chunks of
    ``chunk`` timesteps (0: 512)."""
    devices = list(devices) or [mesh.device]
    mesh.prepare(devices)  # concurrent handle builds (clones share the host state)
    ranges = shard_ranges(k0, k1, len(devices))
    V = np.empty((max(k1 - k0, 0), 2 * mesh.N))
    stats = [None] * len(devices)
    errors = [None] * len(devices)
    ck = Checkpoint(checkpoint) if checkpoint else None
    csize = int(chunk) if chunk and int(chunk) > 0 else 512

    def run(slot, dev, a, b):
        try:
            if b <= a:
                return
            if ck is None:
                _, stats[slot] = mesh.solve_range(I, t_k, a, b, lambda_, I2=I2, device=dev, out=V[a - k0:b - k0],
                                                  **opts)
                return
            acc = None
            for c0 in range(a, b, csize):
                c1 = min(b, c0 + csize)
                dst = V[c0 - k0:c1 - k0]
                fp = chunk_fingerprint(mesh, I, I2, t_k, c0, c1, lambda_, opts)
                saved = ck.load(c0, c1, fp, dst)
                if saved is not None:
                    # the saved run's counts (systems, iterations, ...) carry
                    # over; nothing was solved now
                    st = dict(saved, resumed=c1 - c0)
                else:
                    _, st = mesh.solve_range(I, t_k, c0, c1, lambda_, I2=I2, device=dev, out=dst, **opts)
                    ck.save(c0, c1, fp, dst, st)
                    st = dict(st, resumed=0)
                acc = st if acc is None else _merge(acc, st)
            stats[slot] = acc
        except BaseException as exc:  # re-raised in the caller
            errors[slot] = exc

    if len(devices) == 1:
        run(0, devices[0], *ranges[0])
    else:
        threads = [threading.Thread(target=run, args=(s, d, a, b))
                   for s, (d, (a, b)) in enumerate(zip(devices, ranges))]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
    for e in errors:
        if e is not None:
            raise e
    return V, [s for s in stats if s is not None]


def _merge(a: dict, b: dict) -> dict:
    out = dict(a)
    for k, v in b.items():
        if k.startswith("max_"):
            out[k] = max(out.get(k, v), v)
        elif isinstance(v, (int, float)) and not isinstance(v, bool):
            out[k] = out.get(k, 0) + v
    return out
