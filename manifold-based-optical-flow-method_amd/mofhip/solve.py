"""Timestep sharding across the GPUs of one node.

The reference runs one ``worker`` per timestep on a
``multiprocessing.Pool(processes_num)`` (compute_optical_flow.py:157-177);
timesteps are independent, so here each GPU takes one contiguous k-range
(one host thread per device; ctypes releases the GIL) and results are
concatenated in k order (:190-191). No collective is involved.
"""
from __future__ import annotations

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


def velocity_field_sharded(mesh, I, t_k, k0, k1, lambda_, I2=None, devices=(0,), **opts):
    """Solve k in [k0, k1) on ``devices``; returns (V (k1-k0, 2N), [stats per device])."""
    devices = list(devices) or [mesh.device]
    mesh.prepare(devices)  # concurrent handle builds (clones share the host state)
    ranges = shard_ranges(k0, k1, len(devices))
    V = np.empty((max(k1 - k0, 0), 2 * mesh.N))
    stats = [None] * len(devices)
    errors = [None] * len(devices)

    def run(slot, dev, a, b):
        try:
            if b > a:
                Vs, st = mesh.solve_range(I, t_k, a, b, lambda_, I2=I2, device=dev, **opts)
                V[a - k0:b - k0] = Vs
                stats[slot] = st
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
