"""Driver for tools/spmv_tri_proto.hip: writes the C3
mesh (icosphere frequency 128, 163,842 vertices) in RCM vertex order with
triangles sorted by smallest vertex, tangent bases from the sphere normals and
A_T/12 weights, then runs the micro-benchmark binary as a child process.

    python tools/spmv_tri_proto.py [--freq 128] [--B 256] [--reps 20]
"""
import argparse
import os
import subprocess
import sys

import numpy as np
import scipy.sparse as sp
from scipy.sparse.csgraph import reverse_cuthill_mckee

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "manifold-based-optical-flow-method_amd"))
from mofhip.synth import icosphere  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--freq", type=int, default=128)
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--out", default="gpurun_out/spmv_tri_mesh.bin")
    a = ap.parse_args()
    pts, tri = icosphere(a.freq, jitter=0.01, seed=1)
    N = len(pts)
    e = np.concatenate([tri[:, [0, 1]], tri[:, [1, 2]], tri[:, [2, 0]]])
    adj = sp.coo_matrix((np.ones(len(e)), (e[:, 0], e[:, 1])), shape=(N, N)).tocsr()
    adj = adj + adj.T
    perm = reverse_cuthill_mckee(adj, symmetric_mode=True)
    new = np.empty(N, np.int64)
    new[perm] = np.arange(N)
    pts = pts[perm]
    tri = new[tri]
    tri = tri[np.argsort(tri.min(axis=1), kind="stable")].astype(np.int32)
    n = pts / np.linalg.norm(pts, axis=1, keepdims=True)
    ref = np.where(np.abs(n[:, 2:3]) < 0.9, [[0.0, 0.0, 1.0]], [[1.0, 0.0, 0.0]])
    e1 = np.cross(n, ref)
    e1 /= np.linalg.norm(e1, axis=1, keepdims=True)
    e2 = np.cross(n, e1)
    E = np.concatenate([e1, e2], axis=1).astype(np.float32)
    p = pts[tri]
    area = 0.5 * np.linalg.norm(np.cross(p[:, 1] - p[:, 0], p[:, 2] - p[:, 0]), axis=1)
    w12 = (area / 12.0).astype(np.float32)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "wb") as f:
        np.array([N, len(tri)], np.int32).tofile(f)
        tri.tofile(f)
        E.tofile(f)
        w12.tofile(f)
    exe = os.path.join(HERE, "spmv_tri_proto")
    return subprocess.call([exe, a.out, str(a.B), str(a.reps)])


if __name__ == "__main__":
    sys.exit(main())
