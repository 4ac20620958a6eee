"""Shard-granular checkpoint / resume of the sharded solve (mofhip.solve;
the drop-in's compute_velocity_field with MOF_CHECKPOINT_DIR). The stage
outputs of the reference's S3 are its checkpoints (S3…py:122-137); here the
unit is a chunk of timesteps per device. CPU tests with a stand-in mesh whose
solve writes a known function of (k, I rows) and counts its calls."""
import os

import numpy as np

from mofhip.solve import velocity_field_sharded


class _Mesh:
    N = 5
    device = 0

    def __init__(self):
        self.calls = []

    def prepare(self, devices):
        return {}

    def fingerprint(self):
        return "mesh-1"

    def solve_range(self, I, t_k, k0, k1, lam, I2=None, device=None, out=None, **opts):
        self.calls.append((device, k0, k1))
        I2 = I if I2 is None else I2
        for k in range(k0, k1):
            out[k - k0] = np.concatenate([I[k] * lam, I2[k + 1] + t_k[k]])
        return out, {"systems": k1 - k0, "failed": 0, "iterations": 3 * (k1 - k0), "max_iterations": 3}


def _inputs(T=23, N=5, seed=0):
    rng = np.random.default_rng(seed)
    return rng.standard_normal((T, N)), np.arange(float(T))


def test_resume_skips_saved_chunks(tmp_path):
    I, tk = _inputs()
    m = _Mesh()
    V1, st1 = velocity_field_sharded(m, I, tk, 0, 22, 0.5, devices=[0, 1], checkpoint=str(tmp_path), chunk=4)
    n1 = len(m.calls)
    assert n1 == 6  # two shards of 11 timesteps, chunks of 4: 3 + 3
    assert sum(s["systems"] for s in st1) == 22
    files = sorted(os.listdir(tmp_path))
    assert len([f for f in files if f.endswith(".npy")]) == 6
    # a rerun loads every chunk, solves nothing, and returns the same V
    V2, st2 = velocity_field_sharded(m, I, tk, 0, 22, 0.5, devices=[0, 1], checkpoint=str(tmp_path), chunk=4)
    assert len(m.calls) == n1
    assert np.array_equal(V1, V2)
    assert sum(s["resumed"] for s in st2) == 22
    # an interrupted run: one chunk's manifest missing -> only that chunk is solved again
    os.remove(os.path.join(tmp_path, "V_000000004_000000008.json"))
    V3, _ = velocity_field_sharded(m, I, tk, 0, 22, 0.5, devices=[0, 1], checkpoint=str(tmp_path), chunk=4)
    assert m.calls[n1:] == [(0, 4, 8)]
    assert np.array_equal(V1, V3)


def test_changed_inputs_invalidate_chunks(tmp_path):
    I, tk = _inputs()
    m = _Mesh()
    V1, _ = velocity_field_sharded(m, I, tk, 0, 22, 0.5, checkpoint=str(tmp_path), chunk=8)
    n1 = len(m.calls)
    # another lambda: every chunk is stale
    velocity_field_sharded(m, I, tk, 0, 22, 0.25, checkpoint=str(tmp_path), chunk=8)
    assert len(m.calls) == 2 * n1
    # one changed I row: only the chunks that read it (k = 9 feeds chunk [8, 16) and, as k + 1, chunk [0, 8))
    I2 = I.copy()
    I2[8, 0] += 1.0
    velocity_field_sharded(m, I2, tk, 0, 22, 0.25, checkpoint=str(tmp_path), chunk=8)
    assert sorted(m.calls[2 * n1:]) == [(0, 0, 8), (0, 8, 16)]
    # solver options are part of the key
    velocity_field_sharded(m, I2, tk, 0, 22, 0.25, checkpoint=str(tmp_path), chunk=8, precision="f64")
    assert len(m.calls) == 2 * n1 + 2 + 3


def test_no_checkpoint_writes_in_place():
    I, tk = _inputs()
    m = _Mesh()
    V, st = velocity_field_sharded(m, I, tk, 3, 20, 2.0, devices=[0, 1, 2])
    assert [c[1:] for c in m.calls] == [(3, 9), (9, 15), (15, 20)]
    ref = np.stack([np.concatenate([I[k] * 2.0, I[k + 1] + tk[k]]) for k in range(3, 20)])
    assert np.array_equal(V, ref)


class _FailingMesh(_Mesh):
    """Reports one failed (NaN-filled) system in every chunk containing k = 5."""

    def solve_range(self, I, t_k, k0, k1, lam, I2=None, device=None, out=None, **opts):
        out, st = super().solve_range(I, t_k, k0, k1, lam, I2=I2, device=device, out=out, **opts)
        if k0 <= 5 < k1:
            out[5 - k0] = np.nan
            st = dict(st, failed=1)
        return out, st


def test_failed_chunks_are_solved_again(tmp_path):
    I, tk = _inputs()
    m = _FailingMesh()
    _, st1 = velocity_field_sharded(m, I, tk, 0, 12, 0.5, checkpoint=str(tmp_path), chunk=4)
    assert sum(s["failed"] for s in st1) == 1
    n1 = len(m.calls)
    # the rerun reuses the clean chunks (with their saved counts) and solves
    # the failed one again, whose failure is reported again
    V2, st2 = velocity_field_sharded(m, I, tk, 0, 12, 0.5, checkpoint=str(tmp_path), chunk=4)
    assert m.calls[n1:] == [(0, 4, 8)]
    assert st2[0]["failed"] == 1
    assert st2[0]["resumed"] == 8
    assert st2[0]["systems"] == 12  # saved 4 + 4, solved 4
    assert np.isnan(V2[5]).all()


def test_environment_switches_invalidate_chunks(tmp_path, monkeypatch):
    I, tk = _inputs()
    m = _Mesh()
    monkeypatch.delenv("MOF_AMG_OMEGA", raising=False)
    velocity_field_sharded(m, I, tk, 0, 8, 0.5, checkpoint=str(tmp_path), chunk=8)
    velocity_field_sharded(m, I, tk, 0, 8, 0.5, checkpoint=str(tmp_path), chunk=8)
    assert len(m.calls) == 1
    monkeypatch.setenv("MOF_AMG_OMEGA", "0.8")  # a solver switch: the chunk is stale
    velocity_field_sharded(m, I, tk, 0, 8, 0.5, checkpoint=str(tmp_path), chunk=8)
    assert len(m.calls) == 2
    m.reorder = False  # another device vertex order: stale as well
    velocity_field_sharded(m, I, tk, 0, 8, 0.5, checkpoint=str(tmp_path), chunk=8)
    assert len(m.calls) == 3


def test_log_switches_keep_chunks(tmp_path, monkeypatch):
    """Switches that cannot change V (logging, staging sizes, host threads)
    leave the saved chunks valid (round-4 advisor)."""
    I, tk = _inputs()
    m = _Mesh()
    for k in ("MOF_VERBOSE", "MOF_STAGE_MB", "MOF_IO_THREADS"):
        monkeypatch.delenv(k, raising=False)
    velocity_field_sharded(m, I, tk, 0, 8, 0.5, checkpoint=str(tmp_path), chunk=8)
    monkeypatch.setenv("MOF_VERBOSE", "1")
    monkeypatch.setenv("MOF_STAGE_MB", "8")
    monkeypatch.setenv("MOF_IO_THREADS", "3")
    velocity_field_sharded(m, I, tk, 0, 8, 0.5, checkpoint=str(tmp_path), chunk=8)
    assert len(m.calls) == 1
