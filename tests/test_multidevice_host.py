"""One-process multi-GPU drop-in (compute_velocity_field over
min(processes_num, #GPUs) devices, compute_optical_flow.py:157-177): the
per-device handles are built concurrently, the extra devices by cloning the
primary handle (shared host pattern and multigrid hierarchy), and before the
drop-in's clock starts. CPU tests with the library stubbed: they check the
host orchestration only (no device code runs)."""
import threading
import time

import numpy as np
import pytest

import mofhip.mesh as mm
from mofhip import synth


class _FakeLib:
    """mof_mesh_create / mof_mesh_clone that sleep, recording their intervals."""

    def __init__(self, create_s=0.05, clone_s=0.3):
        self.create_s, self.clone_s = create_s, clone_s
        self.calls = []
        self.lock = threading.Lock()

    def _rec(self, kind, dev, t0):
        with self.lock:
            self.calls.append((kind, dev, t0, time.perf_counter()))

    def mof_mesh_create(self, xyz, nrm, tri, area, N, M, device, flags, out):
        t0 = time.perf_counter()
        time.sleep(self.create_s)
        self._rec("create", device, t0)
        return 0

    def mof_mesh_clone(self, src, device, out):
        t0 = time.perf_counter()
        time.sleep(self.clone_s)
        self._rec("clone", device, t0)
        return 0

    def mof_mesh_destroy(self, h):
        return 0


@pytest.fixture
def fake(monkeypatch):
    f = _FakeLib()
    monkeypatch.setattr(mm.L, "lib", lambda: f)
    return f


def _mesh():
    p, t = synth.icosphere(4, 10.0)
    return p, synth.vertex_normals(p, t), t, synth.triangle_areas(p, t)


def test_handle_builds_overlap(fake):
    p, n, t, a = _mesh()
    m = mm.DeviceMesh(p, n, t, a, device=0)
    t0 = time.perf_counter()
    secs = m.prepare(range(8))
    wall = time.perf_counter() - t0
    clones = [c for c in fake.calls if c[0] == "clone"]
    assert [c[0] for c in fake.calls].count("create") == 1  # the host pattern is built once per mesh
    assert sorted(c[1] for c in clones) == list(range(1, 8))
    # the 7 clone builds overlap: all started before the first one ended
    assert max(c[2] for c in clones) < min(c[3] for c in clones)
    assert wall < 3 * fake.clone_s  # serialised they would take 7 x clone_s
    assert set(secs) == set(range(8))
    # built once: a second prepare builds nothing
    m.prepare(range(8))
    assert len(fake.calls) == 8


def test_same_device_built_once_under_races(fake):
    p, n, t, a = _mesh()
    m = mm.DeviceMesh(p, n, t, a, device=0)
    threads = [threading.Thread(target=m.handle, args=(3,)) for _ in range(6)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    assert [c[1] for c in fake.calls if c[0] == "clone"] == [3]


def test_drop_in_builds_handles_before_its_clock(fake, monkeypatch):
    """compute_velocity_field prepares every device's handle before it starts
    its timer (the reference creates its Pool before start_time, :155-158):
    the returned execution_time holds the solves only."""
    from utils import compute_optical_flow as cof
    p, n, t, a = _mesh()
    m = mm.DeviceMesh(p, n, t, a, device=0)
    monkeypatch.setattr(cof, "device_count", lambda: 4)
    order = []

    def fake_sharded(mesh, I, tk, k0, k1, lam, I2=None, devices=(0,), **kw):
        order.append(("solve", sorted(mesh._handles)))
        return np.zeros((k1 - k0, 2 * mesh.N)), [{"failed": 0}]

    monkeypatch.setattr(cof, "velocity_field_sharded", fake_sharded)
    I = np.zeros((3, len(p)))
    V, secs = cof.compute_velocity_field(4, 3, m, None, None, None, t, [0, 1, 2], a, 0.01, I, I)
    assert order == [("solve", [0, 1, 2, 3])]
    assert secs < fake.clone_s  # the clone builds are outside the timed call
    assert len(V) == 2
