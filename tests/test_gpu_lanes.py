"""Two batches in flight per GPU (MOF_TWO_LANES, mof_solve_range): batches
alternate between the handle and a twin on the same device, each lane on its
own host thread and stream. Batch composition is unchanged, so V and every
count must be bit-identical to the one-lane solve."""
import numpy as np
import pytest
import torch

from mofhip import DeviceMesh, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def case():
    p, t = synth.icosphere(32, jitter=0.005)
    m = DeviceMesh(p, synth.vertex_normals(p, t), t, synth.triangle_areas(p, t))
    I = synth.travelling_wave(p, 81)
    return m, I, np.arange(81, dtype=np.float64)


@pytest.mark.parametrize("opts", [
    dict(precision="mixed", precond="amg", batch=16),
    dict(precision="mixed", precond="amg", batch=24),   # ragged last batch
    dict(precision="f64", precond="jacobi", batch=32, fused=False),
])
def test_two_lanes_bit_identical_host_io(case, opts):
    m, I, tk = case
    V1, s1 = m.solve_range(I, tk, 0, 80, 0.01, **opts)
    V2, s2 = m.solve_range(I, tk, 0, 80, 0.01, lanes=2, **opts)
    assert np.array_equal(V1, V2)
    for k in ("iterations", "max_iterations", "failed", "batches", "max_rel_residual", "systems"):
        assert s1[k] == s2[k], k
    assert s2["failed"] == 0


def test_two_lanes_bit_identical_device_io(case):
    m, I, tk = case
    dev = torch.device("cuda", 0)
    Id = torch.from_numpy(I).to(dev)
    V1 = torch.empty((80, 2 * m.N), dtype=torch.float64, device=dev)
    V2 = torch.empty_like(V1)
    opts = dict(precision="mixed", precond="amg", batch=16, time_spmv=True)
    s1 = m.solve_range_device(Id.data_ptr(), Id.data_ptr(), 81, tk, 0, 80, 0.01, V1.data_ptr(), **opts)
    s2 = m.solve_range_device(Id.data_ptr(), Id.data_ptr(), 81, tk, 0, 80, 0.01, V2.data_ptr(), lanes=2, **opts)
    torch.cuda.synchronize(dev)
    assert torch.equal(V1, V2)
    assert s1["iterations"] == s2["iterations"] and s1["spmv_systems"] == s2["spmv_systems"]
