"""Small batches replay their PCG iteration chunks from HIP graphs (the
eager launches captured once per chunk shape, csrc/mof_pcg.hip): the same
kernels with the same arguments, so V and every count are bit-identical to
the eager launches (MOF_GRAPHS=0), for the multigrid and the block-Jacobi
inner solves, across repeated calls (replays) and ragged batches."""
import numpy as np
import pytest

from mofhip import DeviceMesh, synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg,opts", [
    ("C1", dict(precision="mixed", precond="amg", batch=0)),
    ("C1", dict(precision="mixed", precond="jacobi", batch=6)),
    ("S1s", dict(precision="mixed", precond="amg", batch=16)),
    ("C1", dict(precision="f64", precond="jacobi", batch=5, fused=False)),
])
def test_graphs_bit_identical_to_eager(cfg, opts, monkeypatch):
    p, t, n, a = synth.mesh_for_config(cfg)
    I = synth.config_wave(cfg, p, 41)
    tk = np.arange(41, dtype=np.float64)
    out = {}
    for g in ("0", "1"):
        monkeypatch.setenv("MOF_GRAPHS", g)
        m = DeviceMesh(p, n, t, a)
        res = []
        for _ in range(2):  # the second call replays the captured chunks
            V, st = m.solve_range(I, tk, 0, 40, 0.01, **opts)
            res.append((V, st))
        out[g] = res
        m.close()
    for (Ve, se), (Vg, sg) in zip(out["0"], out["1"]):
        assert np.array_equal(Ve, Vg)
        for k in ("iterations", "max_iterations", "failed", "recovered", "outer_steps"):
            assert se[k] == sg[k], k
        assert sg["failed"] == 0
