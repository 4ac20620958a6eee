"""The per-rank decomposition path across processes, on one GPU.

RCCL refuses two ranks on one device, so the one-part-per-rank transport is
exercised here through its host-staged twin (include/mof.h
mof_dd_create_rank_host): every rank builds only its own part's plan and
mesh, packs its halo segments and partial records with the RCCL transport's
kernels and segment order, and a torch.distributed gloo group carries the
exchanges (mofhip.decomp.HostTransport). V must be bit-identical to the
in-process solve over the same kernels (MOF_DD_STAGED), which the other
tests tie to spsolve. The RCCL calls themselves stay unmeasured on hardware
(one GPU per box)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _case():
    from mofhip import synth
    p, t = synth.icosphere(16, jitter=0.005)
    n, a = synth.vertex_normals(p, t), synth.triangle_areas(p, t)
    return p, t, n, a, synth.travelling_wave(p, 6)


def _rank_worker(rank, world, port, part, opts, out, env=None, oom_rank=-1):
    import sys
    os.environ.update(env or {})
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    sys.path.insert(0, os.path.join(repo, "manifold-based-optical-flow-method_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mofhip import DecomposedMesh
        p, t, n, a, I = _case()
        d = DecomposedMesh(p, n, t, a, world, part=part, group=dist.group.WORLD, transport="host")
        if oom_rank >= 0:
            from mofhip import _lib as L
            L.check(L.lib().mof_dd_test_fail_recovery_alloc(d._h, oom_rank))
        info = d.info()
        V, st = d.solve_range(I, np.arange(len(I), dtype=np.float64), 0, len(I) - 1, 0.01, **opts)
        d.close()
        out.put((rank, info["local_parts"], info["rank"], V, st["iterations"], st["failed"]))
    except BaseException as exc:  # reported to the parent
        out.put((rank, None, None, repr(exc), None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("P,opts", [
    (2, {"precision": "mixed", "batch": 3}),
    (3, {"precision": "f64", "batch": 5}),
    (3, {"precision": "mixed", "precond": "amg", "batch": 2}),
])
def test_host_transport_ranks_match_in_process(P, opts):
    import torch.multiprocessing as mp
    from mofhip import DecomposedMesh
    p, t, n, a, I = _case()
    part = np.random.default_rng(5).integers(0, P, len(p)).astype(np.int32)
    ref = DecomposedMesh(p, n, t, a, P, part=part, staged=True)
    Vr, sr = ref.solve_range(I, np.arange(len(I), dtype=np.float64), 0, len(I) - 1, 0.01, **opts)
    ref.close()
    assert sr["failed"] == sr["recovered"] == 0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker, args=(r, P, port, part, opts, q)) for r in range(P)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=240) for _ in range(P)], key=lambda x: x[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    for rank, local, r, V, its, failed in res:
        assert local == 1 and r == rank, V
        assert failed == 0 and its == sr["iterations"]
        assert np.array_equal(V, Vr)  # every rank receives the whole V, bit for bit


@pytest.mark.parametrize("oom_rank", [-1, 1])
def test_recovery_allocation_failure_agreed_by_all_ranks(oom_rank):
    """The fp64 recovery pass allocates its workspace per rank; a failure on
    one rank (injected: mof_dd_test_fail_recovery_alloc) is agreed by an all-gather of a
    status word before the pass's collectives, so every rank skips the pass
    and returns its systems NaN-filled instead of hanging in the halo
    exchange. Without the failure the same pass recovers
    every system. The first solve fails by construction (2 inner iterations,
    one refinement step)."""
    import torch.multiprocessing as mp
    from mofhip import DecomposedMesh
    p, t, n, a, I = _case()
    P = 2
    part = np.random.default_rng(5).integers(0, P, len(p)).astype(np.int32)
    opts = {"precision": "mixed", "batch": 3, "max_iter": 2, "max_outer": 1}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker, args=(r, P, port, part, opts, q, None, oom_rank)) for r in range(P)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=240) for _ in range(P)], key=lambda x: x[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    T = len(I) - 1
    for rank, local, r, V, its, failed in res:
        assert local == 1 and r == rank, V
        if oom_rank < 0:
            assert failed == 0 and np.isfinite(V).all()
        else:
            assert failed == T and np.isnan(V).all()
    if oom_rank < 0:
        ref = DecomposedMesh(p, n, t, a, P, part=part, staged=True)
        Vr, _ = ref.solve_range(I, np.arange(len(I), dtype=np.float64), 0, T, 0.01, precision="f64", batch=3)
        ref.close()
        assert np.max(np.abs(res[0][3] - Vr)) < 1e-6
