"""Domain-decomposed solve (include/mof.h mof_dd_*).

CPU: the RCB partition and the halo plan (host code through the C ABI)
against a numpy restatement of the plan's definition.
GPU: V of the decomposed solve against spsolve (the oracle, 1e-6 at dt = 1)
and against the single-domain solve (same algorithm, different summation
order), for several part counts, a random (worst-case) partition, fp64 and
mixed precision; determinism; NaN fill on non-convergence; device-resident
I/V; the RCCL transport with one rank.
"""
import numpy as np
import pytest

import oracle
from conftest import load_golden
from mofhip import DecomposedMesh, DeviceMesh, MofError, partition_rcb, plan_info, synth

VTOL = 1e-6


def wave_case(n=24, T=5, jitter=0.005):
    p, t = synth.icosphere(n, jitter=jitter)
    return p, t, synth.vertex_normals(p, t), synth.triangle_areas(p, t), synth.travelling_wave(p, T)


def restated_plan(tri, N, part):
    """Owned / ghost / neighbour / local-triangle counts by definition: a
    part's local triangles touch an owned vertex; its ghosts are their other
    corners; its neighbours own those ghosts."""
    P = part.max() + 1
    own = np.bincount(part, minlength=P)
    ghosts = [set() for _ in range(P)]
    ntri = np.zeros(P, np.int64)
    for T in tri:
        ps = set(part[T])
        for p in ps:
            ntri[p] += 1
            ghosts[p].update(int(v) for v in T if part[v] != p)
    nbr = [len({int(part[v]) for v in g}) for g in ghosts]
    return own, np.array([len(g) for g in ghosts]), np.array(nbr), ntri


# ---- CPU: partition and plan ------------------------------------------------

@pytest.mark.parametrize("P", [1, 2, 3, 5, 8])
def test_rcb_balanced_deterministic(P):
    p, t = synth.icosphere(12)
    part = partition_rcb(p, P)
    sizes = np.bincount(part, minlength=P)
    assert sizes.sum() == len(p) and sizes.min() >= len(p) // P and sizes.max() <= -(-len(p) // P)
    assert np.array_equal(part, partition_rcb(p, P))


@pytest.mark.parametrize("P,random", [(2, False), (4, False), (8, False), (3, True)])
def test_plan_matches_definition(P, random):
    p, t = synth.icosphere(10)
    part = (np.random.default_rng(1).integers(0, P, len(p)).astype(np.int32) if random
            else partition_rcb(p, P))
    info = plan_info(t, len(p), part)
    own, ghost, nbr, ntri = restated_plan(t, len(p), part)
    assert np.array_equal(info["n_own"], own)
    assert np.array_equal(info["n_ghost"], ghost)
    assert np.array_equal(info["n_nbr"], nbr)
    assert np.array_equal(info["n_tri"], ntri)
    # every ghost row is sent by exactly one owner
    assert info["n_send"].sum() == info["n_ghost"].sum()


def test_plan_rejects_bad_partition():
    p, t = synth.icosphere(4)
    part = np.zeros(len(p), np.int32)
    part[3] = -1
    with pytest.raises(MofError):
        plan_info(t, len(p), part)
    with pytest.raises(MofError):
        partition_rcb(p, len(p) + 1)


# ---- GPU: decomposed solve ----------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("P", [1, 2, 3, 8])
@pytest.mark.parametrize("precision", ["f64", "mixed"])
def test_dd_vs_spsolve_golden(P, precision):
    g = load_golden("G1_ico642")
    T = len(g["I"])
    d = DecomposedMesh(g["coordinates"], g["normals"], g["triangles"], g["areas"], P)
    V, st = d.solve_range(g["I"], g["t_k"], 0, T - 1, float(g["lambda_"]), precision=precision,
                          rtol=1e-10)
    assert st["failed"] == st["recovered"] == 0 and st["max_rel_residual"] <= 1e-10
    assert np.abs(V - g["V_k"]).max() <= VTOL
    d.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["G2_cap641", "G3_ico642_f32", "G5_dt512"])
def test_dd_golden_cases(case):
    g = load_golden(case)
    T = len(g["I"])
    d = DecomposedMesh(g["coordinates"], g["normals"], g["triangles"], g["areas"], 4)
    V, st = d.solve_range(g["I"], g["t_k"], 0, T - 1, float(g["lambda_"]), precision="mixed",
                          rtol=1e-10)
    scale = max(1.0, np.abs(g["V_k"]).max())
    assert st["failed"] == st["recovered"] == 0
    assert np.abs(V - g["V_k"]).max() <= VTOL * scale
    d.close()


@pytest.mark.gpu
@pytest.mark.parametrize("P,random", [(2, False), (8, False), (5, True)])
def test_dd_matches_single_domain(P, random):
    p, t, n, a, I = wave_case()
    tk = np.arange(len(I), dtype=np.float64)
    part = (np.random.default_rng(7).integers(0, P, len(p)).astype(np.int32) if random else None)
    ref = DeviceMesh(p, n, t, a)
    V1, s1 = ref.solve_range(I, tk, 0, len(I) - 1, 0.01, precision="f64")
    d = DecomposedMesh(p, n, t, a, P, part=part)
    V2, s2 = d.solve_range(I, tk, 0, len(I) - 1, 0.01, precision="f64")
    assert s2["failed"] == s2["recovered"] == 0 and s2["max_rel_residual"] <= 1e-8
    # the same block-Jacobi CG up to the summation order of the dot products
    assert abs(s2["iterations"] - s1["iterations"]) <= 2 * (len(I) - 1)
    assert np.abs(V2 - V1).max() <= 1e-7 * np.abs(V1).max()
    # deterministic for a fixed partition, and across batch sizes
    V3, _ = d.solve_range(I, tk, 0, len(I) - 1, 0.01, precision="f64", batch=2)
    assert np.array_equal(V2, V3)
    if P == 2:  # spsolve on one timestep
        a2, gw, e, iw = oracle.geometry(p, n, t, a)
        Vo = oracle.worker(1, a2, gw, e, iw, t, list(tk), a, 0.01, I[1], I[2])
        assert np.abs(V2[1] - Vo).max() <= VTOL
    ref.close()
    d.close()


@pytest.mark.gpu
@pytest.mark.parametrize("P,precision", [(3, "mixed"), (8, "f64")])
def test_dd_staged_transport(P, precision):
    """The RCCL transport's pack -> exchange -> unpack kernels and V gather
    (device copies in place of ncclSend/Recv/AllGather) give the same bits
    as the in-process gather."""
    p, t, n, a, I = wave_case(n=16, T=5)
    tk = np.arange(len(I), dtype=np.float64)
    part = np.random.default_rng(3).integers(0, P, len(p)).astype(np.int32)
    d1 = DecomposedMesh(p, n, t, a, P, part=part)
    d2 = DecomposedMesh(p, n, t, a, P, part=part, staged=True)
    V1, s1 = d1.solve_range(I, tk, 0, 4, 0.01, precision=precision, batch=3)
    V2, s2 = d2.solve_range(I, tk, 0, 4, 0.01, precision=precision, batch=3)
    assert s2["failed"] == s2["recovered"] == 0 and s1["iterations"] == s2["iterations"]
    assert np.array_equal(V1, V2)
    d1.close()
    d2.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case,P", [("G1_ico642", 2), ("G1_ico642", 3), ("G2_cap641", 4),
                                    ("G5_dt512", 3)])
def test_dd_amg_vs_spsolve_golden(case, P):
    """Subdomain multigrid (a V-cycle per part on its owned rows, block Jacobi
    across the parts) reaches the same V as spsolve."""
    g = load_golden(case)
    T = len(g["I"])
    d = DecomposedMesh(g["coordinates"], g["normals"], g["triangles"], g["areas"], P)
    V, st = d.solve_range(g["I"], g["t_k"], 0, T - 1, float(g["lambda_"]), precision="mixed",
                          precond="amg", rtol=1e-10)
    scale = max(1.0, np.abs(g["V_k"]).max())
    assert st["failed"] == st["recovered"] == 0 and st["max_rel_residual"] <= 1e-10
    assert np.abs(V - g["V_k"]).max() <= VTOL * scale
    d.close()


@pytest.mark.gpu
def test_dd_amg_fewer_iterations_deterministic():
    p, t, n, a, I = wave_case(n=24, T=7)
    tk = np.arange(len(I), dtype=np.float64)
    d = DecomposedMesh(p, n, t, a, 4)
    Vj, sj = d.solve_range(I, tk, 0, 6, 0.01, precision="mixed")
    V1, s1 = d.solve_range(I, tk, 0, 6, 0.01, precision="mixed", precond="amg", batch=6)
    V2, _ = d.solve_range(I, tk, 0, 6, 0.01, precision="mixed", precond="amg", batch=4)
    d.close()
    assert s1["failed"] == s1["recovered"] == 0 and s1["max_rel_residual"] <= 1e-8
    assert s1["iterations"] < sj["iterations"]
    assert np.array_equal(V1, V2)  # any batch size, the same bits
    # two solves to the same 1e-8 residual bar (measured 6e-7 apart at |V| ~ 1)
    assert np.abs(V1 - Vj).max() <= VTOL
    # the RCCL transport's pack / exchange / unpack path gives the same bits
    ds = DecomposedMesh(p, n, t, a, 4, staged=True)
    V3, _ = ds.solve_range(I, tk, 0, 6, 0.01, precision="mixed", precond="amg", batch=6)
    ds.close()
    assert np.array_equal(V1, V3)


@pytest.mark.gpu
def test_dd_amg_irregular_mesh_vs_smoothed_single_domain():
    """A random hull (valence 3-14) over 3 RCB parts: the parts keep the
    tentative prolongator (amg_build smooths only a whole mesh, nown < 0:
    MOF_VERBOSE shows no "smoothed P" part level), the single domain
    smooths levels 0 and 1 (slab Galerkin, chunked coarse product, sorted
    restriction): two different preconditioners, V within 1e-6 of each
    other and of the oracle; the decomposed solve has the same bits for
    another batch size."""
    p, t = synth.random_sphere(20000, 10.0, seed=11)
    n, a = synth.vertex_normals(p, t), synth.triangle_areas(p, t)
    T = 9
    I = synth.travelling_wave(p, T)
    tk = np.arange(float(T))
    d = DecomposedMesh(p, n, t, a, 3)
    V1, s1 = d.solve_range(I, tk, 0, T - 1, 0.01, precision="mixed", precond="amg", batch=8)
    V2, _ = d.solve_range(I, tk, 0, T - 1, 0.01, precision="mixed", precond="amg", batch=5)
    d.close()
    assert s1["failed"] == s1["recovered"] == 0 and s1["max_rel_residual"] <= 1e-8
    assert np.array_equal(V1, V2)
    ref = DeviceMesh(p, n, t, a)
    V0, s0 = ref.solve_range(I, tk, 0, T - 1, 0.01, precision="mixed", precond="amg")
    ref.close()
    scale = max(1.0, np.abs(V0).max())
    assert np.abs(V1 - V0).max() <= VTOL * scale
    a2, gw, e, iw = oracle.geometry(p, n, t, a)
    Vo = oracle.worker(4, a2, gw, e, iw, t, list(tk), a, 0.01, I[4], I[5])
    assert np.abs(V1[4] - Vo).max() <= VTOL * scale


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.parametrize("precond", ["jacobi", "amg"])
def test_dd_full_size_c3(precond):
    """C3 (163,842 vertices) over 8 RCB parts: every system meets the fp64
    residual bar, V agrees with the single-domain solve to the solver
    tolerance, and with block Jacobi the iteration counts are the
    single-domain ones (the preconditioner is pointwise)."""
    p, t, n, a = synth.mesh_for_config("C3")
    I = synth.travelling_wave(p, 5)
    tk = np.arange(len(I), dtype=np.float64)
    d = DecomposedMesh(p, n, t, a, 8)
    V2, s2 = d.solve_range(I, tk, 0, 4, 0.01, precision="mixed", precond=precond)
    d.close()
    ref = DeviceMesh(p, n, t, a)
    V1, s1 = ref.solve_range(I, tk, 0, 4, 0.01, precision="mixed", precond=precond)
    ref.close()
    assert s2["failed"] == s2["recovered"] == 0 and s2["max_rel_residual"] <= 1e-8
    if precond == "jacobi":
        assert abs(s2["iterations"] - s1["iterations"]) <= 8
    assert np.abs(V2 - V1).max() <= 1e-6


@pytest.mark.gpu
def test_dd_nonconvergence_nan():
    """A solve capped far below its need: NaN-filled and reported with
    MOF_NO_RECOVERY; by default the decomposed path re-solves the failed
    systems (fp64 block Jacobi, the full budget) as mof_solve_range does."""
    p, t, n, a, I = wave_case(n=12, T=3)
    tk = np.arange(len(I), dtype=np.float64)
    d = DecomposedMesh(p, n, t, a, 3)
    V, st = d.solve_range(I, tk, 0, 2, 0.01, precision="f64", max_iter=2, max_outer=1, recovery=False)
    assert st["failed"] == 2 and np.isnan(V).all()
    V, st = d.solve_range(I, tk, 0, 2, 0.01, precision="f64", max_iter=2, max_outer=1)
    assert st["failed"] == 0 and st["recovered"] == 2 and st["recovered_f64"] == 2, st
    d.close()
    m = DeviceMesh(p, n, t, a)
    Vs, _ = m.solve_range(I, tk, 0, 2, 0.01, precision="f64")
    assert np.abs(V - Vs).max() < 1e-6


@pytest.mark.gpu
def test_dd_device_io():
    import torch
    p, t, n, a, I = wave_case(n=16, T=6)
    tk = np.arange(len(I), dtype=np.float64)
    d = DecomposedMesh(p, n, t, a, 4)
    Vh, _ = d.solve_range(I, tk, 0, 5, 0.01, precision="mixed")
    Id = torch.from_numpy(I).to("cuda:0")
    Vd = torch.empty((5, 2 * len(p)), dtype=torch.float64, device="cuda:0")
    torch.cuda.synchronize()
    st = d.solve_range_device(Id.data_ptr(), Id.data_ptr(), len(I), tk, 0, 5, 0.01, Vd.data_ptr(),
                              precision="mixed")
    assert st["failed"] == st["recovered"] == 0
    assert np.array_equal(Vd.cpu().numpy(), Vh)
    d.close()


@pytest.mark.gpu
def test_dd_rccl_single_rank():
    """The RCCL transport end to end with one rank (RCCL needs one GPU per
    rank; the box has one): communicator, all-gathers, V gather."""
    import os
    import torch.distributed as dist
    p, t, n, a, I = wave_case(n=12, T=4)
    tk = np.arange(len(I), dtype=np.float64)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        d = DecomposedMesh(p, n, t, a, 1, group=dist.group.WORLD)
        assert d.info()["rank"] == 0
        V, st = d.solve_range(I, tk, 0, 3, 0.01, precision="f64")
        ref = DecomposedMesh(p, n, t, a, 1)
        V1, _ = ref.solve_range(I, tk, 0, 3, 0.01, precision="f64")
        assert st["failed"] == st["recovered"] == 0 and np.array_equal(V, V1)
        d.close()
        ref.close()
    finally:
        dist.destroy_process_group()
