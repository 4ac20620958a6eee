"""The multigrid-preconditioned inner solve (MOF_PRECOND_AMG) against the
reference's spsolve.

The preconditioner changes the iteration path only: the answer is held to the
same bars as the block-Jacobi solve (max |V - V_spsolve| < 1e-6, relative true
residual <= rtol in fp64), and it keeps the determinism guarantees (identical
bits for any batch size or shard split).
"""
import numpy as np
import pytest

import oracle
from conftest import load_golden
from mofhip import DeviceMesh, synth, velocity_field_sharded

pytestmark = pytest.mark.gpu

VTOL = 1e-6


def mesh_of(g):
    return DeviceMesh(g["coordinates"], g["normals"], g["triangles"], g["areas"])


@pytest.mark.parametrize("case", ["G1_ico642", "G2_cap641", "G3_ico642_f32", "G5_dt512"])
def test_amg_vs_spsolve_golden(case):
    g = load_golden(case)
    m = mesh_of(g)
    T = len(g["I"])
    V, st = m.solve_range(g["I"], g["t_k"], 0, T - 1, float(g["lambda_"]), precision="mixed",
                          precond="amg", rtol=1e-10)
    ref = g["V_k"]
    assert st["failed"] == st["recovered"] == 0
    assert st["max_rel_residual"] <= 1e-10
    assert np.abs(V - ref).max() <= VTOL * max(1.0, np.abs(ref).max())


def test_amg_fewer_iterations_and_deterministic():
    g = load_golden("G1_ico642")
    m = mesh_of(g)
    I, tk, lam = g["I"], g["t_k"], float(g["lambda_"])
    Vj, sj = m.solve_range(I, tk, 0, 15, lam, precision="mixed")
    V1, s1 = m.solve_range(I, tk, 0, 15, lam, precision="mixed", precond="amg", batch=1)
    V8, _ = m.solve_range(I, tk, 0, 15, lam, precision="mixed", precond="amg", batch=8)
    V15, _ = m.solve_range(I, tk, 0, 15, lam, precision="mixed", precond="amg", batch=15)
    assert np.array_equal(V1, V8) and np.array_equal(V1, V15)
    Vs, _ = velocity_field_sharded(m, I, tk, 0, 15, lam, devices=[0, 0], precision="mixed",
                                   precond="amg")
    assert np.array_equal(V1, Vs)
    assert s1["iterations"] < sj["iterations"]
    assert np.abs(V1 - Vj).max() < VTOL


@pytest.mark.parametrize("precision,precond", [("mixed", "amg"), ("mixed", "jacobi"), ("f64", "jacobi")])
def test_partial_system_groups_bit_identical(precision, precond):
    """Batches larger than the XCD system groups (8 and 32 systems) with a
    partial last group: same bits as one system per launch."""
    g = load_golden("G1_ico642")
    m = mesh_of(g)
    T = 42
    I = synth.travelling_wave(g["coordinates"], T)
    tk = np.arange(T, dtype=np.float64)
    V1, s1 = m.solve_range(I, tk, 0, T - 1, 0.01, precision=precision, precond=precond, batch=1)
    V41, s41 = m.solve_range(I, tk, 0, T - 1, 0.01, precision=precision, precond=precond, batch=41)
    assert s1["failed"] == s1["recovered"] == 0 and s41["failed"] == s41["recovered"] == 0
    assert np.array_equal(V1, V41)


def test_amg_tiny_mesh_falls_back():
    """A mesh that does not coarsen (12 vertices) keeps block Jacobi."""
    p, t = synth.icosphere(1, 10.0)
    n, a = synth.vertex_normals(p, t), synth.triangle_areas(p, t)
    I = synth.travelling_wave(p, 3)
    m = DeviceMesh(p, n, t, a)
    V, st = m.solve_range(I, np.arange(3.0), 0, 2, 0.01, precision="mixed", precond="amg")
    a2, gw, e, iw = oracle.geometry(p, n, t, a)
    for k in range(2):
        Vo = oracle.worker(k, a2, gw, e, iw, t, [0, 1, 2], a, 0.01, I[k], I[k + 1])
        assert np.abs(V[k] - Vo).max() < VTOL


def test_amg_needs_mixed_precision():
    g = load_golden("G1_ico642")
    m = mesh_of(g)
    with pytest.raises(Exception):
        m.solve_range(g["I"], g["t_k"], 0, 2, 0.01, precision="f64", precond="amg")


@pytest.mark.parametrize("kind", ["random_hull", "permuted_ico", "cap"])
def test_amg_irregular_meshes(kind):
    if kind == "random_hull":
        p, t = synth.random_sphere(3000, 10.0, seed=3)
    elif kind == "permuted_ico":
        p, t, _ = synth.permute_vertices(*synth.icosphere(16, 10.0, jitter=0.005), seed=2)
    else:
        p, t = synth.spherical_cap(40, 10.0, 0.7)
    n, a = synth.vertex_normals(p, t), synth.triangle_areas(p, t)
    I = synth.travelling_wave(p, 4)
    m = DeviceMesh(p, n, t, a)
    a2, gw, e, iw = oracle.geometry(p, n, t, a)
    V, st = m.solve_range(I, np.arange(4.0), 0, 3, 0.01, precision="mixed", precond="amg")
    assert st["failed"] == st["recovered"] == 0 and st["max_rel_residual"] <= 1e-8
    for k in range(3):
        Vo = oracle.worker(k, a2, gw, e, iw, t, list(range(4)), a, 0.01, I[k], I[k + 1])
        assert np.abs(V[k] - Vo).max() < VTOL * max(1.0, np.abs(Vo).max()), k


@pytest.mark.slow
def test_amg_32k_vs_spsolve():
    p, t, n, a = synth.mesh_for_config("C2")
    I = synth.travelling_wave(p, 3)
    m = DeviceMesh(p, n, t, a)
    a2, gw, e, iw = oracle.geometry(p, n, t, a)
    Ao, fo = oracle.step_system(a2, gw, e, iw, t, a, 0.01, I[0], I[1], 1.0)
    from scipy.sparse.linalg import spsolve
    Vo = spsolve(Ao.tocsc(), fo)
    V, st = m.solve_range(I, np.arange(3.0), 0, 1, 0.01, precision="mixed", precond="amg")
    assert np.abs(V[0] - Vo).max() < VTOL
    assert st["max_rel_residual"] <= 1e-8


@pytest.mark.slow
def test_amg_160k_agrees_with_jacobi():
    p, t, n, a = synth.mesh_for_config("C3")
    I = synth.travelling_wave(p, 5)
    m = DeviceMesh(p, n, t, a)
    tk = np.arange(5.0)
    Vj, sj = m.solve_range(I, tk, 0, 4, 0.01, precision="mixed", batch=4)
    Va, sa = m.solve_range(I, tk, 0, 4, 0.01, precision="mixed", precond="amg", batch=4)
    Va2, _ = m.solve_range(I, tk, 0, 4, 0.01, precision="mixed", precond="amg", batch=2)
    assert sa["failed"] == sa["recovered"] == 0 and sa["max_rel_residual"] <= 1e-8
    assert np.abs(Va - Vj).max() < VTOL
    assert np.array_equal(Va, Va2)
    assert sa["iterations"] < sj["iterations"]


def test_amg_singular_system_is_nan():
    """An unreferenced vertex makes A singular (zero diagonal block): the
    multigrid path must report the system failed with a NaN V, not hang or
    return garbage (spsolve's MatrixRankWarning behaviour)."""
    g = load_golden("G1_ico642")
    coords = np.vstack([g["coordinates"], [[0.0, 0.0, 20.0]]])
    normals = np.vstack([g["normals"], [[0.0, 0.0, 1.0]]])
    m = DeviceMesh(coords, normals, g["triangles"], g["areas"])
    I = np.hstack([g["I"][:3], np.zeros((3, 1))])
    V, st = m.solve_range(I, np.arange(3.0), 0, 2, 0.01, precision="mixed", precond="amg")
    assert st["failed"] == 2
    assert np.isnan(V).all()


def test_amg_unordered_mesh_and_repeat():
    """MOF_NO_REORDER (caller order inside: other aggregates, other iteration
    path) agrees with the default order to the solve tolerance; a second solve
    on the same handle (hierarchy reused) is bit-identical."""
    g = load_golden("G1_ico642")
    I, tk, lam = g["I"], g["t_k"], float(g["lambda_"])
    m0 = DeviceMesh(g["coordinates"], g["normals"], g["triangles"], g["areas"], reorder=False)
    m1 = mesh_of(g)
    V0, s0 = m0.solve_range(I, tk, 0, 15, lam, precision="mixed", precond="amg")
    V1, _ = m1.solve_range(I, tk, 0, 15, lam, precision="mixed", precond="amg")
    V1b, _ = m1.solve_range(I, tk, 0, 15, lam, precision="mixed", precond="amg")
    assert s0["failed"] == s0["recovered"] == 0
    assert np.array_equal(V1, V1b)
    assert np.abs(V0 - V1).max() < VTOL


# ---- smoothed aggregation (level 0, per mesh: irregular meshes) -------------

def _hull(nv=3000, seed=3):
    p, t = synth.random_sphere(nv, 10.0, seed=seed)
    return p, t, synth.vertex_normals(p, t), synth.triangle_areas(p, t)


@pytest.mark.parametrize("smooth", ["0", "1"])
def test_smoothed_aggregation_golden(smooth, monkeypatch):
    """Forced either way on the regular golden mesh: V meets the 1e-6 bar
    against the reference's spsolve (MOF_AMG_SMOOTH is read when the
    hierarchy is built, i.e. at the first multigrid solve of a handle)."""
    monkeypatch.setenv("MOF_AMG_SMOOTH", smooth)
    g = load_golden("G1_ico642")
    m = mesh_of(g)
    V, st = m.solve_range(g["I"], g["t_k"], 0, 15, float(g["lambda_"]), precision="mixed", precond="amg")
    assert st["failed"] == 0 and st["recovered"] == 0
    assert np.abs(V - g["V_k"]).max() < VTOL


def test_smoothed_aggregation_irregular_mesh(monkeypatch):
    """The random hull (valence 3-14) takes the smoothed prolongator by
    default: fewer iterations than the tentative one, both within 1e-6 of
    spsolve, and the same bits for any batch split (the multi-system
    restriction / prolongation / Galerkin kernels put a system in any slot)."""
    p, t, n, a = _hull()
    T = 11
    I = synth.travelling_wave(p, T)
    tk = np.arange(float(T))
    out = {}
    for smooth in ("auto", "0"):
        if smooth == "auto":
            monkeypatch.delenv("MOF_AMG_SMOOTH", raising=False)
        else:
            monkeypatch.setenv("MOF_AMG_SMOOTH", smooth)
        m = DeviceMesh(p, n, t, a)
        V, st = m.solve_range(I, tk, 0, T - 1, 0.01, precision="mixed", precond="amg", batch=10)
        assert st["failed"] == 0 and st["recovered"] == 0, st
        out[smooth] = (V, st["iterations"])
        if smooth == "auto":
            V3, s3 = m.solve_range(I, tk, 0, T - 1, 0.01, precision="mixed", precond="amg", batch=3)
            V7, _ = m.solve_range(I, tk, 0, T - 1, 0.01, precision="mixed", precond="amg", batch=7)
            assert np.array_equal(V, V3) and np.array_equal(V, V7)
        m.close()
    assert out["auto"][1] < 0.8 * out["0"][1], (out["auto"][1], out["0"][1])
    a2, gw, e, iw = oracle.geometry(p, n, t, a)
    for k in (0, 6):
        Vo = oracle.worker(k, a2, gw, e, iw, t, list(tk), a, 0.01, I[k], I[k + 1])
        for smooth in ("auto", "0"):
            assert np.abs(out[smooth][0][k] - Vo).max() < VTOL * max(1.0, np.abs(Vo).max()), (smooth, k)


def test_slab_galerkin_batch_split():
    """A smoothed level 0 (random hull, 20k vertices) takes its level-0 and
    level-1 Galerkin products by system slab (k_a_slab -> k_galerkin_sys,
    64 systems per wave): the same bits for batches that split the slabs
    differently (70 = 64 + 6, 33 + 33 + 4), and V within 1e-6 of the
    oracle's spsolve."""
    p, t, n, a = _hull(20000, seed=5)
    T = 71
    I = synth.travelling_wave(p, T)
    tk = np.arange(float(T))
    m = DeviceMesh(p, n, t, a)
    V, st = m.solve_range(I, tk, 0, T - 1, 0.01, precision="mixed", precond="amg", batch=70)
    V33, _ = m.solve_range(I, tk, 0, T - 1, 0.01, precision="mixed", precond="amg", batch=33)
    m.close()
    assert st["failed"] == 0 and st["recovered"] == 0, st
    assert np.array_equal(V, V33)
    a2, gw, e, iw = oracle.geometry(p, n, t, a)
    for k in (0, 69):
        Vo = oracle.worker(k, a2, gw, e, iw, t, list(tk), a, 0.01, I[k], I[k + 1])
        assert np.abs(V[k] - Vo).max() < VTOL * max(1.0, np.abs(Vo).max()), k


@pytest.mark.parametrize("case", ["G1_ico642", "G2_cap641"])
def test_galerkin_by_entry_batch_split(case):
    """The level-0 Galerkin product by gather entry (k_galerkin0_ent, the
    tentative prolongator's) puts two systems in a thread: the same bits for
    a batch split into partial system pairs (7) as for the whole batch, and
    V within 1e-6 of the reference's spsolve (golden V_k)."""
    g = load_golden(case)
    I, tk, lam = g["I"], g["t_k"], float(g["lambda_"])
    m = mesh_of(g)
    out = []
    for batch in (7, len(I) - 1):
        V, st = m.solve_range(I, tk, 0, len(I) - 1, lam, precision="mixed", precond="amg", batch=batch)
        assert st["failed"] == 0 and st["recovered"] == 0
        out.append((V, st["iterations"]))
    m.close()
    assert out[0][1] == out[1][1]
    assert np.array_equal(out[0][0], out[1][0])
    assert np.abs(out[0][0] - g["V_k"]).max() < VTOL


def test_coarse_galerkin_by_entry_batch_split():
    """Levels >= 1 by gather entry (k_galerkin3_ent) and, for positions past
    kGalBig entries, the chunked k_galerkin3_big, on a mesh with two coarse
    products (10,242 -> ~1.3k -> ~170 nodes): the same bits for ragged system
    groups (batch 7) as for the whole batch, V within 1e-6 of the oracle."""
    p, t = synth.icosphere(32, jitter=0.005)
    n, a = synth.vertex_normals(p, t), synth.triangle_areas(p, t)
    I = synth.travelling_wave(p, 12)
    tk = np.arange(12, dtype=np.float64)
    m = DeviceMesh(p, n, t, a)
    out = []
    for batch in (7, 11):
        V, st = m.solve_range(I, tk, 0, 11, 0.01, precision="mixed", precond="amg", batch=batch)
        assert st["failed"] == 0 and st["recovered"] == 0
        out.append((V, st["iterations"]))
    m.close()
    assert out[0][1] == out[1][1]
    assert np.array_equal(out[0][0], out[1][0])
    a2, gw, e, iw = oracle.geometry(p, n, t, a)
    Vo = oracle.worker(3, a2, gw, e, iw, t, list(tk), a, 0.01, I[3], I[4])
    assert np.abs(out[0][0][3] - Vo).max() < VTOL


def test_open_patch_batch_split_bit_identical():
    """The S1-like open patch (smoothed prolongator, symmetric reads under
    the 2x line bound, fine damping 0.7): the same bits for one system per
    launch and for batches of 17 and 41 -- partial groups of the smoothed-P
    restriction (8 systems per workgroup) and prolongation (16 per thread)."""
    p, t, n, a = synth.mesh_for_config("S1s")
    T = 42
    I = synth.config_wave("S1s", p, T)
    tk = np.arange(float(T))
    m = DeviceMesh(p, n, t, a)
    assert m.info()["blocks_read"] < m.info()["nblocks"]  # symmetric reads chosen
    V1, s1 = m.solve_range(I, tk, 0, T - 1, 0.01, precision="mixed", precond="amg", batch=1)
    V17, _ = m.solve_range(I, tk, 0, T - 1, 0.01, precision="mixed", precond="amg", batch=17)
    V41, s41 = m.solve_range(I, tk, 0, T - 1, 0.01, precision="mixed", precond="amg", batch=41)
    m.close()
    assert s1["failed"] == 0 and s41["failed"] == 0 and s41["recovered"] == 0
    assert np.array_equal(V1, V17) and np.array_equal(V1, V41)
    assert s1["iterations"] == s41["iterations"]


@pytest.mark.parametrize("cfg", ["S1s", "S1m"])
def test_open_patch_boundary_sweeps(monkeypatch, cfg):
    """An open patch takes two extra block-Jacobi sweeps per side on its
    boundary rows and their neighbour ring (k_bsweep, the ring as its own
    SELL matrix; S1s: ring 14 % of the rows, S1m 4 %): fewer PCG iterations
    than without them (MOF_AMG_BSW=0; bench: S1s 28.6 vs 19.8, S1m 43.9 vs
    30.9 per timestep), V within 1e-6 of that solve and of the oracle, no
    failed or recovered system."""
    p, t, n, a = synth.mesh_for_config(cfg)
    T = 13
    I = synth.config_wave(cfg, p, T)
    tk = np.arange(float(T))
    res = {}
    for env in ({}, {"MOF_AMG_BSW": "0"}):
        if env:
            monkeypatch.setenv("MOF_AMG_BSW", env["MOF_AMG_BSW"])
        else:
            monkeypatch.delenv("MOF_AMG_BSW", raising=False)
        m = DeviceMesh(p, n, t, a)
        V, st = m.solve_range(I, tk, 0, T - 1, 0.01, precision="mixed", precond="amg", batch=T - 1)
        m.close()
        assert st["failed"] == 0 and st["recovered"] == 0, (env, st)
        res[tuple(env.items())] = (V, st["iterations"])
    V, its = res[()]
    V0, its0 = res[(("MOF_AMG_BSW", "0"),)]
    assert its < 0.85 * its0, (its, its0)
    scale = max(1.0, np.abs(V0).max())
    assert np.abs(V - V0).max() < VTOL * scale
    a2, gw, e, iw = oracle.geometry(p, n, t, a)
    for k in (0, T - 2):
        Vo = oracle.worker(k, a2, gw, e, iw, t, list(tk), a, 0.01, I[k], I[k + 1])
        assert np.abs(V[k] - Vo).max() < VTOL * max(1.0, np.abs(Vo).max()), k


@pytest.mark.parametrize("kind", ["golden", "hull"])
def test_work_skipping_batch_split(kind):
    """Systems whose |r|^2 after the update already meets the tolerance skip
    that iteration's V-cycle (k_pcg_conv_early), tail chunks launch over the
    running systems only (SysMap), and on the 642-vertex mesh the SpMV and the
    update reduce their own scalars (PcgArgs::selfred). None of it may depend
    on which systems share a launch: the same V bits, iteration counts and
    residuals for batches of 5 and 3, and V within 1e-6 of spsolve."""
    if kind == "golden":
        g = load_golden("G1_ico642")
        p, n, t, a = g["coordinates"], g["normals"], g["triangles"], g["areas"]
        I, tk, lam = g["I"], g["t_k"], float(g["lambda_"])
    else:
        p, t, n, a = _hull(20000, seed=9)
        I = synth.travelling_wave(p, 9)
        tk, lam = np.arange(9.0), 0.01
    T = len(I)
    m = DeviceMesh(p, n, t, a)
    out = []
    for batch in (5, 3):
        V, st = m.solve_range(I, tk, 0, T - 1, lam, precision="mixed", precond="amg", batch=batch)
        assert st["failed"] == 0 and st["recovered"] == 0, st
        out.append((V, st["iterations"], st["max_rel_residual"]))
    m.close()
    assert out[1][1] == out[0][1] and out[1][2] == out[0][2]
    assert np.array_equal(out[1][0], out[0][0])
    if kind == "golden":
        assert np.abs(out[0][0] - g["V_k"]).max() < VTOL
    else:
        a2, gw, e, iw = oracle.geometry(p, n, t, a)
        Vo = oracle.worker(4, a2, gw, e, iw, t, list(tk), a, lam, I[4], I[5])
        assert np.abs(out[0][0][4] - Vo).max() < VTOL * max(1.0, np.abs(Vo).max())
