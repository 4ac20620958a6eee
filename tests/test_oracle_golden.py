"""The CPU oracle (oracle/mof_oracle.c + spsolve) against the golden vectors
captured from the reference itself (tests/golden/make_golden.py).

Bar: bit-exact for e, grad_w, integral_wi_wj, a2, A_k, f_k and V_k."""
import numpy as np
import oracle
from conftest import golden_csr


def _geom(g):
    return oracle.geometry(g["coordinates"], g["normals"], g["triangles"], g["areas"])


def test_geometry_bitexact(golden):
    a2, gw, e, iw = _geom(golden)
    assert np.array_equal(e, golden["e"])
    assert np.array_equal(gw, golden["grad_w"])
    assert np.array_equal(iw, golden["integral_wi_wj"])
    ref = golden_csr(golden, "a2")
    assert np.array_equal(a2.indptr, ref.indptr)
    assert np.array_equal(a2.indices, ref.indices)
    assert np.array_equal(a2.data, ref.data)


def test_step_system_bitexact(golden):
    a2, gw, e, iw = _geom(golden)
    tk = golden["t_k"]
    ks = [int(k[1:-5]) for k in golden if k.startswith("A") and k.endswith("_data")]
    for k in ks:
        A, f = oracle.step_system(a2, gw, e, iw, golden["triangles"], golden["areas"],
                                  float(golden["lambda_"]), golden["I"][k], golden["I"][k + 1],
                                  tk[k + 1] - tk[k])
        ref = golden_csr(golden, "A%d" % k)
        assert np.array_equal(A.indptr, ref.indptr) and np.array_equal(A.indices, ref.indices)
        assert np.array_equal(A.data, ref.data)
        assert np.array_equal(f, golden["f%d" % k])


def test_velocity_field_bitexact(golden):
    a2, gw, e, iw = _geom(golden)
    T = len(golden["I"])
    V = oracle.velocity_field(T, a2, gw, e, iw, golden["triangles"], list(golden["t_k"]),
                              golden["areas"], float(golden["lambda_"]), golden["I"], golden["I"])
    assert np.array_equal(np.asarray(V), golden["V_k"])


def test_structural_superset(golden):
    """The reference's numeric pattern is a subset of the mesh's block pattern."""
    N = len(golden["coordinates"])
    vptr, vcol = oracle.structural_blocks(golden["triangles"], N)
    ref = golden_csr(golden, "a2")
    blocks = set(zip(np.repeat(np.arange(N), np.diff(vptr)).tolist(), vcol.tolist()))
    r = np.repeat(np.arange(2 * N), np.diff(ref.indptr))
    for i, j in zip((r % N).tolist(), (ref.indices % N).tolist()):
        assert (i, j) in blocks
