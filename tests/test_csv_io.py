"""the S3 CSV files through libmofhip's host writer/reader.

The reference writes e and V_k with ``pd.DataFrame(...).to_csv``
(compute_optical_flow.py:314-320) and reads the potentials with
``pd.read_csv(path, sep=',', header='infer', index_col=0).values`` (:203-207);
pandas is the oracle here: the written bytes and the parsed values must be
identical. Host-only entry points (no GPU), so these run on the CPU.
"""
import numpy as np
import pandas as pd
import pytest

from mofhip import csvio
from mofhip._lib import MofError


def special_matrix(rows=40, cols=33, seed=0):
    rng = np.random.default_rng(seed)
    a = rng.standard_normal((rows, cols)) * 10.0 ** rng.integers(-310, 300, (rows, cols))
    a[0, :8] = [0.0, -0.0, np.nan, np.inf, -np.inf, 5e-324, -2.2250738585072014e-308, 1.7976931348623157e308]
    a[1, :9] = [1e16, 9999999999999998.0, 1e-5, 1e-4, 0.0001234, 123456789012345678.0, 1.0, 0.1, -1e-4]
    a[2] = rng.integers(-1000, 1000, cols).astype(float)
    a[3] = np.float32(rng.standard_normal(cols)).astype(float)
    a[4] = rng.standard_normal(cols)
    return a


def pandas_bytes(a, tmp_path):
    p = tmp_path / "pandas.csv"
    pd.DataFrame(a).to_csv(p)
    return p.read_bytes()


@pytest.mark.parametrize("shape", [(40, 33), (1, 1), (7, 6), (3, 1284), (12, 1284)])
def test_write_is_pandas_bytes(tmp_path, shape):
    a = special_matrix(*shape) if min(shape) >= 9 else np.random.default_rng(1).standard_normal(shape)
    out = tmp_path / "mof.csv"
    csvio.write_csv(out, a)
    assert out.read_bytes() == pandas_bytes(a, tmp_path)


def test_write_thread_count_invariant(tmp_path):
    a = special_matrix(97, 50)
    outs = []
    for t in (1, 3, 8):
        p = tmp_path / ("t%d.csv" % t)
        csvio.write_csv(p, a, threads=t)
        outs.append(p.read_bytes())
    assert outs[0] == outs[1] == outs[2]


def test_read_matches_pandas_default_and_round_trip(tmp_path):
    rng = np.random.default_rng(2)
    rows = []
    for i in range(200):
        vals = []
        for j in range(16):
            k = rng.integers(0, 9)
            if k == 0:
                vals.append("%.25f" % rng.standard_normal())
            elif k == 1:
                vals.append("%.20e" % (rng.standard_normal() * 10.0 ** rng.integers(-320, 300)))
            elif k == 2:
                vals.append(str(rng.integers(-10**15, 10**15)) + ".5")
            elif k == 3:
                vals.append("%.3g" % rng.standard_normal())
            elif k == 4:
                vals.append("0.000%d" % rng.integers(0, 10**15))
            elif k == 5:
                vals.append(repr(float(rng.standard_normal() * 1e-310)))
            elif k == 6:
                vals.append("")
            elif k == 7:
                vals.append("%d.%de%d" % (rng.integers(0, 99999), rng.integers(0, 99999), rng.integers(-20, 20)))
            else:
                vals.append(repr(float(rng.standard_normal())))
        rows.append(str(i) + "," + ",".join(vals))
    p = tmp_path / "adv.csv"
    p.write_text("," + ",".join(str(j) for j in range(16)) + "\n" + "\n".join(rows) + "\n")
    ref = pd.read_csv(p, sep=",", header="infer", index_col=0).values
    got = csvio.read_csv(p)
    assert got.shape == ref.shape and got.dtype == np.float64
    # bit-identical, NaN where pandas has NaN
    assert np.array_equal(got.view(np.int64)[~np.isnan(ref)], ref.view(np.int64)[~np.isnan(ref)])
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    rt = pd.read_csv(p, index_col=0, float_precision="round_trip").values
    assert np.array_equal(csvio.read_csv(p, round_trip=True), rt, equal_nan=True)


def test_round_trip_and_drop_in(tmp_path, capsys):
    from utils import compute_optical_flow as cof
    a = special_matrix(30, 12)
    p = tmp_path / "V_k.csv"
    cof.reshape_and_save_data(list(a), p)
    assert "文件保存成功" in capsys.readouterr().out
    assert p.read_bytes() == pandas_bytes(a, tmp_path)
    back = cof.load_potentials(p)
    ref = pd.read_csv(p, sep=",", header="infer", index_col=0).values
    assert np.array_equal(back, ref, equal_nan=True)
    # the shortest-repr text parses back to the same doubles when read
    # correctly rounded (pandas' default parser itself is not exact)
    fin = np.isfinite(a)
    assert np.array_equal(csvio.read_csv(p, round_trip=True)[fin], a[fin])
    # e: (N, 2, 3) -> (N, 6)
    e = np.random.default_rng(3).standard_normal((11, 2, 3))
    q = tmp_path / "e.csv"
    cof.reshape_and_save_data(e, q)
    assert q.read_bytes() == pandas_bytes(e.reshape(11, 6), tmp_path)


def test_na_strings_and_errors(tmp_path):
    p = tmp_path / "na.csv"
    p.write_text(",0,1,2\n0,1.5,NaN,inf\n1,,-inf,NA\n2,3,4,5\r\n")
    ref = pd.read_csv(p, index_col=0).values.astype(float)
    assert np.array_equal(csvio.read_csv(p), ref, equal_nan=True)
    bad = tmp_path / "bad.csv"
    bad.write_text(",0,1\n0,1.0,abc\n")
    with pytest.raises(MofError):
        csvio.read_csv(bad)
    ragged = tmp_path / "ragged.csv"
    ragged.write_text(",0,1\n0,1.0,2.0\n1,3.0\n")
    with pytest.raises(MofError):
        csvio.read_csv(ragged)
    with pytest.raises(MofError):
        csvio.read_csv(tmp_path / "missing.csv")
