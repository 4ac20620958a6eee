"""The S3 CSV files through libmofhip's threaded host writer/reader
(C ABI mof_csv_write / mof_csv_shape / mof_csv_read).

``write_csv(path, data)`` writes exactly the bytes of
``pd.DataFrame(data.reshape(rows, -1)).to_csv(path)`` (reference
``reshape_and_save_data``, compute_optical_flow.py:314-320);
``read_csv(path)`` returns ``pd.read_csv(path, header='infer',
index_col=0).values`` as float64 (reference ``load_potentials``,
compute_optical_flow.py:203-207). Host only: no GPU is touched.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib as L


def _path(p) -> bytes:
    return os.fsencode(os.fspath(p))


def write_csv(path, data, threads: int = 0) -> None:
    arr = np.asarray(data)
    rows = arr.shape[0] if arr.ndim else 1
    a = np.ascontiguousarray(arr.reshape(rows, -1), dtype=np.float64)
    L.check(L.lib().mof_csv_write(_path(path), L.ptr(a), a.shape[0], a.shape[1], int(threads)))


def read_csv(path, threads: int = 0, round_trip: bool = False) -> np.ndarray:
    """Values of a pandas CSV (header line and index column dropped), parsed
    exactly as pandas' default float parser does, or correctly rounded
    (pandas float_precision='round_trip') with ``round_trip=True``."""
    rows, cols = ctypes.c_int64(0), ctypes.c_int64(0)
    L.check(L.lib().mof_csv_shape(_path(path), ctypes.byref(rows), ctypes.byref(cols)))
    out = np.empty((rows.value, cols.value), dtype=np.float64)
    flags = L.MOF_CSV_ROUND_TRIP if round_trip else 0
    L.check(L.lib().mof_csv_read(_path(path), L.ptr(out), rows.value, cols.value, flags,
                                 int(threads)))
    return out
