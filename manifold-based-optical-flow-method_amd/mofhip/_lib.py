"""ctypes binding of libmofhip.so (the C ABI in include/mof.h).

The shared library is built in-tree by ``csrc/Makefile`` (or
``mofhip.build_native()``) for gfx950. There is no CPU fallback: if the
library is missing or no HIP device is visible, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT_DIR = os.path.dirname(PKG_DIR)
CSRC_DIR = os.path.join(ROOT_DIR, "csrc")
# MOFHIP_LIB: another in-tree build of the same library (A/B measurements)
LIB_PATH = os.environ.get("MOFHIP_LIB") or os.path.join(PKG_DIR, "libmofhip.so")

# include/mof.h MOF_ABI_VERSION this binding's structs follow
MOF_ABI_VERSION = 4

MOF_OK = 0
MOF_E_ARG = -1
MOF_E_HIP = -2
MOF_E_NOCONV = -3
MOF_E_STATE = -4

MOF_GEOM_F32_POINTS = 1
MOF_NO_REORDER = 2
MOF_PREC_F64 = 0
MOF_PREC_MIXED = 1
MOF_IO_DEVICE = 1
MOF_NO_BLOCK_JACOBI = 2
MOF_TIME_SPMV = 4
MOF_PRECOND_AMG = 8
MOF_NO_RECOVERY = 16
MOF_SOLVE_FUSED = 128
MOF_SOLVE_EAGER = 256
MOF_CSV_ROUND_TRIP = 1
MOF_COORDS_F32 = 32
MOF_DD_STAGED = 64
MOF_CSR_A2 = 0
MOF_CSR_A_LAST = 1

# every symbol include/mof.h declares
EXPORTS = (
    "mof_version", "mof_abi_version", "mof_last_error", "mof_device_count", "mof_mesh_create", "mof_mesh_clone",
    "mof_mesh_destroy", "mof_mesh_get_info", "mof_geometry_export", "mof_csr_export",
    "mof_assemble", "mof_solve_range", "mof_bench_spmv", "mof_velocity_vectors",
    "mof_csv_write", "mof_csv_shape", "mof_csv_read", "mof_ply_info", "mof_ply_read",
    "mof_point_normals", "mof_cell_areas", "mof_singularities", "mof_amg_probe",
    "mof_partition_rcb", "mof_dd_plan_info", "mof_dd_create", "mof_dd_unique_id",
    "mof_dd_create_rank", "mof_dd_destroy", "mof_dd_get_info", "mof_dd_solve_range",
    "mof_dd_test_fail_recovery_alloc", "mof_mesh_prepare", "mof_mesh_sync",
    "mof_singularities_compact", "mof_xcd_map_check", "mof_xcd_batch_cap", "mof_dd_create_rank_host",
)


class MofError(RuntimeError):
    """A libmofhip call returned a non-zero status."""

    def __init__(self, code, msg):
        super().__init__("libmofhip error %d: %s" % (code, msg))
        self.code = code


class NotConverged(MofError):
    pass


class MofOpts(ctypes.Structure):
    _fields_ = [
        ("struct_size", ctypes.c_uint32), ("precision", ctypes.c_uint32),
        ("flags", ctypes.c_uint32), ("batch", ctypes.c_int32), ("max_iter", ctypes.c_int32),
        ("max_outer", ctypes.c_int32), ("rtol", ctypes.c_double),
        ("inner_rtol", ctypes.c_double), ("stream", ctypes.c_void_p),
        ("etol", ctypes.c_double),
    ]


class MofStats(ctypes.Structure):
    _fields_ = [
        ("systems", ctypes.c_int64), ("iterations", ctypes.c_int64),
        ("max_iterations", ctypes.c_int32), ("failed", ctypes.c_int32),
        ("outer_steps", ctypes.c_int32), ("batches", ctypes.c_int32),
        ("max_rel_residual", ctypes.c_double), ("ms_assembly", ctypes.c_double),
        ("ms_solve", ctypes.c_double), ("spmv_launches", ctypes.c_int64),
        ("ms_spmv", ctypes.c_double), ("spmv_bytes", ctypes.c_double),
        ("spmv_systems", ctypes.c_int64), ("spmv_full_launches", ctypes.c_int64),
        ("ms_spmv_full", ctypes.c_double), ("recovered", ctypes.c_int32),
        ("recovered_f64", ctypes.c_int32), ("fused_launches", ctypes.c_int64),
        ("ms_fused", ctypes.c_double), ("max_err_est", ctypes.c_double),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class MofMeshInfo(ctypes.Structure):
    _fields_ = [
        ("N", ctypes.c_int32), ("M", ctypes.c_int32), ("device", ctypes.c_int32),
        ("nblocks", ctypes.c_int32), ("nnz_struct", ctypes.c_int64),
        ("sell_blocks", ctypes.c_int64), ("ms_geometry", ctypes.c_double),
        ("ms_pattern", ctypes.c_double), ("blocks_read", ctypes.c_int64),
        ("max_batch", ctypes.c_int32), ("pad_", ctypes.c_int32),
    ]


class MofDdInfo(ctypes.Structure):
    _fields_ = [
        ("nparts", ctypes.c_int32), ("local_parts", ctypes.c_int32), ("rank", ctypes.c_int32),
        ("max_neighbours", ctypes.c_int32), ("max_owned", ctypes.c_int32),
        ("pad_", ctypes.c_int32), ("ghost_rows", ctypes.c_int64), ("send_rows", ctypes.c_int64),
        ("ms_setup", ctypes.c_double),
    ]


MOF_DD_ID_BYTES = 128

# mof_dd_transport callbacks
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64)
EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32),
                               ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_int64),
                               ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_int64))


class MofDdTransport(ctypes.Structure):
    _fields_ = [("ctx", ctypes.c_void_p), ("allgather", ALLGATHER_FN), ("exchange", EXCHANGE_FN)]

_lib = None
_lock = threading.Lock()


def build_native(force: bool = False, jobs: int = 4) -> str:
    """Compile csrc/ into mofhip/libmofhip.so with hipcc (gfx950)."""
    cmd = ["make", "-C", CSRC_DIR, "-j%d" % jobs]
    if force:
        subprocess.check_call(["make", "-C", CSRC_DIR, "clean"])
    subprocess.check_call(cmd)
    return LIB_PATH


def lib():
    """The loaded library (raises if it is not built)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                "libmofhip.so is not built (%s); run `make -C %s` or "
                "mofhip.build_native()" % (LIB_PATH, CSRC_DIR))
        L = ctypes.CDLL(LIB_PATH)
        P, i32, u32, i64, f64 = (ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint32,
                                 ctypes.c_int64, ctypes.c_double)
        sig = {
            "mof_version": ([], ctypes.c_char_p),
            "mof_abi_version": ([], ctypes.c_int),
            "mof_last_error": ([], ctypes.c_char_p),
            "mof_device_count": ([P], ctypes.c_int),
            "mof_mesh_create": ([P, P, P, P, i32, i32, i32, u32, P], ctypes.c_int),
            "mof_mesh_clone": ([P, i32, P], ctypes.c_int),
            "mof_mesh_destroy": ([P], ctypes.c_int),
            "mof_mesh_get_info": ([P, P], ctypes.c_int),
            "mof_geometry_export": ([P, P, P, P], ctypes.c_int),
            "mof_csr_export": ([P, i32, i32, P, P, P, P], ctypes.c_int),
            "mof_assemble": ([P, P, P, f64, f64, P], ctypes.c_int),
            "mof_solve_range": ([P, P, P, P, i32, i32, i32, f64, P, P, P], ctypes.c_int),
            "mof_bench_spmv": ([P, u32, i32, i32, P, P], ctypes.c_int),
            "mof_velocity_vectors": ([i32, P, P, i32, i32, P, P, u32, P], ctypes.c_int),
            "mof_csv_write": ([ctypes.c_char_p, P, i64, i64, i32], ctypes.c_int),
            "mof_csv_shape": ([ctypes.c_char_p, P, P], ctypes.c_int),
            "mof_csv_read": ([ctypes.c_char_p, P, i64, i64, u32, i32], ctypes.c_int),
            "mof_ply_info": ([ctypes.c_char_p, P, P, P], ctypes.c_int),
            "mof_ply_read": ([ctypes.c_char_p, P, P, P], ctypes.c_int),
            "mof_point_normals": ([P, P, i64, i64, P], ctypes.c_int),
            "mof_cell_areas": ([P, P, i64, i64, P], ctypes.c_int),
            "mof_singularities": ([i32, P, P, i32, i32, P, i32, f64, u32, P, P, P, P, P],
                                  ctypes.c_int),
            "mof_amg_probe": ([P, P, i32, i32, P, P, P, P], ctypes.c_int),
            "mof_xcd_map_check": ([i32, i32, i32], ctypes.c_int),
            "mof_xcd_batch_cap": ([i64, i32, P], ctypes.c_int),
            "mof_singularities_compact": ([i32, P, P, i32, i32, P, i32, f64, u32, P, i64, P, P, P, P, P,
                                           P, P], ctypes.c_int),
            "mof_partition_rcb": ([P, i32, i32, P], ctypes.c_int),
            "mof_dd_plan_info": ([P, i32, i32, i32, P, P, P, P, P, P], ctypes.c_int),
            "mof_dd_create": ([P, P, P, P, i32, i32, i32, P, i32, u32, P], ctypes.c_int),
            "mof_dd_unique_id": ([P], ctypes.c_int),
            "mof_dd_create_rank": ([P, P, P, P, i32, i32, i32, P, i32, P, i32, u32, P],
                                   ctypes.c_int),
            "mof_dd_create_rank_host": ([P, P, P, P, i32, i32, i32, P, i32, P, i32, u32, P],
                                        ctypes.c_int),
            "mof_dd_destroy": ([P], ctypes.c_int),
            "mof_dd_get_info": ([P, P], ctypes.c_int),
            "mof_mesh_prepare": ([P, P], ctypes.c_int),
            "mof_mesh_sync": ([P], ctypes.c_int),
            "mof_dd_test_fail_recovery_alloc": ([P, i32], ctypes.c_int),
            "mof_dd_solve_range": ([P, P, P, P, i32, i32, i32, f64, P, P, P], ctypes.c_int),
        }
        for name, (args, res) in sig.items():
            if os.environ.get("MOFHIP_LIB") and not hasattr(L, name):
                continue  # an older build under A/B measurement
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        # the library writes whole mof_stats / mof_mesh_info structs: a
        # library of another ABI would overrun (or under-fill) these
        if not os.environ.get("MOFHIP_LIB"):
            abi = L.mof_abi_version() if hasattr(L, "mof_abi_version") else 1
            if abi != MOF_ABI_VERSION:
                raise ImportError("libmofhip.so has ABI %d, this binding needs %d (rebuild: make -C %s)"
                                  % (abi, MOF_ABI_VERSION, CSRC_DIR))
        _lib = L
    return _lib


def check(rc: int) -> int:
    if rc == MOF_OK:
        return rc
    msg = lib().mof_last_error().decode(errors="replace")
    if rc == MOF_E_NOCONV:
        raise NotConverged(rc, msg)
    raise MofError(rc, msg)


def ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def device_count() -> int:
    n = ctypes.c_int32(0)
    check(lib().mof_device_count(ctypes.byref(n)))
    return int(n.value)


def version() -> str:
    return lib().mof_version().decode()
