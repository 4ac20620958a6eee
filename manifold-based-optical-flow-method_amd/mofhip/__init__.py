"""mofhip -- MI355X-native manifold optical-flow solver.

Per-timestep FEM assembly (smoothness a2 + brightness-constancy a1/f) and a
batched block-Jacobi PCG in hand-written HIP kernels for gfx950, behind the C
ABI of include/mof.h. The drop-in module mirroring the reference's
``utils.compute_optical_flow`` lives in ``utils/compute_optical_flow.py``
next to this package.
"""
from ._lib import (MofError, NotConverged, build_native, device_count, lib,  # noqa: F401
                   version, EXPORTS, LIB_PATH)
from .mesh import DeviceMesh  # noqa: F401
from .decomp import DecomposedMesh, partition_rcb, plan_info  # noqa: F401
from .solve import velocity_field_sharded, shard_ranges  # noqa: F401
