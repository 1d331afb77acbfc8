"""MapPoint::ComputeDistinctiveDescriptors over liborbg.

Reference: src/MapPoint.cc:342-420.  The point's descriptor becomes the observation
descriptor with the least median Hamming distance to the others (the first on ties):

    best = ComputeDistinctiveDescriptors(descs)        # descs: (N, 32) u8, mObservations order
    best = distinctive_descriptors_device(ctx, pool_ptr, rows_ptr, off_ptr, npoints, best_ptr)
"""
import ctypes as C

import numpy as np

from . import _lib as L


def ComputeDistinctiveDescriptors(descs, ctx=None):
    """BestIdx over one map point's observation descriptors (-1 if there are none)."""
    from .orbmatcher import _ctx
    d = np.ascontiguousarray(descs, np.uint8).reshape(-1, 32)
    best = C.c_int32()
    ctx = ctx or _ctx()
    L.check(L.lib().orbg_distinctive_descriptor(ctx.handle, L.ptr(d), len(d), C.byref(best)),
            "orbg_distinctive_descriptor")
    return best.value


def distinctive_descriptors_device(ctx, d_pool, d_rows, d_off, npoints, d_best, d_desc=None):
    """Batched, device pointers (include/orbg.h orbg_distinctive_descriptors_batch_device)."""
    L.check(L.lib().orbg_distinctive_descriptors_batch_device(ctx.handle, d_pool, d_rows, d_off,
                                                              int(npoints), d_best, d_desc),
            "orbg_distinctive_descriptors_batch_device")
