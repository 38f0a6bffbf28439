"""ctypes front-end to the oracle's Monte-Carlo profile (oracle/mc.c). TEST INFRASTRUCTURE ONLY."""
import ctypes as C
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

import oracle_lib


def _lib():
    L = oracle_lib.lib()
    if not getattr(L, "_mc_sigs", False):
        L.o_mc_profile.restype = C.c_int
        L.o_mc_profile.argtypes = [oracle_lib.f32p, C.c_int, C.c_float, C.c_int, C.c_uint64, C.c_uint64, C.c_uint64,
                                   C.c_uint64, C.c_void_p, C.c_void_p, C.POINTER(C.c_double)]
        L._mc_sigs = True
    return L


def mc_profile(layers, mfp_range=16.0, nsegments=1024, nphotons=100, seed=89, nthreads=None):
    """Same outputs as mpss.Context.mc_profile (ring-normalised profiles + totals)."""
    lay = np.ascontiguousarray(layers, np.float32).reshape(-1, 4)
    nthreads = nthreads or min(16, os.cpu_count() or 1)
    chunks = np.linspace(0, nphotons, nthreads + 1).astype(np.uint64)
    ext = C.c_double()
    parts = []

    def run(k):
        r = np.zeros(nsegments, np.float64)
        t = np.zeros(nsegments, np.float64)
        e = C.c_double()
        rc = _lib().o_mc_profile(lay, len(lay), mfp_range, nsegments, nphotons, seed, int(chunks[k]),
                                 int(chunks[k + 1]), r.ctypes.data, t.ctypes.data, C.byref(e))
        assert rc == 0
        return r, t, e.value

    with ThreadPoolExecutor(nthreads) as ex:
        parts = list(ex.map(run, range(nthreads)))
    r = sum(p[0] for p in parts)
    t = sum(p[1] for p in parts)
    extent = parts[0][2]
    i = np.arange(nsegments, dtype=np.float64)
    area = np.pi * ((2 * i + 1) * extent / nsegments) * (extent / nsegments)
    factor = float(nphotons) * area
    return dict(reflectance=r / factor, transmittance=t / factor, total_r=r.sum() / nphotons,
                total_t=t.sum() / nphotons, extent=extent, raw_r=r, raw_t=t)
