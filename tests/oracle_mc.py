"""ctypes front-end to the oracle's Monte-Carlo profile (oracle/mc.c). TEST INFRASTRUCTURE ONLY."""
import ctypes as C
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

import oracle_lib

PBRT_PI = float(np.float32(np.pi))  # pbrt's M_PI is a float literal (core/pbrt.h:193-196)


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
    area = PBRT_PI * ((2 * i + 1) * extent / nsegments) * (extent / nsegments)
    factor = float(nphotons) * area
    return dict(reflectance=r / factor, transmittance=t / factor, total_r=r.sum() / nphotons,
                total_t=t.sum() / nphotons, extent=extent, raw_r=r, raw_t=t)


def mc_reference(layers, mfp_range=16.0, nsegments=1024, lerp=True):
    """MultipoleReferenceTask::Run (renderers/mcprofile.cpp:381-425) restated over the oracle's MPC:
    desiredLength 1024, step (float)(extent * 1.01 / 1024), the unresampled profile read at the
    ring centres (float)((i + .5) * (extent / nSegments)); extent as in Render (:457-463)."""
    lay = np.asarray(layers, np.float32).reshape(-1, 4)  # (mua, musp, ior, thickness)
    mfp = sum(1.0 / float(np.float32(a + b)) for a, b in lay[:, :2])
    extent = float(np.float32(mfp_range)) * (mfp / len(lay))
    specs = [(float(l[2]), float(l[3]), float(l[0]), float(l[1])) for l in lay]  # (ior, thickness, mua, musp)
    d, r, t, tr, tt = oracle_lib.mpc_profile(specs, float(np.float32(extent * 1.01 / 1024)), 1024, lerp, False)
    L = _lib()
    if not getattr(L, "_mpcr_sigs", False):
        L.o_mpc_resample.argtypes = [C.c_int] + [oracle_lib.f32p] * 3 + [C.c_int] + [oracle_lib.f32p] * 3
        L._mpcr_sigs = True
    pts = ((np.arange(nsegments) + 0.5) * (extent / nsegments)).astype(np.float32)
    ro = np.zeros(nsegments, np.float32)
    to = np.zeros(nsegments, np.float32)
    L.o_mpc_resample(len(d), d, r, t, nsegments, pts, ro, to)
    return dict(reflectance=ro.astype(np.float64), transmittance=to.astype(np.float64), total_r=tr, total_t=tt,
                extent=extent)


def mc_skin_tables(mua, musp, eta, thickness, photons, seed=89, nthreads=None):
    """ComputeMonteCarloProfile (core/multipole.cpp:298-368) restated over the oracle's walk: per
    band a 2-layer walk over 4096 rings within 12 mfp, the rings as d^2 = (float)(((i + .5) *
    extent / 4096)^2) with float values, resampled to 65536 entries uniform in d^2.
    Returns (table [NB, 65536], rcp [NB], total_r [NB])."""
    L = _lib()
    if not getattr(L, "_mpcu_sigs", False):
        L.o_mpc_resample_uniform.argtypes = [C.c_int, oracle_lib.f32p, oracle_lib.f32p, C.c_int, oracle_lib.f32p]
        L._mpcu_sigs = True
    nb = mua.shape[1]
    nseg, target = 4096, 65536
    tab = np.zeros((nb, target), np.float32)
    rcp = np.zeros(nb, np.float32)
    tot = np.zeros(nb, np.float64)
    for c in range(nb):
        layers = [(mua[k][c], musp[k][c], eta[k], thickness[k]) for k in range(2)]
        g = mc_profile(layers, mfp_range=12.0, nsegments=nseg, nphotons=photons, seed=seed, nthreads=nthreads)
        ext = g["extent"]
        x = (np.arange(nseg) + 0.5) * ext / nseg
        d = (x * x).astype(np.float32)
        r = g["reflectance"].astype(np.float32)
        L.o_mpc_resample_uniform(nseg, d, r, target, tab[c])
        last = np.float32(np.float32(target - 1) * d[-1] / np.float32(target - 1))
        rcp[c] = np.float32(target - 1) / last
        tot[c] = g["total_r"]
    return tab, rcp, tot
