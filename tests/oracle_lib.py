"""ctypes front-end to the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: the oracle is the parity checker; it is imported by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the
product package.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
NB = 30

_lib = None

f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")


class SkinParams(C.Structure):
    _fields_ = [("roughness", C.c_float), ("nmperunit", C.c_float), ("f_mel", C.c_float),
                ("f_eu", C.c_float), ("f_blood", C.c_float), ("f_ohg", C.c_float),
                ("layer_thickness_nm", C.c_float * 2), ("layer_ior", C.c_float * 2)]


class LayerSpec(C.Structure):
    _fields_ = [("ior", C.c_float), ("thickness", C.c_float), ("mua", C.c_float), ("musp", C.c_float)]


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    path = os.path.join(ORACLE_DIR, "liboracle.so")
    if not os.path.exists(path):
        build()
    L = C.CDLL(path)
    L.o_average_spectrum_samples.restype = C.c_float
    L.o_average_spectrum_samples.argtypes = [f32p, f32p, C.c_int, C.c_float, C.c_float]
    L.o_from_rgb.argtypes = [f32p, C.c_int, f32p]
    L.o_to_rgb.argtypes = [f32p, f32p]
    L.o_y.restype = C.c_float
    L.o_y.argtypes = [f32p]
    L.o_to_xyz.argtypes = [f32p, f32p]
    L.o_skin_layers.argtypes = [C.POINTER(SkinParams), f32p, f32p, f32p, f32p]
    L.o_kiss_fft.argtypes = [C.c_int, C.c_int, f64p, f64p]
    L.o_kiss_fftndr2.argtypes = [C.c_int, C.c_int, f64p, f64p]
    L.o_kiss_fftndri2.argtypes = [C.c_int, C.c_int, f64p, f64p]
    L.o_mpc_profile.restype = C.c_int
    L.o_mpc_profile.argtypes = [C.c_int, C.POINTER(LayerSpec), C.c_float, C.c_int, C.c_int, C.c_int,
                                C.POINTER(C.POINTER(C.c_float)), C.POINTER(C.POINTER(C.c_float)),
                                C.POINTER(C.POINTER(C.c_float)), C.POINTER(C.c_float), C.POINTER(C.c_float)]
    L.o_free.argtypes = [C.c_void_p]
    L.o_dipole_rd.restype = C.c_float
    L.o_dipole_rd.argtypes = [C.c_float] * 5 + [C.c_int, C.c_int, C.c_float]
    L.o_compute_profile.restype = C.c_int
    L.o_compute_profile.argtypes = [f32p, f32p, f32p, f32p, C.c_int, C.c_int, C.c_int,
                                    C.POINTER(C.POINTER(C.c_float)), f32p, f32p, f32p]
    L.o_sample_profile.restype = C.c_float
    L.o_sample_profile.argtypes = [f32p, C.c_int, C.c_float, C.c_float]
    L.o_rho_table.argtypes = [C.c_float, C.c_float, C.c_int, C.c_int, C.c_int, f32p, C.POINTER(C.c_float)]
    L.o_rho_table_ex.argtypes = [C.c_float, C.c_float, C.c_int, C.c_int, C.c_int, C.c_int, f32p, C.POINTER(C.c_float)]
    L.o_mt_first.restype = C.c_uint32
    L.o_mt_first.argtypes = [C.c_uint32, C.c_int, np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")]
    L.o_octree_build.restype = C.c_void_p
    L.o_octree_build.argtypes = [C.c_int, f32p, f32p, f32p, f32p]
    L.o_octree_free.argtypes = [C.c_void_p]
    L.o_octree_num_nodes.restype = C.c_int
    L.o_octree_num_nodes.argtypes = [C.c_void_p]
    L.o_mo_batch.argtypes = [C.c_void_p, C.c_int, f32p, f32p, C.c_int, f32p, C.c_float, f32p,
                             C.c_void_p, C.c_void_p, C.c_int]
    L.o_mo_batch_rgb.argtypes = [C.c_void_p, C.c_int, f32p, f32p, C.c_int, f32p, C.c_float, f32p,
                                 C.c_void_p, C.c_void_p, C.c_int]
    L.o_diffusion_init.argtypes = [f32p, f32p, C.c_float, C.c_void_p]
    L.o_diffusion_eval.argtypes = [C.c_void_p, C.c_float, f32p]
    L.o_diffusion_total.argtypes = [C.c_void_p, f32p]
    L.o_mo_batch_diffusion.argtypes = [C.c_void_p, C.c_int, f32p, C.c_void_p, C.c_float, f32p, C.c_void_p,
                                       C.c_void_p, C.c_int]
    L.o_octree_export.restype = C.c_int
    L.o_octree_export.argtypes = [C.c_void_p] + [C.c_void_p] * 10
    L.o_octree_bounds.argtypes = [C.c_void_p, f32p, f32p]
    _lib = L
    return L


def nthreads():
    return max(1, min(os.cpu_count() or 1, 16))


def to_rgb(s):
    """SampledSpectrum::ToRGB (ToXYZ + XYZToRGB, spectrum.h:51-55, 374-398)."""
    out = np.zeros(3, np.float32)
    lib().o_to_rgb(np.ascontiguousarray(s, np.float32), out)
    return out


def from_rgb(rgb, illuminant=False):
    out = np.zeros(NB, np.float32)
    lib().o_from_rgb(np.asarray(rgb, np.float32), int(illuminant), out)
    return out


def y_of(s):
    return lib().o_y(np.ascontiguousarray(s, np.float32))


def skin_layers(roughness=0.3, nmperunit=40e6, f_mel=0.5, f_eu=0.5, f_blood=0.5, f_ohg=0.5,
                thickness_nm=(0.25e6, 20e6), ior=(1.4, 1.4)):
    p = SkinParams(roughness, nmperunit, f_mel, f_eu, f_blood, f_ohg, (C.c_float * 2)(*thickness_nm),
                   (C.c_float * 2)(*ior))
    mua = np.zeros((2, NB), np.float32)
    musp = np.zeros((2, NB), np.float32)
    th = np.zeros(2, np.float32)
    eta = np.zeros(2, np.float32)
    lib().o_skin_layers(C.byref(p), mua, musp, th, eta)
    return mua, musp, th, eta


def mpc_profile(layers, step, desired_length=512, lerp=True, resample=True):
    specs = (LayerSpec * len(layers))(*[LayerSpec(*l) for l in layers])
    d = C.POINTER(C.c_float)()
    r = C.POINTER(C.c_float)()
    t = C.POINTER(C.c_float)()
    tr = C.c_float()
    tt = C.c_float()
    n = lib().o_mpc_profile(len(layers), specs, step, desired_length, int(lerp), int(resample),
                            C.byref(d), C.byref(r), C.byref(t), C.byref(tr), C.byref(tt))
    out = [np.ctypeslib.as_array(x, shape=(n,)).copy() for x in (d, r, t)]
    for x in (d, r, t):
        lib().o_free(x)
    return out[0], out[1], out[2], tr.value, tt.value


def compute_profile(mua, musp, eta, thickness, desired_length=512, lerp=True):
    tab = C.POINTER(C.c_float)()
    rcp = np.zeros(NB, np.float32)
    spacing = np.zeros(NB, np.float32)
    total = np.zeros(NB, np.float32)
    n = lib().o_compute_profile(np.ascontiguousarray(mua, np.float32), np.ascontiguousarray(musp, np.float32),
                                np.ascontiguousarray(eta, np.float32), np.ascontiguousarray(thickness, np.float32),
                                desired_length, int(lerp), nthreads(), C.byref(tab), rcp, spacing, total)
    if n < 0:
        raise RuntimeError("channel profile lengths differ")
    table = np.ctypeslib.as_array(tab, shape=(NB, n)).copy()
    lib().o_free(tab)
    return table, rcp, spacing, total


def rho_table(roughness, eta, n_entries=1025, sqrt_samples=256, fixed=False):
    """fixed: LayeredSkin's doublerefsslf (FixedFresnelDielectric, reflection.h:315-324)."""
    hd = np.zeros(n_entries, np.float32)
    hh = C.c_float()
    lib().o_rho_table_ex(roughness, eta, int(fixed), n_entries, sqrt_samples, nthreads(), hd, C.byref(hh))
    return hd, hh.value


class Diffusion:
    """DiffusionReflectance (diffusionutil.h:38-83): the single-dipole Rd functor."""

    def __init__(self, sigma_a, sigmap_s, eta):
        # o_diffusion: 5 x 30 floats + A
        self.buf = C.create_string_buffer(4 * (5 * NB + 1))
        lib().o_diffusion_init(np.ascontiguousarray(sigma_a, np.float32), np.ascontiguousarray(sigmap_s, np.float32),
                               eta, self.buf)

    def __call__(self, d2):
        d2 = np.atleast_1d(np.asarray(d2, np.float32))
        out = np.zeros((len(d2), NB), np.float32)
        row = np.zeros(NB, np.float32)
        for i, v in enumerate(d2):
            lib().o_diffusion_eval(self.buf, float(v), row)
            out[i] = row
        return out

    def total(self):
        out = np.zeros(NB, np.float32)
        lib().o_diffusion_total(self.buf, out)
        return out


class Octree:
    def __init__(self, p, n, E, area):
        self.p = np.ascontiguousarray(p, np.float32)
        self.handle = lib().o_octree_build(len(self.p), self.p, np.ascontiguousarray(n, np.float32),
                                           np.ascontiguousarray(E, np.float32),
                                           np.ascontiguousarray(area, np.float32))

    def __del__(self):
        if getattr(self, "handle", None):
            lib().o_octree_free(self.handle)
            self.handle = None

    def num_nodes(self):
        return lib().o_octree_num_nodes(self.handle)

    def bounds(self):
        a = np.zeros(3, np.float32)
        b = np.zeros(3, np.float32)
        lib().o_octree_bounds(self.handle, a, b)
        return a, b

    def mo(self, q, table, rcp, max_error, counters=False):
        q = np.ascontiguousarray(q, np.float32)
        table = np.ascontiguousarray(table, np.float32)
        out = np.zeros((len(q), NB), np.float32)
        nn = np.zeros(len(q), np.int32) if counters else None
        npt = np.zeros(len(q), np.int32) if counters else None
        lib().o_mo_batch(self.handle, len(q), q, table, table.shape[1], np.ascontiguousarray(rcp, np.float32),
                         max_error, out, nn.ctypes.data if counters else None,
                         npt.ctypes.data if counters else None, nthreads())
        return (out, nn, npt) if counters else out

    def mo_rgb(self, q, table, rcp, max_error):
        """Mo with an rgbprofile material: table rows 0..2 = the R, G, B profiles, rcp[:3]."""
        q = np.ascontiguousarray(q, np.float32)
        table = np.ascontiguousarray(table[:3], np.float32)
        out = np.zeros((len(q), NB), np.float32)
        lib().o_mo_batch_rgb(self.handle, len(q), q, table, table.shape[1],
                             np.ascontiguousarray(np.asarray(rcp, np.float32)[:3]), max_error, out, None, None,
                             nthreads())
        return out

    def mo_diffusion(self, q, dip, max_error, counters=False):
        q = np.ascontiguousarray(q, np.float32)
        out = np.zeros((len(q), NB), np.float32)
        nn = np.zeros(len(q), np.int32) if counters else None
        npt = np.zeros(len(q), np.int32) if counters else None
        lib().o_mo_batch_diffusion(self.handle, len(q), q, dip.buf, max_error, out,
                                   nn.ctypes.data if counters else None, npt.ctypes.data if counters else None,
                                   nthreads())
        return (out, nn, npt) if counters else out

    def export(self):
        n = lib().o_octree_export(self.handle, *([None] * 10))
        d = dict(p=np.zeros((n, 3), np.float32), area=np.zeros(n, np.float32), Et=np.zeros((n, NB), np.float32),
                 bmin=np.zeros((n, 3), np.float32), bmax=np.zeros((n, 3), np.float32),
                 depth=np.zeros(n, np.int32), skip=np.zeros(n, np.int32), leaf_first=np.zeros(n, np.int32),
                 leaf_count=np.zeros(n, np.int32), order=np.zeros(len(self.p), np.int32))
        lib().o_octree_export(self.handle, *[d[k].ctypes.data for k in
                                             ("p", "area", "Et", "bmin", "bmax", "depth", "skip",
                                              "leaf_first", "leaf_count", "order")])
        return d
