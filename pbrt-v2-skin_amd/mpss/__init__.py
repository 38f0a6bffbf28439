"""mpss -- Python host binding of libmpss (the MI355X-native multipole subsurface path).

Thin ctypes layer over the C ABI in include/mpss.h.  Device buffers are passed as raw
HIP pointers (torch CUDA tensors' ``data_ptr()``); torch is plumbing here, not the product.
The HIP library is mandatory: importing this module raises if libmpss.so is missing, and
there is no CPU fallback anywhere in the product path.
"""
import ctypes as C
import os

import numpy as np

NB = 30
_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MPSS_LIB") or os.path.join(_HERE, "libmpss.so")  # MPSS_LIB: a variant build (tools/)

if not os.path.exists(LIB_PATH):
    raise ImportError("libmpss.so not built (%s): run __graft_entry__.build() or make -C pbrt-v2-skin_amd/csrc"
                      % LIB_PATH)

# torch-ROCm ships its own libamdhip64/libhsa-runtime64 (same SONAME, different NEEDED spelling).
# Loading libmpss first would pull /opt/rocm's runtime in beside torch's and leave two HSA
# runtimes fighting over /dev/kfd; importing torch first makes libmpss bind to torch's copy.
try:
    import torch  # noqa: F401
except ImportError:  # pure C/ctypes use without torch: /opt/rocm's runtime is used
    torch = None

_lib = C.CDLL(LIB_PATH)

f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
vp = C.c_void_p
u32 = C.c_uint32
u32p = C.POINTER(C.c_uint32)


class Config(C.Structure):
    """mpss_config (CreateMultipoleSubsurfaceIntegrator params, multipolesubsurface.cpp:393-401)."""
    _fields_ = [("device", C.c_int), ("max_depth", C.c_int), ("max_error", C.c_float),
                ("min_sample_distance", C.c_float), ("mix", C.c_float), ("show_irradiance_points", C.c_int),
                ("incenter", C.c_int), ("quick_render", C.c_int), ("exact_mo", C.c_int),
                ("kernel_timing", C.c_int), ("count_traversal", C.c_int), ("profile_on_host", C.c_int),
                ("max_batch_samples", C.c_int64), ("use_poisson_point_finder", C.c_int), ("sampler", C.c_int),
                ("replay_cores", C.c_int), ("octree_on_host", C.c_int), ("mo_band_dealing", C.c_int),
                ("mo_work_stealing", C.c_int), ("mo_near_field", C.c_int), ("tessellate_on_host", C.c_int),
                ("mo_common_grid", C.c_int)]

SAMPLER_HASH, SAMPLER_REFERENCE = 0, 1


class RenderStats(C.Structure):
    """mpss_render_stats."""
    _fields_ = [("ms_irradiance", C.c_double), ("ms_camera", C.c_double), ("ms_shade", C.c_double),
                ("ms_film", C.c_double), ("n_irradiance", C.c_int64), ("n_camera", C.c_int64),
                ("n_shade", C.c_int64), ("n_film", C.c_int64), ("samples", C.c_int64), ("sss_samples", C.c_int64),
                ("mo_nodes", C.c_int64), ("mo_points", C.c_int64), ("group_nodes", C.c_int64 * 8),
                ("group_points", C.c_int64 * 8), ("group_bands", (C.c_int32 * 4) * 8), ("ms_direct", C.c_double),
                ("n_direct", C.c_int64), ("mo_wave_node_iters", C.c_int64), ("mo_wave_point_iters", C.c_int64),
                ("mo_lookups", C.c_int64), ("mo_lookups_near", C.c_int64 * 3), ("mo_row_lane_records", C.c_int64),
                ("mo_lds_lane_records", C.c_int64), ("mo_table_lane_records", C.c_int64), ("ms_tex", C.c_double),
                ("n_tex", C.c_int64), ("ms_replay", C.c_double), ("n_replay", C.c_int64),
                ("group_path_records", (C.c_int64 * 3) * 8), ("group_path_sectors", (C.c_int64 * 2) * 8),
                ("group_path_lines", (C.c_int64 * 2) * 8), ("group_path_fetches", (C.c_int64 * 2) * 8)]


class LayeredSkin(C.Structure):
    """mpss_layeredskin (CreateLayeredSkinMaterial params, layeredskin.cpp:234-257)."""
    _fields_ = [("roughness", C.c_float), ("nmperunit", C.c_float), ("f_mel", C.c_float), ("f_eu", C.c_float),
                ("f_blood", C.c_float), ("f_ohg", C.c_float), ("ga_epi", C.c_float), ("ga_derm", C.c_float),
                ("b_derm", C.c_float), ("layer_thickness_nm", C.c_float * 2), ("layer_ior", C.c_float * 2),
                ("albedo", C.c_float * NB), ("Kr", C.c_float * NB), ("Kt", C.c_float * NB),
                ("desired_length", C.c_int), ("lerp_on_thin_slab", C.c_int),
                ("double_ref_sslf", C.c_int), ("use_monte_carlo", C.c_int), ("photons", C.c_uint64),
                ("rgb_profile", C.c_int), ("gen_profile", C.c_int), ("show_irradiance_points", C.c_int),
                ("irradiance_point_size", C.c_float)]


class Imagemap(C.Structure):
    """mpss_imagemap (Texture "imagemap" params, textures/imagemap.cpp:110-180)."""
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("texels", vp), ("is_float", C.c_int),
                ("shift", C.c_float), ("scale", C.c_float), ("gamma", C.c_float), ("wrap", C.c_int),
                ("trilinear", C.c_int), ("max_anisotropy", C.c_float), ("uscale", C.c_float), ("vscale", C.c_float),
                ("udelta", C.c_float), ("vdelta", C.c_float)]


def _sig(name, res, args):
    f = getattr(_lib, name)
    f.restype = res
    f.argtypes = args
    return f


_sig("mpss_abi_version", C.c_int, [])
_sig("mpss_last_error", C.c_char_p, [])
_sig("mpss_config_defaults", None, [C.POINTER(Config)])
_sig("mpss_create", C.c_int, [C.POINTER(Config), C.POINTER(vp)])
_sig("mpss_destroy", None, [vp])
_sig("mpss_layeredskin_defaults", None, [C.POINTER(LayeredSkin)])
_sig("mpss_add_layeredskin", C.c_int, [vp, C.POINTER(LayeredSkin), u32p])
_sig("mpss_set_material_tables", C.c_int, [vp, f32p, u32, f32p, f32p, u32, vp, C.c_int, u32p])
_sig("mpss_add_dipole_material", C.c_int, [vp, f32p, f32p, C.c_float, u32p])
_sig("mpss_host_dipole_rd", C.c_int, [f32p, f32p, C.c_float, u32, vp, vp, vp])
_sig("mpss_get_material_tables", C.c_int, [vp, u32, vp, u32p, vp, vp, u32p, vp])
_sig("mpss_get_gather_info", C.c_int, [vp, u32, C.POINTER(C.c_int), vp, vp])
_sig("mpss_set_irradiance_points", C.c_int, [vp, u32, f32p, f32p, f32p, f32p])
_sig("mpss_octree_info", C.c_int, [vp, u32p, u32p, u32p])
_sig("mpss_octree_export", C.c_int, [vp, vp, vp, vp, vp, vp])
_sig("mpss_mo_batch", C.c_int, [vp, u32, u32, vp, vp, vp, vp])
_sig("mpss_add_mesh", C.c_int, [vp, u32, f32p, vp, vp, vp, u32, C.POINTER(C.c_int32), f32p, f32p, C.c_int, u32])
_sig("mpss_add_sphere_light", C.c_int, [vp, f32p, C.c_float, f32p, C.c_int])
_sig("mpss_add_infinite_light", C.c_int, [vp, f32p, C.c_int, f32p, f32p])
_sig("mpss_add_infinite_light_map", C.c_int, [vp, f32p, C.c_int, f32p, f32p, C.c_int, C.c_int, f32p])
_sig("mpss_set_camera", C.c_int, [vp, f32p, f32p, C.c_int, C.c_int])
_sig("mpss_set_surface_points", C.c_int, [vp, u32, vp])
_sig("mpss_get_surface_points", C.c_int, [vp, vp, u32p])
_sig("mpss_get_irradiance", C.c_int, [vp, vp, u32p])
_sig("mpss_replay_samples", C.c_int, [vp, C.c_int, vp, C.POINTER(C.c_uint64), C.POINTER(C.c_int)])
_sig("mpss_load_pointsfile", C.c_int, [vp, C.c_char_p])
_sig("mpss_save_pointsfile", C.c_int, [vp, C.c_char_p])
_sig("mpss_preprocess", C.c_int, [vp, u32])
_sig("mpss_get_render_stats", C.c_int, [vp, C.POINTER(RenderStats)])
_sig("mpss_reset_render_stats", C.c_int, [vp])
_sig("mpss_set_instrumentation", C.c_int, [vp, C.c_int, C.c_int])
_sig("mpss_render_tile", C.c_int, [vp, C.c_int, u32, C.c_int, C.c_int, C.c_int, C.c_int, vp, vp])
_sig("mpss_render_tiles", C.c_int, [vp, C.c_int, u32, C.c_int, C.POINTER(C.c_int32), C.POINTER(vp), vp])
_sig("mpss_tile_costs", C.c_int, [vp, C.c_int, C.POINTER(C.c_int32), vp, vp])
_sig("mpss_host_from_rgb", C.c_int, [f32p, C.c_int, f32p])
_sig("mpss_mc_reference", C.c_int, [f32p, C.c_int, C.c_float, C.c_int, C.c_int, vp, vp, C.POINTER(C.c_double),
                                    C.POINTER(C.c_double)])
_sig("mpss_mc_profile", C.c_int, [vp, f32p, C.c_int, C.c_float, C.c_int, C.c_uint64, C.c_uint64, vp, vp,
                                  C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_uint64), vp])
_sig("mpss_host_tessellate", C.c_int, [u32, f32p, vp, vp, vp, u32, C.POINTER(C.c_int32), f32p, f32p, C.c_int, u32,
                                       C.c_float, C.c_int, vp, u32p])
_sig("mpss_imagemap_defaults", None, [C.POINTER(Imagemap)])
_sig("mpss_add_imagemap", C.c_int, [vp, C.POINTER(Imagemap), u32p])
_sig("mpss_set_material_textures", C.c_int, [vp, u32, C.c_int32, C.c_int32])
_sig("mpss_host_tessellate_bumped", C.c_int, [u32, f32p, vp, vp, vp, u32, C.POINTER(C.c_int32), f32p, f32p, C.c_int,
                                              u32, C.c_float, C.c_int, vp, vp, u32p])
_sig("mpss_host_imagemap_lookup", C.c_int, [C.POINTER(Imagemap), u32, f32p, f32p])
_sig("mpss_host_skin_layers", C.c_int, [C.POINTER(LayeredSkin), f32p, f32p, f32p, f32p])
_sig("mpss_host_build_profile", C.c_int, [f32p, f32p, f32p, f32p, C.c_int, C.c_int, vp, u32p, vp, vp])
_sig("mpss_host_rho_table", C.c_int, [C.c_float, C.c_float, C.c_int, C.c_int, C.c_int, f32p, C.POINTER(C.c_float)])
_sig("mpss_host_common_grid", C.c_int, [f32p, u32, f32p, C.c_int, C.c_int, vp, u32p] + [vp] * 11 + [C.POINTER(C.c_int)])
_sig("mpss_host_octree_export", C.c_int, [u32, f32p, f32p, f32p, f32p, u32p] + [vp] * 8)


class MpssError(RuntimeError):
    pass


def check(rc):
    if rc != 0:
        raise MpssError("libmpss error %d: %s" % (rc, _lib.mpss_last_error().decode()))


def lib():
    return _lib


def exported_symbols():
    """Names declared in include/mpss.h (checked by tests/test_abi.py)."""
    import re
    hdr = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "mpss.h")
    txt = open(hdr).read()
    return sorted(set(re.findall(r"\b(mpss_[a-z0-9_]+)\s*\(", txt)))


def default_config(**kw):
    c = Config()
    _lib.mpss_config_defaults(C.byref(c))
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def default_skin(**kw):
    m = LayeredSkin()
    _lib.mpss_layeredskin_defaults(C.byref(m))
    for k, v in kw.items():
        if k in ("layer_thickness_nm", "layer_ior"):
            setattr(m, k, (C.c_float * 2)(*v))
        elif k in ("albedo", "Kr", "Kt"):
            setattr(m, k, (C.c_float * NB)(*v))
        else:
            setattr(m, k, v)
    return m


_WRAP = {"repeat": 0, "black": 1, "clamp": 2}


def imagemap(texels=None, is_float=False, shift=0.0, scale=1.0, gamma=1.0, wrap="repeat", trilinear=False,
             maxanisotropy=8.0, uscale=1.0, vscale=1.0, udelta=0.0, vdelta=0.0):
    """An mpss_imagemap for an (H, W, 3) texel array (ReadImage's RGB, mpss.imageio), or for an
    image that could not be read (texels None: the reference's one-valued map). Returns (struct,
    the array it points at -- keep it alive while the struct is used)."""
    t = Imagemap()
    _lib.mpss_imagemap_defaults(C.byref(t))
    arr = None
    if texels is not None:
        arr = np.ascontiguousarray(texels, np.float32)
        if arr.ndim != 3 or arr.shape[2] != 3:
            raise ValueError("texels must be (height, width, 3)")
        t.height, t.width = arr.shape[:2]
        t.texels = arr.ctypes.data
    t.is_float = int(bool(is_float))
    t.shift, t.scale, t.gamma = float(shift), float(scale), float(gamma)
    if wrap not in _WRAP:
        raise ValueError("wrap mode %r" % wrap)
    t.wrap = _WRAP[wrap]
    t.trilinear = int(bool(trilinear))
    t.max_anisotropy = float(maxanisotropy)
    t.uscale, t.vscale, t.udelta, t.vdelta = float(uscale), float(vscale), float(udelta), float(vdelta)
    return t, arr


def host_imagemap_lookup(tex, uvd):
    """ImageTexture::Evaluate of the product's host code: tex = imagemap(...) kwargs dict;
    uvd (n, 6) = u, v, dudx, dvdx, dudy, dvdy -> (n, 3) MIPMap values."""
    t, keep = imagemap(**tex)
    uvd = np.ascontiguousarray(uvd, np.float32).reshape(-1, 6)
    out = np.zeros((len(uvd), 3), np.float32)
    check(_lib.mpss_host_imagemap_lookup(C.byref(t), len(uvd), uvd, out))
    del keep
    return out


# SurfacePoint record, the "pointsfile" format (renderers/surfacepoints.h:45-55), 44 B.
SURFACE_POINT = np.dtype([("p", "<f4", 3), ("n", "<f4", 3), ("u", "<f4"), ("v", "<f4"), ("material", "<u4"),
                          ("area", "<f4"), ("ray_eps", "<f4")])
assert SURFACE_POINT.itemsize == 44


# ------------------------------------------------------------------ host utilities
def host_from_rgb(rgb, illuminant=False):
    out = np.zeros(NB, np.float32)
    check(_lib.mpss_host_from_rgb(np.ascontiguousarray(rgb, np.float32), int(illuminant), out))
    return out


def host_tessellate(P, idx, o2w, w2o, min_dist, N=None, S=None, uv=None, flip=False, material=0, incenter=False,
                    bump=None):
    """TessellateSurfacePoints of one mesh by the product's host code; bump: imagemap(...) kwargs
    dict of a float "bumpmap" texture, or None."""
    P = np.ascontiguousarray(P, np.float32).reshape(-1, 3)
    idx = np.ascontiguousarray(idx, np.int32).reshape(-1, 3)
    opt = [None if a is None else np.ascontiguousarray(a, np.float32) for a in (N, S, uv)]
    args = [len(P), P] + [None if a is None else a.ctypes.data for a in opt] + \
        [len(idx), idx.ctypes.data_as(C.POINTER(C.c_int32)), np.ascontiguousarray(o2w, np.float32),
         np.ascontiguousarray(w2o, np.float32), int(flip), material, min_dist, int(incenter)]
    bt, keep = imagemap(**bump) if bump is not None else (None, None)
    args.append(C.byref(bt) if bt is not None else None)
    n = C.c_uint32(0)
    check(_lib.mpss_host_tessellate_bumped(*args, None, C.byref(n)))
    out = np.zeros(n.value, SURFACE_POINT)
    check(_lib.mpss_host_tessellate_bumped(*args, out.ctypes.data, C.byref(n)))
    del keep
    return out


def host_skin_layers(skin):
    mua = np.zeros((2, NB), np.float32)
    musp = np.zeros((2, NB), np.float32)
    th = np.zeros(2, np.float32)
    eta = np.zeros(2, np.float32)
    check(_lib.mpss_host_skin_layers(C.byref(skin), mua, musp, th, eta))
    return mua, musp, th, eta


def host_build_profile(mua, musp, thickness, eta, desired_length=512, lerp=True):
    args = [np.ascontiguousarray(x, np.float32) for x in (mua, musp, thickness, eta)]
    n = C.c_uint32()
    check(_lib.mpss_host_build_profile(*args, desired_length, int(lerp), None, C.byref(n), None, None))
    # the length query above ran the whole build; run once more into buffers
    tab = np.zeros((NB, n.value), np.float32)
    rcp = np.zeros(NB, np.float32)
    tot = np.zeros(NB, np.float32)
    check(_lib.mpss_host_build_profile(*args, desired_length, int(lerp), tab.ctypes.data, C.byref(n),
                                       rcp.ctypes.data, tot.ctypes.data))
    return tab, rcp, tot


def mc_reference(layers, mfp_range=16.0, nsegments=1024, lerp=True):
    """MultipoleReferenceTask (mcprofile.cpp:356-425): the multipole model of `layers`
    [(mua, musp, ior, thickness), ...] at the MC profile's ring centres; host code."""
    lay = np.ascontiguousarray(layers, np.float32).reshape(-1, 4)
    r = np.zeros(nsegments, np.float64)
    t = np.zeros(nsegments, np.float64)
    tr, tt = C.c_double(), C.c_double()
    check(_lib.mpss_mc_reference(lay, len(lay), mfp_range, nsegments, int(lerp), r.ctypes.data, t.ctypes.data,
                                 C.byref(tr), C.byref(tt)))
    return dict(reflectance=r, transmittance=t, total_r=tr.value, total_t=tt.value)


def host_dipole_rd(sigma_a, sigmap_s, eta, d2):
    """DiffusionReflectance(sigma_a, sigmap_s, eta)(d2) per squared distance (n x 30) and its
    TotalReflectance() (diffusionutil.h:38-83)."""
    d2 = np.ascontiguousarray(np.atleast_1d(d2), np.float32)
    rd = np.zeros((len(d2), NB), np.float32)
    tot = np.zeros(NB, np.float32)
    check(_lib.mpss_host_dipole_rd(np.ascontiguousarray(sigma_a, np.float32), np.ascontiguousarray(sigmap_s, np.float32),
                                   eta, len(d2), d2.ctypes.data, rd.ctypes.data, tot.ctypes.data))
    return rd, tot


def host_rho_table(roughness, eta, n=1025, sqrt_samples=256, double_ref_sslf=False):
    hd = np.zeros(n, np.float32)
    hh = C.c_float()
    check(_lib.mpss_host_rho_table(roughness, eta, int(double_ref_sslf), n, sqrt_samples, hd, C.byref(hh)))
    return hd, hh.value


def host_common_grid(table, rcp, snake=False, rgb=False, near_field=5088):
    """The sharded gather's common grid for a profile (mpss_host_common_grid): dict of rows
    (n_rows, 8), bands (8, 4), rg, u0lim, u1lim, u1start, row0, ubase (8,), rel_err / l1_err (30,),
    ok. rgb: an rgbprofile table (rows 0..2 in every group). near_field: the LDS layout the grid is
    built for (mpss_config.mo_near_field; 5088 is the default)."""
    table = np.ascontiguousarray(table, np.float32)
    rcp = np.ascontiguousarray(rcp, np.float32)
    L = table.shape[1]
    mode = 2 if rgb else int(snake)
    n = C.c_uint32(0)
    nul = [None] * 11
    ok = C.c_int()
    check(_lib.mpss_host_common_grid(table, L, rcp, mode, int(near_field), None, C.byref(n), *nul, C.byref(ok)))
    out = dict(rows=np.zeros((n.value, 8), np.float32), bands=np.zeros((8, 4), np.int32),
               rg=np.zeros(8, np.float32), u0lim=np.zeros(8, np.float32), u1lim=np.zeros(8, np.float32),
               u1start=np.zeros(8, np.float32), row0=np.zeros(8, np.uint32), ubase=np.zeros(8, np.uint32),
               rel_err=np.zeros(NB, np.float32), l1_err=np.zeros(NB, np.float32), ua=np.zeros(8, np.float32),
               hinv=np.zeros(8, np.float32))
    check(_lib.mpss_host_common_grid(table, L, rcp, mode, int(near_field), out["rows"].ctypes.data, C.byref(n),
                                     *[out[k].ctypes.data for k in ("bands", "rg", "u0lim", "u1lim", "u1start", "row0",
                                                                    "ubase", "rel_err", "l1_err", "ua", "hinv")],
                                     C.byref(ok)))
    out["ok"] = bool(ok.value)
    return out


def host_octree_export(p, n, E, area):
    p, n, E, area = [np.ascontiguousarray(x, np.float32) for x in (p, n, E, area)]
    nn = C.c_uint32()
    check(_lib.mpss_host_octree_export(len(p), p, n, E, area, C.byref(nn), *([None] * 8)))
    N = nn.value
    d = dict(p=np.zeros((N, 3), np.float32), area=np.zeros(N, np.float32), Et=np.zeros((N, NB), np.float32),
             depth=np.zeros(N, np.int32), skip=np.zeros(N, np.int32), leaf_first=np.zeros(N, np.int32),
             leaf_count=np.zeros(N, np.int32), order=np.zeros(len(p), np.int32))
    check(_lib.mpss_host_octree_export(len(p), p, n, E, area, C.byref(nn),
                                       *[d[k].ctypes.data for k in ("p", "area", "Et", "depth", "skip",
                                                                    "leaf_first", "leaf_count", "order")]))
    return d


# ------------------------------------------------------------------ device context
class Context:
    """One MultipoleSubsurfaceIntegrator instance (multipolesubsurface.h:36-80) on one GPU."""

    def __init__(self, **cfg):
        self.cfg = default_config(**cfg)
        h = vp()
        check(_lib.mpss_create(C.byref(self.cfg), C.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            _lib.mpss_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def add_layeredskin(self, skin):
        mid = C.c_uint32()
        check(_lib.mpss_add_layeredskin(self.h, C.byref(skin), C.byref(mid)))
        return mid.value

    def set_material_tables(self, table, rcp, rho_hd, albedo=None, is_mc=False):
        table = np.ascontiguousarray(table, np.float32)
        al = None if albedo is None else np.ascontiguousarray(albedo, np.float32)
        mid = C.c_uint32()
        check(_lib.mpss_set_material_tables(self.h, table, table.shape[1], np.ascontiguousarray(rcp, np.float32),
                                            np.ascontiguousarray(rho_hd, np.float32), len(rho_hd),
                                            None if al is None else al.ctypes.data, int(is_mc), C.byref(mid)))
        return mid.value

    def add_dipole_material(self, sigma_a, sigmap_s, eta):
        """A DiffusionReflectance Rd functor for mo_batch (the dipolesubsurface integrator's Rd)."""
        mid = C.c_uint32()
        check(_lib.mpss_add_dipole_material(self.h, np.ascontiguousarray(sigma_a, np.float32),
                                            np.ascontiguousarray(sigmap_s, np.float32), eta, C.byref(mid)))
        return mid.value

    def material_tables(self, mid):
        L = C.c_uint32()
        nr = C.c_uint32()
        check(_lib.mpss_get_material_tables(self.h, mid, None, C.byref(L), None, None, C.byref(nr), None))
        tab = np.zeros((NB, L.value), np.float32)
        rcp = np.zeros(NB, np.float32)
        rho = np.zeros(nr.value, np.float32)
        tot = np.zeros(NB, np.float32)
        check(_lib.mpss_get_material_tables(self.h, mid, tab.ctypes.data, C.byref(L), rcp.ctypes.data,
                                            rho.ctypes.data, C.byref(nr), tot.ctypes.data))
        return tab, rcp, rho, tot

    def gather_info(self, mid):
        """mpss_get_gather_info: {common_grid: bool, rel_err: (30,), l1_err: (30,)}."""
        on = C.c_int()
        rel = np.zeros(NB, np.float32)
        l1 = np.zeros(NB, np.float32)
        check(_lib.mpss_get_gather_info(self.h, mid, C.byref(on), rel.ctypes.data, l1.ctypes.data))
        return dict(common_grid=bool(on.value), rel_err=rel, l1_err=l1)

    def set_irradiance_points(self, p, n, E, area):
        p, n, E, area = [np.ascontiguousarray(x, np.float32) for x in (p, n, E, area)]
        check(_lib.mpss_set_irradiance_points(self.h, len(p), p, n, E, area))

    def octree_info(self):
        a, b, c = C.c_uint32(), C.c_uint32(), C.c_uint32()
        check(_lib.mpss_octree_info(self.h, C.byref(a), C.byref(b), C.byref(c)))
        return dict(n_nodes=a.value, max_depth=b.value, n_points=c.value)

    def octree_export(self):
        """The device octree as the gather reads it (mpss_octree_export): nodes as raw 64-B records
        (np.void), node_et [N, 32], pt_hdr [M, 4], pt_e [M, 32], pt_index [M]."""
        info = self.octree_info()
        N, M = info["n_nodes"], info["n_points"]
        d = dict(nodes=np.zeros((N, 16), np.uint32), node_et=np.zeros((N, 32), np.float32),
                 pt_hdr=np.zeros((M, 4), np.float32), pt_e=np.zeros((M, 32), np.float32),
                 pt_index=np.zeros(M, np.int32))
        check(_lib.mpss_octree_export(self.h, *[d[k].ctypes.data_as(vp) for k in
                                                ("nodes", "node_et", "pt_hdr", "pt_e", "pt_index")]))
        return d

    def mo_batch(self, mid, q, p_dev, mo_dev, counters_dev=None, stream=None):
        check(_lib.mpss_mo_batch(self.h, mid, q, p_dev, mo_dev, counters_dev, stream))

    # ---- scene slice of the per-pixel path
    def add_mesh(self, P, idx, o2w, w2o, material, N=None, S=None, uv=None, reverse=False):
        P = np.ascontiguousarray(P, np.float32).reshape(-1, 3)
        idx = np.ascontiguousarray(idx, np.int32).reshape(-1, 3)
        opt = [None if a is None else np.ascontiguousarray(a, np.float32) for a in (N, S, uv)]
        self._keep = opt
        check(_lib.mpss_add_mesh(self.h, len(P), P, *[None if a is None else a.ctypes.data for a in opt],
                                 len(idx), idx.ctypes.data_as(C.POINTER(C.c_int32)),
                                 np.ascontiguousarray(o2w, np.float32), np.ascontiguousarray(w2o, np.float32),
                                 int(reverse), material))

    def add_imagemap(self, **tex):
        """Texture "imagemap" (see mpss.imagemap for the keywords); returns its texture id."""
        t, keep = imagemap(**tex)
        tid = C.c_uint32(0)
        check(_lib.mpss_add_imagemap(self.h, C.byref(t), C.byref(tid)))
        del keep
        return tid.value

    def set_material_textures(self, material, albedo=-1, bump=-1):
        check(_lib.mpss_set_material_textures(self.h, material, albedo, bump))

    def add_sphere_light(self, center, radius, Lemit, nsamples=1):
        check(_lib.mpss_add_sphere_light(self.h, np.ascontiguousarray(center, np.float32), radius,
                                         np.ascontiguousarray(Lemit, np.float32), nsamples))

    def add_infinite_light(self, L, nsamples=1, light_to_world=None, world_to_light=None, texels=None):
        """LightSource "infinite"; L = the 30-band L * scale (CreateInfiniteLight); texels = the
        map as an (H, W, 3) float array (ReadImage's RGB), or None for a constant light."""
        l2w = np.eye(4, dtype=np.float32) if light_to_world is None else light_to_world
        w2l = np.linalg.inv(np.asarray(l2w, np.float64)) if world_to_light is None else world_to_light
        args = (self.h, np.ascontiguousarray(L, np.float32), nsamples, np.ascontiguousarray(l2w, np.float32),
                np.ascontiguousarray(w2l, np.float32))
        if texels is None:
            check(_lib.mpss_add_infinite_light(*args))
        else:
            tex = np.ascontiguousarray(texels, np.float32)
            if tex.ndim != 3 or tex.shape[2] != 3:
                raise ValueError("texels must be (height, width, 3)")
            check(_lib.mpss_add_infinite_light_map(*args, tex.shape[1], tex.shape[0], tex))

    def set_camera(self, raster_to_camera, camera_to_world, xres, yres):
        check(_lib.mpss_set_camera(self.h, np.ascontiguousarray(raster_to_camera, np.float32),
                                   np.ascontiguousarray(camera_to_world, np.float32), xres, yres))

    def set_surface_points(self, recs):
        recs = np.ascontiguousarray(recs, SURFACE_POINT)
        check(_lib.mpss_set_surface_points(self.h, len(recs), recs.ctypes.data))

    def surface_points(self):
        n = C.c_uint32()
        check(_lib.mpss_get_surface_points(self.h, None, C.byref(n)))
        out = np.zeros(n.value, SURFACE_POINT)
        check(_lib.mpss_get_surface_points(self.h, out.ctypes.data, C.byref(n)))
        return out

    def load_pointsfile(self, path):
        check(_lib.mpss_load_pointsfile(self.h, os.fsencode(path)))

    def save_pointsfile(self, path):
        check(_lib.mpss_save_pointsfile(self.h, os.fsencode(path)))

    def mc_profile(self, layers, mfp_range=16.0, nsegments=1024, nphotons=100, seed=89, stream=None):
        """Monte-Carlo layered profile; layers: [(mua, musp, ior, thickness), ...]."""
        lay = np.ascontiguousarray(layers, np.float32).reshape(-1, 4)
        r = np.zeros(nsegments, np.float64)
        t = np.zeros(nsegments, np.float64)
        tr, tt, ev = C.c_double(), C.c_double(), C.c_uint64()
        check(_lib.mpss_mc_profile(self.h, lay, len(lay), mfp_range, nsegments, nphotons, seed, r.ctypes.data,
                                   t.ctypes.data, C.byref(tr), C.byref(tt), C.byref(ev), stream))
        return dict(reflectance=r, transmittance=t, total_r=tr.value, total_t=tt.value, events=ev.value)

    def replay_samples(self, spp, xres, yres):
        """The reference sampler's values over the sample extent: (yres+1, xres+1, spp', K) float32."""
        n, k = C.c_uint64(), C.c_int()
        check(_lib.mpss_replay_samples(self.h, spp, None, C.byref(n), C.byref(k)))
        out = np.zeros(n.value, np.float32)
        check(_lib.mpss_replay_samples(self.h, spp, out.ctypes.data, C.byref(n), C.byref(k)))
        return out.reshape(yres + 1, xres + 1, -1, k.value)

    def irradiance(self):
        n = C.c_uint32()
        check(_lib.mpss_get_irradiance(self.h, None, C.byref(n)))
        out = np.zeros((n.value, NB), np.float32)
        check(_lib.mpss_get_irradiance(self.h, out.ctypes.data, C.byref(n)))
        return out

    def render_stats(self):
        st = RenderStats()
        check(_lib.mpss_get_render_stats(self.h, C.byref(st)))
        out = {}
        for k, _ in RenderStats._fields_:
            v = getattr(st, k)
            out[k] = [list(x) for x in v] if k == "group_bands" or k.startswith("group_path") else (
                list(v) if k.startswith("group_") or k == "mo_lookups_near" else v)
        return out

    def set_instrumentation(self, kernel_timing=False, count_traversal=False):
        """count_traversal: False/0, True/1 (the gather's own visits), or 2 (the reference
        traversal's visits: reach pruning off, results unchanged)."""
        check(_lib.mpss_set_instrumentation(self.h, int(kernel_timing), int(count_traversal)))

    def reset_render_stats(self):
        check(_lib.mpss_reset_render_stats(self.h))

    def preprocess(self, seed=0):
        check(_lib.mpss_preprocess(self.h, seed))

    def render_tile(self, spp, seed, x0, x1, y0, y1, out_dev, stream=None):
        check(_lib.mpss_render_tile(self.h, spp, seed, x0, x1, y0, y1, out_dev, stream))

    def tile_costs(self, rects):
        """Per rectangle (x0, x1, y0, y1): camera rays through pixel centres that hit a BSSRDF
        surface, and that hit any mesh (mpss_tile_costs) -> two int64 arrays."""
        n = len(rects)
        r = (C.c_int32 * (4 * max(n, 1)))(*[int(v) for rc in rects for v in rc])
        sss = np.zeros(max(n, 1), np.int64)
        surf = np.zeros(max(n, 1), np.int64)
        check(_lib.mpss_tile_costs(self.h, n, r, sss.ctypes.data, surf.ctypes.data))
        return sss[:n], surf[:n]

    def render_tiles(self, spp, seed, rects, outs_dev, stream=None):
        """rects: [(x0, x1, y0, y1)], outs_dev: device pointers (one float4 XYZW tile each)."""
        n = len(rects)
        r = (C.c_int32 * (4 * n))(*[int(v) for rc in rects for v in rc])
        o = (vp * n)(*outs_dev)
        check(_lib.mpss_render_tiles(self.h, spp, seed, n, r, o, stream))
