"""LightSource "infinite" without a map (lights/infinite.cpp): CPU checks of the oracle's
restatement against closed forms, and of the scene loader. The GPU-vs-oracle parity tests are
in test_render_parity_gpu.py.

  sky pixels     a camera ray that escapes returns sum_i lights[i]->Le(ray)
                 (samplerrenderer.cpp:144-151): for a constant map, Spectrum(L.ToRGBSpectrum(),
                 SPECTRUM_ILLUMINANT) up to the rounding of the four bilinear texel weights
  irradiance     IrradianceTask (multipolesubsurface.cpp:196-236) with Sample_L's
                 pdf = 1 / (2 pi^2 sin(theta)) converges to alb_mix * Le * 2 pi *
                 int_0^1 (1 - rho(mu)) mu dmu on an unoccluded upward plane -- this pins the
                 pdf normalisation and the Dot(wi, n) <= 0 rejection
"""
import os

import numpy as np
import pytest

import oracle_lib
import oracle_render as orr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NB = 30


def envmap_texels(W, H, seed=0):
    """A synthetic lat-long sky: a smooth gradient plus a small bright sun (row 0 = theta 0)."""
    v, u = np.meshgrid((np.arange(H) + 0.5) / H, (np.arange(W) + 0.5) / W, indexing="ij")
    base = 0.3 + 0.2 * np.cos(np.pi * v)[..., None] * np.array([0.8, 0.9, 1.2])
    d2 = (u - 0.3) ** 2 + (v - 0.25) ** 2
    sun = 40.0 * np.exp(-d2 / 0.002)[..., None] * np.array([1.0, 0.9, 0.7])
    rng = np.random.default_rng(seed)
    return (base + sun + 0.05 * rng.random((H, W, 3))).astype(np.float32)


def _write_pfm_file_order(path, tex):
    """PFM with rows in array order (ReadImagePFM does not flip)."""
    h, w, _ = tex.shape
    with open(path, "wb") as f:
        f.write(b"PF\n%d %d\n-1\n" % (w, h))
        f.write(np.ascontiguousarray(tex, "<f4").tobytes())


def _plane_scene(mpss, light, xres=16, yres=16, half=50.0, spp=4):
    from mpss import pbrtscene
    sc = pbrtscene.Scene()
    sc.xres, sc.yres, sc.spp = xres, yres, spp
    sc.fov = 60.0
    sc.materials = [{"desired_length": 64}]
    P = np.array([[-half, -half, 0], [half, -half, 0], [half, half, 0], [-half, half, 0]], np.float32)
    idx = np.array([[0, 1, 2], [0, 2, 3]], np.int32)
    eye = np.eye(4, dtype=np.float32)
    sc.meshes = [dict(P=P, N=None, S=None, uv=None, indices=idx, o2w=eye, w2o=eye, reverse=False, material=0)]
    sc.lights = [light]
    return sc


def _sky(L=(0.3, 0.35, 0.45), scale=(2, 2, 2), ns=4, rot=None):
    l2w = np.eye(4) if rot is None else rot
    return dict(kind="infinite", L=list(L), scale=list(scale), nsamples=ns, l2w=l2w.astype(np.float32),
                w2l=np.linalg.inv(l2w).astype(np.float32))


def _le(li):
    """Spectrum(L.ToRGBSpectrum(), SPECTRUM_ILLUMINANT) with the oracle's own helpers."""
    Lsc = oracle_lib.from_rgb(li["L"]) * oracle_lib.from_rgb(li["scale"])
    rgb = _to_rgb(Lsc)
    return oracle_lib.from_rgb(rgb, illuminant=True)


def _to_rgb(s):
    lib = oracle_lib.lib()
    lib.o_to_rgb.argtypes = [oracle_lib.f32p, oracle_lib.f32p]
    out = np.zeros(3, np.float32)
    lib.o_to_rgb(np.ascontiguousarray(s, np.float32), out)
    return out


def test_loader_reads_infinite_light(mpss):
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "tissue_sky.pbrt"))
    kinds = [li.get("kind", "area") for li in sc.lights]
    assert kinds == ["infinite", "area"]  # scene->lights in declaration order
    sky = sc.lights[0]
    assert sky["nsamples"] == 4 and sky["L"] == [0.3, 0.35, 0.45] and sky["scale"] == [2.0, 2.0, 2.0]
    c, s = np.cos(np.radians(30)), np.sin(np.radians(30))
    np.testing.assert_allclose(sky["l2w"][:3, :3], [[1, 0, 0], [0, c, -s], [0, s, c]], atol=1e-6)
    np.testing.assert_allclose(sky["l2w"][:3, :3] @ sky["w2l"][:3, :3], np.eye(3), atol=1e-6)


def test_loader_reads_mapname_relative_to_scene(mpss, tmp_path):
    from mpss import film, imageio, pbrtscene
    tex = envmap_texels(12, 7)
    _write_pfm_file_order(tmp_path / "sky.pfm", tex)
    f = tmp_path / "m.pbrt"
    f.write_text('WorldBegin\nLightSource "infinite" "string mapname" "sky.pfm" "integer nsamples" 2\nWorldEnd\n')
    sc = pbrtscene.load(str(f))
    li = sc.lights[0]
    assert li["mapname"] == str(tmp_path / "sky.pfm") and li["nsamples"] == 2
    np.testing.assert_array_equal(pbrtscene.infinite_texels(li), tex)
    bad = tmp_path / "b.pbrt"
    bad.write_text('WorldBegin\nLightSource "infinite" "string mapname" "sky.hdr"\nWorldEnd\n')
    with pytest.raises(ValueError, match="suffix"):
        pbrtscene.infinite_texels(pbrtscene.load(str(bad)).lights[0])


def test_oracle_sky_pixels(mpss, oracle):
    """A camera looking up at the sky (the plane is behind it): every sample escapes and the
    film gets Le of the constant map in every pixel."""
    li = _sky(rot=np.array([[0, 0, 1, 0], [1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 0, 1]], np.float64))
    sc = _plane_scene(mpss, li)
    sc.world_to_camera = np.eye(4)
    sc.world_to_camera[2, 3] = -10.0   # camera at z = 10 looking along +z, away from the plane
    cfg = mpss.default_config(min_sample_distance=10.0)
    o = orr.OracleScene(sc, orr.tables_from_host(sc, mpss), cfg, mpss)
    img = o.render_tile(sc.spp, 1, 0, sc.xres, 0, sc.yres, nthreads=4)
    xyz = (img[..., :3] / img[..., 3:4]).reshape(-1, 3)
    np.testing.assert_allclose(xyz[:, 1], oracle_lib.y_of(_le(li)), rtol=2e-6)
    np.testing.assert_allclose(xyz, np.tile(xyz[0], (len(xyz), 1)), rtol=2e-6)


@pytest.mark.parametrize("ns", [4, 16])
def test_oracle_irradiance_under_constant_sky(mpss, oracle, ns):
    li = _sky(ns=ns)
    sc = _plane_scene(mpss, li, half=1.0)
    cfg = mpss.default_config(min_sample_distance=0.02)
    tabs = orr.tables_from_host(sc, mpss)
    o = orr.OracleScene(sc, tabs, cfg, mpss)
    pts = o.tessellate()
    assert len(pts) > 5000
    E = o.irradiance(pts, 7)
    rho = tabs[0][2].astype(np.float64)
    mu = np.linspace(0, 1, 200001)
    r = np.interp(mu, np.linspace(0, 1, len(rho)), rho)
    expect = _le(li).astype(np.float64) * 2 * np.pi * np.trapezoid((1 - r) * mu, mu)
    got = E.astype(np.float64).mean(0)
    np.testing.assert_allclose(got, expect, rtol=0.02)
    # the per-point estimator is bounded: Ft Le cos / pdf <= Le * 2 pi^2
    assert np.all(E <= _le(li) * 2 * np.pi ** 2 * 1.0001)


# ------------------------------------------------------------------ image readers (mapname)
def _exr_bytes(tex, comp, ptype=1, channels="BGR"):
    """A scanline OpenEXR with the given compression (0 NONE, 1 RLE, 2 ZIPS, 3 ZIP) and pixel type
    (1 HALF, 2 FLOAT): the encoder side of the formats mpss.imageio decodes."""
    import struct
    import zlib
    h, w, _ = tex.shape
    dt = {1: "<f2", 2: "<f4"}[ptype]

    def attr(name, typ, data):
        return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(data)) + data

    chans = b"".join(c.encode() + b"\0" + struct.pack("<iB3xii", ptype, 0, 1, 1) for c in sorted(channels)) + b"\0"
    hdr = struct.pack("<ii", 20000630, 2) + attr("channels", "chlist", chans)
    hdr += attr("compression", "compression", bytes([comp]))
    hdr += attr("dataWindow", "box2i", struct.pack("<iiii", 0, 0, w - 1, h - 1))
    hdr += attr("displayWindow", "box2i", struct.pack("<iiii", 0, 0, w - 1, h - 1))
    hdr += attr("lineOrder", "lineOrder", b"\0") + b"\0"
    lpb = {0: 1, 1: 1, 2: 1, 3: 16}[comp]
    idx = {"R": 0, "G": 1, "B": 2}
    blocks = []
    for y0 in range(0, h, lpb):
        raw = b"".join(tex[y, :, idx[c]].astype(dt).tobytes() for y in range(y0, min(h, y0 + lpb))
                       for c in sorted(channels))
        if comp == 0:
            data = raw
        else:
            b = np.frombuffer(raw, np.uint8)
            inter = np.concatenate([b[0::2], b[1::2]]).astype(np.int32)
            pred = inter.copy()
            pred[1:] = (inter[1:] - inter[:-1] + 128) & 0xFF
            pred = pred.astype(np.uint8).tobytes()
            if comp == 1:  # literal runs only (valid RLE)
                out = bytearray()
                for k in range(0, len(pred), 127):
                    chunk = pred[k:k + 127]
                    out += struct.pack("b", -len(chunk)) + chunk
                data = bytes(out)
            else:
                data = zlib.compress(pred)
            if len(data) >= len(raw):
                data = raw
        blocks.append(struct.pack("<ii", y0, len(data)) + data)
    off = len(hdr) + 8 * len(blocks)
    table = []
    for bl in blocks:
        table.append(off)
        off += len(bl)
    return hdr + struct.pack("<%dQ" % len(blocks), *table) + b"".join(blocks)


@pytest.mark.parametrize("comp", [0, 1, 2, 3])
@pytest.mark.parametrize("ptype", [1, 2])
def test_imageio_exr(mpss, tmp_path, comp, ptype):
    from mpss import imageio
    tex = envmap_texels(37, 21, seed=comp)
    p = tmp_path / "m.exr"
    p.write_bytes(_exr_bytes(tex, comp, ptype))
    got = imageio.read_image(str(p))
    # ReadImageEXR reads through HALF slices: float channels round to half
    np.testing.assert_array_equal(got, tex.astype(np.float16).astype(np.float32))
    p.write_bytes(_exr_bytes(tex, comp, ptype, channels="GR"))  # a missing channel reads as 0
    got = imageio.read_image(str(p))
    assert np.all(got[..., 2] == 0) and np.array_equal(got[..., 0], tex[..., 0].astype(np.float16).astype(np.float32))


def test_imageio_pfm_and_tga(mpss, tmp_path):
    import struct
    from mpss import imageio
    tex = envmap_texels(9, 5)
    p = tmp_path / "a.pfm"
    with open(p, "wb") as f:  # big endian, scale 2, no flip
        f.write(b"PF\n9 5\n2.0\n" + np.ascontiguousarray(tex, ">f4").tobytes())
    np.testing.assert_array_equal(imageio.read_image(str(p)), tex * np.float32(2))
    g = tex[..., 1].copy()
    with open(p, "wb") as f:
        f.write(b"Pf\n9 5\n-1\n" + np.ascontiguousarray(g, "<f4").tobytes())
    np.testing.assert_array_equal(imageio.read_image(str(p)), np.repeat(g[..., None], 3, 2))
    rgb8 = (np.arange(5 * 9 * 3) % 256).astype(np.uint8).reshape(5, 9, 3)
    t = tmp_path / "a.tga"  # uncompressed BGR, origin bottom-left (descriptor 0)
    t.write_bytes(struct.pack("<BBBHHBHHHHBB", 0, 0, 2, 0, 0, 0, 0, 0, 9, 5, 24, 0) +
                  rgb8[..., ::-1].tobytes())
    got = imageio.read_image(str(t))
    # file rows are bottom-to-top; ReadImageTGA flips to top-to-bottom then walks y from the bottom
    np.testing.assert_array_equal(got, rgb8.astype(np.float32) / np.float32(255))


# ------------------------------------------------------------------ environment-map oracle
class _EnvMap:
    def __init__(self, tex):
        import ctypes as C
        lib = oracle_lib.lib()

        class M(C.Structure):
            _fields_ = [("tw", C.c_int), ("th", C.c_int), ("nu", C.c_int), ("nv", C.c_int)] + \
                       [(n, C.POINTER(C.c_float)) for n in ("tex", "func", "cdf", "rint", "mcdf")] + [("mint", C.c_float)]
        self.C, self.lib, self.m = C, lib, M()
        lib.o_envmap_build.argtypes = [C.c_int, C.c_int, oracle_lib.f32p, C.POINTER(M)]
        lib.o_envmap_sample.argtypes = [C.POINTER(M), C.c_float, C.c_float, oracle_lib.f32p, oracle_lib.f32p]
        lib.o_envmap_pdf.argtypes = [C.POINTER(M), C.c_float, C.c_float]
        lib.o_envmap_pdf.restype = C.c_float
        lib.o_envmap_lookup.argtypes = [C.POINTER(M), C.c_float, C.c_float, oracle_lib.f32p]
        lib.o_envmap_free.argtypes = [C.POINTER(M)]
        tex = np.ascontiguousarray(tex, np.float32)
        assert lib.o_envmap_build(tex.shape[1], tex.shape[0], tex, C.byref(self.m)) == 0

    def sample(self, u0, u1):
        uv, pdf = np.zeros(2, np.float32), np.zeros(1, np.float32)
        self.lib.o_envmap_sample(self.C.byref(self.m), u0, u1, uv, pdf)
        return uv, float(pdf[0])

    def pdf(self, u, v):
        return self.lib.o_envmap_pdf(self.C.byref(self.m), u, v)

    def lookup(self, s, t):
        out = np.zeros(3, np.float32)
        self.lib.o_envmap_lookup(self.C.byref(self.m), s, t, out)
        return out

    def close(self):
        self.lib.o_envmap_free(self.C.byref(self.m))


def test_oracle_envmap_distribution(mpss, oracle):
    """Distribution2D over img * sin(theta): the sampled uv's pdf equals Pdf(uv) away from cell
    edges; the marginal/conditional pdf integrates to 1; the level-0 map of a non-power-of-two
    image is its Lanczos resampling (a constant image stays constant)."""
    em = _EnvMap(envmap_texels(37, 21))
    m = em.m
    assert (m.tw, m.th, m.nu, m.nv) == (64, 32, 37, 21)
    rng = np.random.default_rng(1)
    for u0, u1 in rng.random((400, 2)).astype(np.float32):
        uv, p = em.sample(u0, u1)
        assert 0 <= uv[0] < 1 and 0 <= uv[1] < 1 and p > 0
        fu, fv = uv[0] * m.nu, uv[1] * m.nv
        if min(fu % 1, 1 - fu % 1, fv % 1, 1 - fv % 1) > 1e-3:
            assert em.pdf(uv[0], uv[1]) == pytest.approx(p, rel=1e-5)
    uu, vv = np.meshgrid((np.arange(m.nu) + .5) / m.nu, (np.arange(m.nv) + .5) / m.nv)
    total = sum(em.pdf(u, v) for u, v in zip(uu.ravel(), vv.ravel())) / (m.nu * m.nv)
    assert total == pytest.approx(1.0, rel=1e-5)
    em.close()
    c = np.full((19, 37, 3), [0.5, 0.25, 2.0], np.float32)
    em = _EnvMap(c)
    for s, t in rng.random((50, 2)).astype(np.float32):
        np.testing.assert_allclose(em.lookup(s, t), c[0, 0], rtol=2e-6)
    em.close()


def test_oracle_irradiance_under_env_map(mpss, oracle):
    """E on an unoccluded upward plane under a lat-long map = alb_mix * int over the upper
    hemisphere of Ft(cos) Le(w) cos dw; the expectation is a quadrature of the oracle's own
    level-0 lookups, so this pins Sample_L's uv -> direction map and pdf / (2 pi^2 sin theta)."""
    tex = envmap_texels(24, 12)
    tex[..., :] = tex[..., :] * 0 + (0.4 + 0.3 * np.cos(np.pi * (np.arange(12) + .5) / 12))[:, None, None]
    tex[:, 5:9] *= np.array([1.6, 1.2, 0.8], np.float32)
    li = _sky(ns=16)
    li["texels"] = tex
    sc = _plane_scene(mpss, li, half=1.0)
    cfg = mpss.default_config(min_sample_distance=0.02)
    tabs = orr.tables_from_host(sc, mpss)
    o = orr.OracleScene(sc, tabs, cfg, mpss)
    pts = o.tessellate()
    E = o.irradiance(pts, 3).astype(np.float64).mean(0)
    # quadrature: theta in (0, pi/2) (the map's z axis is the plane normal), phi in (0, 2 pi)
    rgbL = _to_rgb(oracle_lib.from_rgb(li["L"]) * oracle_lib.from_rgb(li["scale"]))
    em = _EnvMap(tex * rgbL)
    rho = tabs[0][2].astype(np.float64)
    nt, nphi = 256, 256
    acc = np.zeros(NB)
    for i in range(nt):
        th = (i + .5) / nt * (np.pi / 2)
        mu = np.cos(th)
        ft = 1 - np.interp(mu, np.linspace(0, 1, len(rho)), rho)
        for j in range(0, nphi, 4):
            ph = (j + .5) / nphi * 2 * np.pi
            le = oracle_lib.from_rgb(em.lookup(np.float32(ph / (2 * np.pi)), np.float32(th / np.pi)), illuminant=True)
            acc += ft * le * mu * np.sin(th) * (np.pi / 2 / nt) * (2 * np.pi / nphi * 4)
    em.close()
    np.testing.assert_allclose(E, acc, rtol=0.03)


def test_reads_reference_envmap(mpss):
    """The reference's own environment map (scenes/textures/grace_latlong.exr, an OpenEXR file
    written by OpenEXR, ZIP-compressed, copied to tests/golden/): ReadImageEXR's HALF slices
    (imageio.cpp:120-150) decoded by this package, rows top to bottom."""
    import hashlib
    from mpss import imageio
    tex = imageio.read_image(os.path.join(ROOT, "tests", "golden", "grace_latlong.exr"))
    assert tex.shape == (512, 1024, 3) and tex.dtype == np.float32
    assert np.all(np.isfinite(tex)) and tex.min() >= 0
    assert np.array_equal(tex.astype(np.float16).astype(np.float32), tex)  # HALF values
    assert float(tex.max()) == 18.375
    assert hashlib.sha256(tex.tobytes()).hexdigest()[:16] == "27123b8a7e761b7d"
