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


def test_loader_rejects_env_maps(mpss, tmp_path):
    from mpss import pbrtscene
    f = tmp_path / "m.pbrt"
    f.write_text('WorldBegin\nLightSource "infinite" "string mapname" "sky.exr"\nWorldEnd\n')
    with pytest.raises(ValueError, match="mapname"):
        pbrtscene.load(str(f))


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
