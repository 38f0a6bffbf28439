"""LayeredSkin with image textures on the GPU vs the CPU oracle: an "albedo" imagemap
(Pow(albedo, mix) per irradiance point from its (u, v); Pow(albedo, 1 - mix) per camera hit with
EWA filtering over the camera ray differentials) and a "bumpmap" (the bumped shading frame for
the BSDF and Ft, and bumped SurfacePoint normals). Tolerances as test_render_parity_gpu.py:
tessellation bit-exact, irradiance rel 1e-5, film 1e-4 relative per pixel (floor 1e-3 of peak)."""
import os

import numpy as np
import pytest

import oracle_render as orr
import synth
from test_render_parity_gpu import _check, _render_gpu

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

ALBEDO = dict(texels=synth.texture_texels(93, 61, seed=7), wrap="clamp", gamma=2.2, scale=2.0)  # S007's map params
BUMP = dict(texels=synth.texture_texels(64, 48, seed=8), is_float=True, shift=-0.5, scale=0.02)


@pytest.mark.parametrize("scene,alb,bump,spp", [("skin.pbrt", True, False, 8), ("skin.pbrt", False, True, 4),
                                                ("skin.pbrt", True, True, 4), ("tissue.pbrt", True, True, 4)])
def test_textured_skin_parity(mpss, oracle, scene, alb, bump, spp):
    import torch
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", scene), xres=48, yres=48, spp=spp)
    sc.integrator["minsampledistance"] = 0.008 if scene == "skin.pbrt" else sc.integrator["minsampledistance"]
    for m in sc.materials:
        m["desired_length"] = 128
        if alb:
            m["albedo_tex"] = ALBEDO
        if bump:
            m["bump_tex"] = BUMP
    ctx = pbrtscene.build_context(sc)
    ctx.preprocess(seed=3)
    o = orr.OracleScene(sc, orr.tables_from_ctx(ctx, len(sc.materials)), ctx.cfg, mpss)
    pts = ctx.surface_points()
    assert pts.tobytes() == o.tessellate().tobytes()
    E = o.irradiance(pts, 3)
    got_E = ctx.irradiance()
    np.testing.assert_allclose(got_E, E, rtol=1e-5, atol=1e-6 * float(E.max()))
    assert (got_E == E).mean() >= 0.99
    o.set_octree(pts, E)
    got = _render_gpu(torch, ctx, sc, 0, sc.xres, 0, sc.yres, 23)
    ref = o.render_tile(sc.spp, 23, 0, sc.xres, 0, sc.yres)
    _check(got, ref)
    o.close()
    ctx.close()


def test_texture_changes_the_image(mpss, oracle):
    """The albedo texture is really applied: the textured render differs from the untextured one
    and the irradiance is the untextured irradiance times Pow(FromRGB(texel), mix) band by band
    (checked at the points, where the lookup is bilinear at level 0)."""
    import torch
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin.pbrt"), xres=32, yres=32, spp=4)
    sc.integrator["minsampledistance"] = 0.01
    for m in sc.materials:
        m["desired_length"] = 128
    ctx0 = pbrtscene.build_context(sc)
    ctx0.preprocess(seed=1)
    E0 = ctx0.irradiance()
    img0 = _render_gpu(torch, ctx0, sc, 0, 32, 0, 32, 2)
    for m in sc.materials:
        m["albedo_tex"] = ALBEDO
    ctx1 = pbrtscene.build_context(sc)
    ctx1.preprocess(seed=1)
    pts = ctx1.surface_points()
    E1 = ctx1.irradiance()
    img1 = _render_gpu(torch, ctx1, sc, 0, 32, 0, 32, 2)
    uvd = np.zeros((len(pts), 6), np.float32)
    uvd[:, 0], uvd[:, 1] = pts["u"], pts["v"]
    rgb = mpss.host_imagemap_lookup(ALBEDO, uvd)
    alb = np.stack([mpss.host_from_rgb(c) for c in rgb[:2000]])
    want = (E0[:2000].astype(np.float64) * np.power(alb.astype(np.float64), 0.5)).astype(np.float32)
    np.testing.assert_allclose(E1[:2000], want, rtol=2e-6, atol=1e-30)
    assert np.abs(img1[..., 1] - img0[..., 1]).max() > 1e-3 * np.abs(img0[..., 1]).max()
    ctx0.close()
    ctx1.close()


def test_textured_c2_window_parity(mpss, oracle):
    """scenes/skin_textured.pbrt at the benched C2 parameters (1024x1024, 64 spp, desiredlength 512,
    minsampledistance 0.0015): imagemap albedo (gamma 2.2, scale 2, clamp) and bumpmap on the head,
    a 32x32 cheek window through the production path (the common-grid gather, the textured assemble
    fast path) vs the oracle with its own tables, irradiance and octree; the tessellation with the
    bumped normals bit-exact."""
    import torch
    import oracle_lib
    from mpss import pbrtscene
    from test_configs_gpu import _windows
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin_textured.pbrt"))
    assert (sc.xres, sc.spp) == (1024, 64)
    m = sc.materials[0]
    assert m["albedo_tex"]["texels"] is not None and m["bump_tex"]["texels"] is not None
    ctx = pbrtscene.build_context(sc)
    ctx.preprocess(seed=1)
    assert ctx.gather_info(0)["common_grid"]  # the production gather: far lookups from the common grid
    o = orr.OracleScene(sc, orr.tables_from_oracle(sc), ctx.cfg, mpss)
    pts = ctx.surface_points()
    assert pts.tobytes() == o.tessellate().tobytes()
    E = o.irradiance(pts, 1, nthreads=oracle_lib.nthreads())  # the oracle's own irradiance and octree
    np.testing.assert_allclose(ctx.irradiance(), E, rtol=1e-5, atol=1e-6 * float(E.max()))
    o.set_octree(pts, E)
    x0, x1, y0, y1 = _windows(ctx, sc.xres, sc.yres, 32, 32, lambda f: f == 1.0)
    got = _render_gpu(torch, ctx, sc, x0, x1, y0, y1, 7)
    ref = o.render_tile(sc.spp, 7, x0, x1, y0, y1, nthreads=oracle_lib.nthreads())
    _check(got, ref)
    assert (ref[..., 1] > 0).all()
    o.close()
    ctx.close()
