"""Per-pixel path parity: libmpss on the GPU vs the CPU oracle (oracle/render.c) on the same
scene, sampler seeds and material tables.

  surface points (tessellation)   bit-exact (44-byte records compared as bytes)
  irradiance E                    rel 1e-5 per value, >= 99% of values bit-identical
                                  (transcendentals are double-evaluated on both sides; only
                                  double-rounding ties of OCML vs glibc can differ)
  film XYZW                       weights bit-exact; XYZ per pixel within north_star's 1e-4
                                  relative L-inf, |gpu - cpu| <= 1e-4 |cpu|, no floor
                                  (tests/parity.py; measured <= 8e-7). The GPU sums Mo() per band
                                  in one running sum (<= 2e-5 relative vs the reference recursion)
"""
import os

import numpy as np
import pytest

import oracle_render as orr
import parity

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOL = 1e-4


@pytest.fixture(scope="module")
def pair(mpss, oracle):
    import torch
    assert torch.cuda.is_available()
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin.pbrt"), xres=64, yres=64, spp=8)
    sc.integrator["minsampledistance"] = 0.008
    for m in sc.materials:
        m["desired_length"] = 128
    ctx = pbrtscene.build_context(sc)
    ctx.preprocess(seed=11)
    o = orr.OracleScene(sc, orr.tables_from_ctx(ctx, len(sc.materials)), ctx.cfg, mpss)
    return torch, sc, ctx, o


@pytest.mark.gpu
def test_surface_points_bit_exact(pair):
    torch, sc, ctx, o = pair
    got = ctx.surface_points()
    ref = o.tessellate()
    assert len(got) == len(ref)
    assert got.tobytes() == ref.tobytes()


@pytest.mark.gpu
def test_irradiance_parity(pair):
    torch, sc, ctx, o = pair
    pts = ctx.surface_points()
    got = ctx.irradiance()
    ref = o.irradiance(pts, 11)
    assert got.shape == ref.shape
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6 * float(ref.max()))
    assert (got == ref).mean() >= 0.99


def _render_gpu(torch, ctx, sc, x0, x1, y0, y1, seed):
    out = torch.zeros(((y1 - y0) * (x1 - x0) * 4,), dtype=torch.float32, device="cuda")
    ctx.render_tile(sc.spp, seed, x0, x1, y0, y1, out.data_ptr())
    torch.cuda.synchronize()
    return out.cpu().numpy().reshape(y1 - y0, x1 - x0, 4)


def _check(got, ref):
    """tests/parity.py's criterion: weights bit-exact, XYZ within 1e-4 relative L-inf (no floor)."""
    parity.check_image(got, ref)


@pytest.mark.gpu
def test_image_parity_full_frame(pair):
    torch, sc, ctx, o = pair
    pts = ctx.surface_points()
    o.set_octree(pts, o.irradiance(pts, 11))
    got = _render_gpu(torch, ctx, sc, 0, sc.xres, 0, sc.yres, 5)
    ref = o.render_tile(sc.spp, 5, 0, sc.xres, 0, sc.yres)
    _check(got, ref)
    assert (ref[..., 1] > 0).mean() > 0.05  # the test actually covers shaded pixels


@pytest.mark.gpu
def test_image_parity_ragged_tile(pair):
    """An interior tile whose borders cut through the face (edge samples of neighbours)."""
    torch, sc, ctx, o = pair
    pts = ctx.surface_points()
    o.set_octree(pts, o.irradiance(pts, 11))
    x0, x1, y0, y1 = 21, 45, 30, 57
    got = _render_gpu(torch, ctx, sc, x0, x1, y0, y1, 9)
    ref = o.render_tile(sc.spp, 9, x0, x1, y0, y1)
    _check(got, ref)


@pytest.mark.gpu
def test_c1_tissue_full_frame(mpss, oracle):
    """Config C1 (BASELINE.json configs[0]): scenes/tissue.pbrt at its full 256x256, 8 spp, the
    reference's CPU-runnable case -- the whole frame on the GPU against the CPU restatement."""
    import torch
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "tissue.pbrt"))
    assert (sc.xres, sc.yres, sc.spp) == (256, 256, 8)
    ctx = pbrtscene.build_context(sc)
    ctx.preprocess(seed=2)
    o = orr.OracleScene(sc, orr.tables_from_ctx(ctx, len(sc.materials)), ctx.cfg, mpss)
    pts = ctx.surface_points()
    assert pts.tobytes() == o.tessellate().tobytes()
    E = o.irradiance(pts, 2)
    np.testing.assert_allclose(ctx.irradiance(), E, rtol=1e-5, atol=1e-6 * float(E.max()))
    o.set_octree(pts, E)
    got = _render_gpu(torch, ctx, sc, 0, sc.xres, 0, sc.yres, 13)
    ref = o.render_tile(sc.spp, 13, 0, sc.xres, 0, sc.yres)
    _check(got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("scene,kt", [("skin.pbrt", None), ("tissue.pbrt", [0.6, 0.8, 1.0])])
def test_image_parity_transmission_lobe(mpss, oracle, scene, kt):
    """LayeredSkin with a non-black Kt (CreateLayeredSkinMaterial's default Spectrum(1), or a
    coloured one): the BSDF gains MicrofacetTransmission, so BSDF sampling picks a lobe with
    uComponent and the MIS pdfs average both lobes (reflection.cpp:675-751)."""
    import torch
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", scene), xres=48, yres=48, spp=4)
    sc.integrator["minsampledistance"] = 0.008
    for m in sc.materials:
        m["desired_length"] = 128
        if kt is None:
            m.pop("Kt", None)   # the default Spectrum(1)
        else:
            m["Kt"] = kt
    ctx = pbrtscene.build_context(sc)
    ctx.preprocess(seed=4)
    o = orr.OracleScene(sc, orr.tables_from_ctx(ctx, len(sc.materials)), ctx.cfg, mpss)
    pts = ctx.surface_points()
    o.set_octree(pts, o.irradiance(pts, 4))
    got = _render_gpu(torch, ctx, sc, 0, sc.xres, 0, sc.yres, 21)
    ref = o.render_tile(sc.spp, 21, 0, sc.xres, 0, sc.yres)
    _check(got, ref)


def _sky_light(deg, axis, L=(0.3, 0.35, 0.45), scale=(2, 2, 2), ns=4):
    from mpss import pbrtscene
    l2w = pbrtscene.rotate(deg, axis)
    return dict(kind="infinite", L=list(L), scale=list(scale), nsamples=ns, l2w=l2w.astype(np.float32),
                w2l=np.linalg.inv(l2w).astype(np.float32))


@pytest.mark.parametrize("scene,lights", [("tissue_sky.pbrt", None), ("skin.pbrt", "sky+area"),
                                          ("skin.pbrt", "sky"), ("tissue.pbrt", "map+area"), ("skin.pbrt", "map"),
                                          ("skin.pbrt", "grace")])
@pytest.mark.gpu
def test_image_parity_infinite_light(mpss, oracle, scene, lights):
    """LightSource "infinite" (lights/infinite.cpp), constant or with a radiance map: Sample_L /
    Pdf (Distribution2D) for irradiance and both MIS halves of EstimateDirect, Le (MIPMap
    lookups) for BSDF rays and camera rays that escape; alone, and mixed with the sphere light
    in either order."""
    import torch
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", scene), xres=48, yres=48, spp=4)
    sc.integrator["minsampledistance"] = 0.008
    for m in sc.materials:
        m["desired_length"] = 128
    if lights == "sky+area":
        sc.lights = [sc.lights[0], _sky_light(40, [1, 1, 0], ns=2)]
    elif lights == "sky":
        sc.lights = [_sky_light(-70, [0, 1, 1], L=(0.8, 0.6, 0.5), ns=8)]
    elif lights == "map+area":  # a non-power-of-two map (Lanczos-resampled MIPMap) with a sun
        from test_infinite_light import envmap_texels
        sky = _sky_light(100, [1, 0, 0], L=(1, 1, 1), scale=(3, 3, 3), ns=4)
        sky["texels"] = envmap_texels(37, 21, seed=3)
        sc.lights = [sc.lights[0], sky]
    elif lights == "map":
        from test_infinite_light import envmap_texels
        sky = _sky_light(-60, [0, 1, 0], L=(1, 1, 1), ns=4)
        sky["texels"] = envmap_texels(64, 32, seed=4)
        sc.lights = [sky]
    elif lights == "grace":  # the reference's own map (scenes/textures/grace_latlong.exr, 1024x512 ZIP)
        from mpss import imageio
        sky = _sky_light(-90, [1, 0, 0], L=(1, 1, 1), ns=4)
        sky["texels"] = imageio.read_exr(os.path.join(ROOT, "tests", "golden", "grace_latlong.exr"))
        sc.lights = [sc.lights[0], sky]
    ctx = pbrtscene.build_context(sc)
    ctx.preprocess(seed=6)
    o = orr.OracleScene(sc, orr.tables_from_ctx(ctx, len(sc.materials)), ctx.cfg, mpss)
    pts = ctx.surface_points()
    E = o.irradiance(pts, 6)
    got_E = ctx.irradiance()
    np.testing.assert_allclose(got_E, E, rtol=1e-5, atol=1e-6 * float(E.max()))
    assert (got_E == E).mean() >= 0.99
    o.set_octree(pts, E)
    got = _render_gpu(torch, ctx, sc, 0, sc.xres, 0, sc.yres, 17)
    ref = o.render_tile(sc.spp, 17, 0, sc.xres, 0, sc.yres)
    _check(got, ref)


def _visible_sphere_scene(pbrtscene):
    """skin.pbrt with a second sphere light in front of the face, in frame: its surface carries pbrt's
    default "matte" material (api.cpp:241,1085), so a camera ray that hits it returns Le(wo) plus the
    direct light the matte surface receives from the scene's other lights (multipolesubsurface.cpp:
    253-304); it also shadows and lights the face."""
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin.pbrt"), xres=48, yres=48, spp=4)
    sc.integrator["minsampledistance"] = 0.008
    for m in sc.materials:
        m["desired_length"] = 128
    front = dict(center=[0.53, -2.53, 0.51], radius=0.12, L=[6.0, 5.0, 4.0], nsamples=2)
    sc.lights = [sc.lights[0], front, _sky_light(40, [1, 1, 0], ns=2)]
    return sc


@pytest.mark.gpu
def test_image_parity_light_sphere_in_frame(mpss, oracle):
    import torch
    from mpss import pbrtscene
    sc = _visible_sphere_scene(pbrtscene)
    ctx = pbrtscene.build_context(sc)
    ctx.preprocess(seed=8)
    o = orr.OracleScene(sc, orr.tables_from_ctx(ctx, len(sc.materials)), ctx.cfg, mpss)
    pts = ctx.surface_points()
    o.set_octree(pts, o.irradiance(pts, 8))
    got = _render_gpu(torch, ctx, sc, 0, sc.xres, 0, sc.yres, 23)
    ref = o.render_tile(sc.spp, 23, 0, sc.xres, 0, sc.yres)
    _check(got, ref)
    assert _sphere_pixels(sc, sc.lights[1]).sum() >= 20  # the case covers the sphere


def _sphere_pixels(sc, li):
    """Pixels whose centre ray meets the sphere (the camera's own matrices; test bookkeeping only)."""
    r2c, c2w = (m.astype(np.float64) for m in sc.raster_to_camera())
    ys, xs = np.mgrid[0:sc.yres, 0:sc.xres] + 0.5
    pc = np.stack([xs, ys, np.zeros_like(xs), np.ones_like(xs)], -1) @ r2c.T
    dc = pc[..., :3] / pc[..., 3:]
    d = dc @ c2w[:3, :3].T
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    oc = c2w[:3, 3] - np.asarray(li["center"], np.float64)
    b = d @ oc
    return b * b - (oc @ oc - li["radius"] ** 2) > 0


def test_light_sphere_matte_shading_oracle(oracle):
    """The oracle's light-sphere shading (CPU only): with the scene's other lights on, the pixels
    whose centre ray meets the front sphere gain its matte surface's direct light on top of Le."""
    import mpss
    from mpss import pbrtscene
    ys = []
    for others in (True, False):
        sc = _visible_sphere_scene(pbrtscene)
        sc.xres = sc.yres = 24
        sc.materials[0]["desired_length"] = 64
        if not others:
            sc.lights = [sc.lights[1]]
        o = orr.OracleScene(sc, orr.tables_from_host(sc, mpss), mpss.default_config(
            **pbrtscene.integrator_config(sc)), mpss)
        ys.append(o.render_tile(sc.spp, 3, 0, sc.xres, 0, sc.yres)[..., 1])
    px = _sphere_pixels(sc, sc.lights[0])
    assert px.sum() >= 5
    assert np.all(ys[0][px] > ys[1][px])
