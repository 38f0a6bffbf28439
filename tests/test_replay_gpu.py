"""The reference sampler replayed on the GPU (mpss_config.sampler = MPSS_SAMPLER_REFERENCE; row a16)
against the oracle's restatement of the same loop (oracle/render.c o_replay_*, itself checked
against a pure-Python restatement in test_sampler_replay.py).

  sample table     bit-exact: every task's MT19937 stream, LDPixelSample scrambles and shuffles,
                   and the 6 Li draws per camera hit (the GPU's hit tests are the render kernels'
                   own BVH traversal, bit-identical to the oracle's)
  irradiance       IrradianceTask's RNG(47 k) scrambles: rel 1e-5, >= 99 % bit-identical (as the
                   hash-sampler irradiance parity)
  film             render parity tolerance (test_render_parity_gpu._check); any tiling renders
                   the same film bit for bit, and another emulated core count another film
"""
import os

import numpy as np
import pytest

import oracle_render as orr

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _scene(name, lights=None, W=40, H=32, spp=4):
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", name), xres=W, yres=H, spp=spp)
    sc.integrator["minsampledistance"] = 0.008
    for m in sc.materials:
        m["desired_length"] = 64
    if lights == "sky+area":
        from test_render_parity_gpu import _sky_light
        sc.lights = [sc.lights[0], _sky_light(40, [1, 1, 0], ns=2)]
    elif lights == "24 spheres":
        # 3 x 24 = 72 light-sample arrays per pixel: more than one wave's 63 shuffle lanes
        # (replay_gen.hip strides the arrays' block shuffles over the lanes)
        sc.lights = []
        for k in range(24):
            a = 2 * np.pi * k / 24
            sc.lights.append(dict(center=np.array([5 * np.cos(a), -4 + 2 * np.sin(a), 3 + 0.1 * k], np.float32),
                                  radius=0.1, L=[40.0 + k, 40.0, 40.0 - k], nsamples=1 + k % 3))
    elif lights == "edge geometry":
        # the camera-ray candidate lists' edge cases (scene.h CameraBins): a strip crossing the camera
        # plane (from behind the camera to in front of it: tested by every pixel), a wall behind the head
        # larger than kCamBinMaxArea pixels (also every pixel), a triangle entirely behind the camera and
        # one off the frame (in no list)
        def tri_mesh(P, idx):
            P = np.asarray(P, np.float32)
            o2w = np.eye(4, dtype=np.float32)
            return dict(P=P, N=None, S=None, uv=None, indices=np.asarray(idx, np.int32).reshape(-1, 3),
                        o2w=o2w, w2o=o2w, reverse=False, material=0)
        sc.meshes.append(tri_mesh([[-0.3, -7.0, -0.45], [0.3, -7.0, -0.45], [0.0, 2.0, -0.45]], [0, 1, 2]))
        sc.meshes.append(tri_mesh([[-1.6, 1.5, -1.0], [1.6, 1.5, -1.0], [1.6, 1.5, 1.6], [-1.6, 1.5, 1.6]],
                                  [0, 1, 2, 0, 2, 3]))
        sc.meshes.append(tri_mesh([[0.0, -8.0, 1.0], [0.3, -8.0, 1.2], [0.0, -8.2, 1.3]], [0, 1, 2]))
        sc.meshes.append(tri_mesh([[6.0, 0.0, 0.0], [6.3, 0.0, 0.2], [6.0, 0.2, 0.3]], [0, 1, 2]))
        # an axis-aligned quad (a zero-thickness box: the slab test's most fragile case) whose edges lie
        # inside the frame, between the camera and the head, so its edges and diagonal cut through pixel
        # samples (the candidate lists and the oracle both take a hit iff some triangle is met)
        sc.meshes.append(tri_mesh([[-0.22, -0.9, 0.05], [0.18, -0.9, 0.05], [0.18, -0.9, 0.41], [-0.22, -0.9, 0.41]],
                                  [0, 1, 2, 0, 2, 3]))
        sc.integrator["minsampledistance"] = 0.05
    elif lights and lights.startswith("ns="):
        # the light's sample count (rounded up to a power of 2 by LDShuffleScrambled): the generator
        # keeps each sample's own shuffle in registers up to 8 values, in LDS past that
        sc.lights[0]["nsamples"] = int(lights[3:])
    return sc


def _pair(mpss, sc, cores=8):
    import torch
    assert torch.cuda.is_available()
    from mpss import pbrtscene
    ctx = pbrtscene.build_context(sc, sampler=mpss.SAMPLER_REFERENCE, replay_cores=cores)
    ctx.preprocess(seed=0)
    o = orr.OracleScene(sc, orr.tables_from_ctx(ctx, len(sc.materials)), ctx.cfg, mpss)
    return torch, ctx, o


def _render_many(torch, ctx, sc, rects):
    """All rectangles in ONE render_tiles call (mpss_render_tiles: batches, one replay window each)."""
    outs = [torch.zeros(((y1 - y0) * (x1 - x0) * 4,), dtype=torch.float32, device="cuda") for x0, x1, y0, y1 in rects]
    ctx.render_tiles(sc.spp, 0, rects, [o.data_ptr() for o in outs])
    torch.cuda.synchronize()
    img = np.zeros((sc.yres, sc.xres, 4), np.float32)
    for (x0, x1, y0, y1), o in zip(rects, outs):
        img[y0:y1, x0:x1] = o.cpu().numpy().reshape(y1 - y0, x1 - x0, 4)
    return img


def _render(torch, ctx, sc, rects):
    img = np.zeros((sc.yres, sc.xres, 4), np.float32)
    for (x0, x1, y0, y1) in rects:
        out = torch.zeros(((y1 - y0) * (x1 - x0) * 4,), dtype=torch.float32, device="cuda")
        ctx.render_tile(sc.spp, 0, x0, x1, y0, y1, out.data_ptr())
        torch.cuda.synchronize()
        img[y0:y1, x0:x1] = out.cpu().numpy().reshape(y1 - y0, x1 - x0, 4)
    return img


@pytest.mark.parametrize("name,lights,cores", [("skin.pbrt", None, 8), ("skin.pbrt", "sky+area", 8),
                                               ("tissue.pbrt", None, 2), ("skin.pbrt", "24 spheres", 8),
                                               ("skin.pbrt", "ns=5", 8), ("skin.pbrt", "ns=16", 8),
                                               ("skin.pbrt", "edge geometry", 8)])
def test_replay_table_bit_exact(mpss, oracle, name, lights, cores):
    sc = _scene(name, lights, W=128, H=96) if lights == "edge geometry" else _scene(name, lights)
    torch, ctx, o = _pair(mpss, sc, cores)
    got = ctx.replay_samples(sc.spp, sc.xres, sc.yres)
    ref = o.replay_table(sc.spp, cores=cores, li_draws=6)
    assert got.shape == ref.shape
    bad = np.argwhere(np.any(got != ref, axis=(2, 3)))
    assert len(bad) == 0, "first differing pixels (y, x): %s" % bad[:5].tolist()
    ctx.close()


@pytest.mark.parametrize("name,lights", [("skin.pbrt", None), ("skin.pbrt", "sky+area")])
def test_replay_irradiance_and_image(mpss, oracle, name, lights):
    from test_render_parity_gpu import _check
    sc = _scene(name, lights)
    torch, ctx, o = _pair(mpss, sc)
    pts = ctx.surface_points()
    E = o.irradiance_replay(pts, cores=8)
    got_E = ctx.irradiance()
    np.testing.assert_allclose(got_E, E, rtol=1e-5, atol=1e-6 * float(E.max()))
    assert (got_E == E).mean() >= 0.99
    o.set_octree(pts, E)
    vals = o.replay_table(sc.spp, cores=8, li_draws=6)
    ref = o.render_tile_replay(sc.spp, vals, 0, sc.xres, 0, sc.yres)
    full = _render(torch, ctx, sc, [(0, sc.xres, 0, sc.yres)])
    _check(full, ref)
    tiles = [(x, min(x + 13, sc.xres), y, min(y + 11, sc.yres)) for y in range(0, sc.yres, 11)
             for x in range(0, sc.xres, 13)]
    assert np.array_equal(_render(torch, ctx, sc, tiles), full)
    # tiles behind the task cursors (reverse and shuffled order: each such task restarts from
    # RNG(task)), and all tiles in one call split into many batches (one window per batch)
    assert np.array_equal(_render(torch, ctx, sc, tiles[::-1]), full)
    rng = np.random.default_rng(3)
    assert np.array_equal(_render(torch, ctx, sc, [tiles[i] for i in rng.permutation(len(tiles))]), full)
    ctx.close()
    from mpss import pbrtscene
    ctx2 = pbrtscene.build_context(sc, sampler=mpss.SAMPLER_REFERENCE, replay_cores=8, max_batch_samples=1 << 10)
    ctx2.set_irradiance_points(pts["p"], pts["n"], got_E, pts["area"])
    ctx2.set_instrumentation(kernel_timing=True)
    assert np.array_equal(_render_many(torch, ctx2, sc, tiles), full)
    st = ctx2.render_stats()
    assert st["n_camera"] > 1 and st["n_replay"] >= 1  # many batches (one window may serve several)
    ctx2.close()


def test_replay_depends_on_core_count_and_not_on_seed(mpss):
    import torch
    from mpss import pbrtscene
    sc = _scene("skin.pbrt")
    imgs = []
    for cores in (8, 8, 16):
        ctx = pbrtscene.build_context(sc, sampler=mpss.SAMPLER_REFERENCE, replay_cores=cores)
        ctx.preprocess(seed=len(imgs))  # seeds are ignored by the replay sampler
        out = torch.zeros((sc.yres * sc.xres * 4,), dtype=torch.float32, device="cuda")
        ctx.render_tile(sc.spp, 77 * len(imgs), 0, sc.xres, 0, sc.yres, out.data_ptr())
        torch.cuda.synchronize()
        imgs.append(out.cpu().numpy())
        ctx.close()
    assert np.array_equal(imgs[0], imgs[1])
    assert not np.array_equal(imgs[0], imgs[2])


def test_replay_lds_limit_is_named(mpss):
    """The generator keeps a pixel's draws, index arrays and shuffles of one pbrt task in one wave's
    LDS: a pixel-sample count past that budget is refused up front, with the constraint named."""
    import torch
    from mpss import pbrtscene
    sc = _scene("skin.pbrt", spp=4096)
    ctx = pbrtscene.build_context(sc, sampler=mpss.SAMPLER_REFERENCE, replay_cores=8)
    ctx.preprocess(seed=0)
    out = torch.zeros((4 * 4 * 4,), dtype=torch.float32, device="cuda")
    with pytest.raises(mpss.MpssError, match="KB"):
        ctx.render_tile(4096, 0, 0, 4, 0, 4, out.data_ptr())
    ctx.render_tile(1024, 0, 0, 4, 0, 4, out.data_ptr())  # 1024 spp x 4 light samples fits
    torch.cuda.synchronize()
    assert float(out.cpu()[3]) > 0
    ctx.close()
