"""Per-pixel path on the GPU (camera rays, BVH, direct lighting, Mo gather, film) -- properties
that hold independently of the oracle: determinism, tile-decomposition invariance (the sampler
is a per-pixel counter-based hash and the film sums each pixel's samples in a fixed order, so
any tiling gives bit-identical pixels), physical sanity and Preprocess products.
Oracle parity of the same path lives in test_render_parity_gpu.py."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch


@pytest.fixture(scope="module")
def small_skin(torch_dev, mpss):
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin.pbrt"), xres=96, yres=96, spp=4)
    # coarser tessellation keeps the test fast (quick-render style)
    sc.integrator["minsampledistance"] = 0.01
    ctx = pbrtscene.build_context(sc)
    ctx.preprocess(seed=1)
    return sc, ctx


def render(torch, ctx, sc, x0, x1, y0, y1, spp, seed=3):
    out = torch.zeros(((y1 - y0) * (x1 - x0) * 4,), dtype=torch.float32, device="cuda")
    ctx.render_tile(spp, seed, x0, x1, y0, y1, out.data_ptr())
    torch.cuda.synchronize()
    return out.cpu().numpy().reshape(y1 - y0, x1 - x0, 4)


def test_preprocess_products(small_skin):
    sc, ctx = small_skin
    pts = ctx.surface_points()
    E = ctx.irradiance()
    assert len(pts) > 1000 and E.shape == (len(pts), 30)
    assert np.all(np.isfinite(E)) and np.all(E >= 0)
    assert (E.sum(1) > 0).mean() > 0.2      # the lit side of the head
    assert (E.sum(1) == 0).mean() > 0.05    # and the side facing away from the light
    assert np.all(pts["area"] > 0)
    info = ctx.octree_info()
    assert info["n_points"] == len(pts)


def test_render_deterministic_and_sane(torch_dev, small_skin):
    sc, ctx = small_skin
    a = render(torch_dev, ctx, sc, 0, sc.xres, 0, sc.yres, sc.spp)
    b = render(torch_dev, ctx, sc, 0, sc.xres, 0, sc.yres, sc.spp)
    assert np.array_equal(a, b)
    assert np.all(np.isfinite(a))
    w = a[..., 3]
    # every pixel gets its own spp samples (+ edge samples of neighbours landing on u==0/v==0)
    assert np.all(w >= sc.spp)
    Y = a[..., 1] / w
    assert Y.max() > 0 and (Y > 0).mean() > 0.05
    assert (Y == 0).mean() > 0.2  # background: rays that miss everything


def test_tile_invariance(torch_dev, small_skin):
    sc, ctx = small_skin
    full = render(torch_dev, ctx, sc, 0, sc.xres, 0, sc.yres, sc.spp)
    T = 40  # does not divide 96: ragged tiles on the right and bottom
    tiled = np.zeros_like(full)
    for y0 in range(0, sc.yres, T):
        for x0 in range(0, sc.xres, T):
            x1, y1 = min(x0 + T, sc.xres), min(y0 + T, sc.yres)
            tiled[y0:y1, x0:x1] = render(torch_dev, ctx, sc, x0, x1, y0, y1, sc.spp)
    assert np.array_equal(full, tiled)


def test_render_stats(torch_dev, small_skin):
    sc, ctx = small_skin
    ctx.set_instrumentation(kernel_timing=True, count_traversal=True)
    ctx.reset_render_stats()
    render(torch_dev, ctx, sc, 0, sc.xres, 0, sc.yres, sc.spp)
    st = ctx.render_stats()
    ctx.set_instrumentation(False, False)
    assert st["n_camera"] >= 1 and st["n_shade"] == st["n_camera"] and st["ms_shade"] > 0
    assert st["samples"] >= sc.xres * sc.yres * sc.spp
    assert 0 < st["sss_samples"] < st["samples"]
    assert st["mo_nodes"] > st["sss_samples"]


def test_bad_arguments(torch_dev, small_skin, mpss):
    sc, ctx = small_skin
    out = torch_dev.zeros(16, device="cuda")
    with pytest.raises(mpss.MpssError):
        ctx.render_tile(4, 0, 0, sc.xres + 1, 0, 1, out.data_ptr())
    with pytest.raises(mpss.MpssError):
        ctx.render_tile(0, 0, 0, 1, 0, 1, out.data_ptr())


@pytest.mark.parametrize("max_batch", [1 << 16, 1 << 24])
def test_render_tiles_batching_invariance(torch_dev, small_skin, mpss, max_batch):
    """mpss_render_tiles (several tiles, one Mo() launch per batch; a tiny batch limit forces row
    pieces and many batches) gives the same bits as per-tile mpss_render_tile calls."""
    from mpss import pbrtscene
    sc, ctx = small_skin
    ref = render(torch_dev, ctx, sc, 0, sc.xres, 0, sc.yres, sc.spp)
    ctx2 = pbrtscene.build_context(sc, max_batch_samples=max_batch)
    ctx2.set_surface_points(ctx.surface_points())
    ctx2.preprocess(seed=1)
    rects = [(0, 50, 0, 37), (50, 96, 0, 37), (0, 96, 37, 96)]
    outs = [torch_dev.zeros(((r[1] - r[0]) * (r[3] - r[2]) * 4,), device="cuda") for r in rects]
    ctx2.render_tiles(sc.spp, 3, rects, [o.data_ptr() for o in outs])
    torch_dev.cuda.synchronize()
    got = np.zeros_like(ref)
    for r, o in zip(rects, outs):
        got[r[2]:r[3], r[0]:r[1]] = o.cpu().numpy().reshape(r[3] - r[2], r[1] - r[0], 4)
    assert np.array_equal(got, ref)
