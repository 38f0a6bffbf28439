"""The benched C2 frame (scenes/skin.pbrt, 1024x1024, 64 spp, minsampledistance 0.0015, desiredlength
512: L = 119,766, 2.2 M irradiance points) rendered with the reference sampler replayed
(mpss_config.sampler = MPSS_SAMPLER_REFERENCE, replay_cores = 8) through the production sharded
Mo() gather, against the oracle, and against the benched hash-sampler frame.

  irradiance   IrradianceTask's RNG(47 k) streams (multipolesubsurface.cpp:72-152) for the whole
               2.2 M-point cloud, every point vs the oracle's: rel 1e-5, >= 99 % bit-identical
  windows      the cheek and silhouette windows of test_configs_gpu.py rendered by the GPU's replay
               (SamplerRendererTask::Run's per-task MT19937 streams, samplerrenderer.cpp:60-167;
               LDSampler, lowdiscrepancy.cpp:67-79) vs the oracle fed the same tasks' streams
               (o_replay_render_table_window): tests/parity.py's criterion, unfloored L-inf reported
  full frame   EVERY pixel of the frame in reference-sampler mode -- north_star's literal criterion,
               the output of pbrt's own sampler -- vs the oracle, generated and rendered in bands of
               rows so host memory stays bounded; the same criterion
The oracle side is its own end to end: its profile / rho tables, its replayed irradiance, its octree.
  exrdiff      the hash-sampler frame (what bench.py times) vs the replay frame, judged by pbrt's
               own exrdiff (src/tools/exrdiff.cpp:76-94; mpss.film.exrdiff) with a mean-delta
               tolerance of EXRDIFF_TOL_PCT percent (-d), plus a per-block convergence test
               (render sampler only: both frames on the same irradiance) -- the two samplers must
               converge to the same image.
"""
import os

import numpy as np
import pytest

import oracle_lib
import oracle_render as orr
import parity
from test_configs_gpu import _render, _windows

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NT = oracle_lib.nthreads()
EXRDIFF_TOL_PCT = 0.5   # exrdiff -d: |avg1 - avg2| / min(avg1, avg2) in percent
BLOCK = 32              # convergence blocks (pixels per side)


@pytest.fixture(scope="module")
def c2ref(mpss, oracle):
    import torch
    assert torch.cuda.is_available()
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin.pbrt"))
    assert (sc.xres, sc.yres, sc.spp) == (1024, 1024, 64)
    ctx = pbrtscene.build_context(sc, sampler=mpss.SAMPLER_REFERENCE, replay_cores=8)
    ctx.preprocess(seed=0)  # seeds are ignored by the replay sampler
    o = orr.OracleScene(sc, orr.tables_from_oracle(sc), ctx.cfg, mpss)
    pts = ctx.surface_points()
    o.E = o.irradiance_replay(pts, cores=8, nthreads=NT)
    o.set_octree(pts, o.E)
    return torch, sc, ctx, o


def test_c2_replay_irradiance(c2ref):
    torch, sc, ctx, o = c2ref
    pts = ctx.surface_points()
    assert len(pts) > 2_000_000
    E = o.E
    got = ctx.irradiance()
    assert got.shape == E.shape
    np.testing.assert_allclose(got, E, rtol=1e-5, atol=1e-6 * float(E.max()))
    assert (got == E).mean() >= 0.99


@pytest.mark.parametrize("where", ["cheek", "silhouette"])
def test_c2_replay_window_parity(c2ref, where):
    torch, sc, ctx, o = c2ref
    if where == "cheek":
        x0, x1, y0, y1 = _windows(ctx, sc.xres, sc.yres, 32, 32, lambda f: f == 1.0)
    else:
        x0, x1, y0, y1 = _windows(ctx, sc.xres, sc.yres, 37, 29, lambda f: 0.3 < f < 0.7)
    got = _render(torch, ctx, sc.spp, 0, x0, x1, y0, y1)
    win = o.replay_window(x0, x1, y0, y1)
    vals = o.replay_table_window(sc.spp, win, cores=8, li_draws=6, nthreads=NT)
    ref = o.render_tile_replay(sc.spp, vals, x0, x1, y0, y1, nthreads=NT, window=win)
    parity.check_image(got, ref, "c2_replay_window_%s" % where)
    assert (ref[..., 1] > 0).mean() > (0.9 if where == "cheek" else 0.2)


BAND = 64  # rows of the frame per oracle pass (the sample values of one band: ~0.4 GB)


def test_c2_replay_full_frame_parity(c2ref):
    """Every pixel of the C2 frame rendered with pbrt's own sampler replayed (8 cores' task split,
    4,096 render tasks) vs the oracle fed the same tasks' MT19937 streams, band by band: the
    north_star criterion (1e-4 relative L-inf, unfloored) on the whole output of the reference
    sampler."""
    torch, sc, ctx, o = c2ref
    got = _render(torch, ctx, sc.spp, 0, 0, sc.xres, 0, sc.yres)
    ref = np.zeros_like(got)
    for y0 in range(0, sc.yres, BAND):
        y1 = min(y0 + BAND, sc.yres)
        win = o.replay_window(0, sc.xres, y0, y1)
        vals = o.replay_table_window(sc.spp, win, cores=8, li_draws=6, nthreads=NT)
        ref[y0:y1] = o.render_tile_replay(sc.spp, vals, 0, sc.xres, y0, y1, nthreads=NT, window=win)
        del vals
    st = parity.check_image(got, ref, "c2_replay_full_frame")
    assert 0.03 < (ref[..., 1] > 0).mean() < 0.5
    print("C2 reference-sampler full frame: relative L-inf %.3g over %d values" % (st["rel_linf"], st["values"]))


def _frame(torch, ctx, sc, seed):
    return _render(torch, ctx, sc.spp, seed, 0, sc.xres, 0, sc.yres)


def _block_z(a, b, skin):
    """Per BLOCK x BLOCK block of skin pixels: z = mean(a - b) / (std(a - b) / sqrt(n)) over the
    block's pixel differences (the two renders' noise is independent per pixel, the signal cancels)."""
    H, W = skin.shape
    zs = []
    for y in range(0, H, BLOCK):
        for x in range(0, W, BLOCK):
            m = skin[y:y + BLOCK, x:x + BLOCK]
            if m.sum() < BLOCK * BLOCK // 2:
                continue
            d = (a[y:y + BLOCK, x:x + BLOCK] - b[y:y + BLOCK, x:x + BLOCK])[m].astype(np.float64)
            zs.append(d.mean() / (d.std(ddof=1) / np.sqrt(len(d))))
    return np.array(zs)


def test_c2_hash_frame_converges_to_reference_sampler_frame(mpss, c2ref):
    """The benched hash-sampler frame against the reference-sampler frame (exrdiff), and the render
    samplers alone (same irradiance) block by block."""
    from mpss import film, pbrtscene
    torch, sc, ctx, o = c2ref
    ref_img = _frame(torch, ctx, sc, 0)
    hctx = pbrtscene.build_context(sc)  # the benched configuration
    hctx.preprocess(seed=1)
    hash_img = _frame(torch, hctx, sc, 7)
    hctx.close()
    assert np.array_equal(ref_img[..., 3] > 0, hash_img[..., 3] > 0)
    rgb_ref, rgb_hash = film.finalize(ref_img), film.finalize(hash_img)
    rep = film.exrdiff(rgb_ref, rgb_hash, tol=EXRDIFF_TOL_PCT)
    # the render sampler alone: the hash sampler on the reference-sampler run's irradiance
    pts = ctx.surface_points()
    sctx = pbrtscene.build_context(sc)
    sctx.set_irradiance_points(pts["p"], pts["n"], ctx.irradiance(), pts["area"])
    same_e = film.finalize(_frame(torch, sctx, sc, 7))
    sctx.close()
    Y = lambda rgb: 0.212671 * rgb[..., 0] + 0.715160 * rgb[..., 1] + 0.072169 * rgb[..., 2]  # noqa: E731
    skin = Y(rgb_ref) > 0
    z = _block_z(Y(same_e), Y(rgb_ref), skin)
    z_pre = _block_z(Y(rgb_hash), Y(rgb_ref), skin)
    rep2 = film.exrdiff(rgb_ref, same_e, tol=EXRDIFF_TOL_PCT)
    parity.record("c2_hash_vs_reference_sampler", {
        "exrdiff": rep, "exrdiff_same_irradiance": rep2, "blocks": int(len(z)),
        "block_z_render_sampler": {"max_abs": float(np.abs(z).max()), "rms": float(np.sqrt((z ** 2).mean())),
                                   "mean": float(z.mean())},
        "block_z_full": {"max_abs": float(np.abs(z_pre).max()), "rms": float(np.sqrt((z_pre ** 2).mean())),
                         "mean": float(z_pre.mean())}})
    assert not rep["differ"], rep            # exrdiff -d 0.5 passes on the two full runs
    assert not rep2["differ"], rep2
    assert len(z) >= 20
    # render samplers alone: block means agree within the noise (z ~ N(0, 1): no block off by 6
    # sigma, and the spread is the noise's)
    assert np.abs(z).max() < 6.0, np.abs(z).max()
    assert 0.5 < np.sqrt((z ** 2).mean()) < 2.0
