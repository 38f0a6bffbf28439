"""BASELINE.json's configurations at their benched parameters, on the GPU, against the oracle.

  C2  scenes/skin.pbrt exactly as bench.py runs it (1024x1024, 64 spp, minsampledistance 0.0015,
      desiredlength 512, the production sharded Mo() gather): surface points bit-exact, the GPU
      profile and rho tables vs the oracle, irradiance of ALL 2.2 M points vs the oracle's, and two
      windows rendered by both: a 32x32 window on the cheek and a ragged 37x29 window across
      the silhouette, with the image tolerance of test_render_parity_gpu.py; and the WHOLE benched
      frame (1024x1024 x 64 spp, every pixel) against the oracle on the host's CPUs. The oracle side
      is end to end its own: its profile and rho tables (tables_from_oracle), its irradiance and
      its octree built from that irradiance.
  C3  2048x2048 at 256 spp: a cheek window and a silhouette window at the config's own 256 spp vs
      the oracle; dealt over 8 ranks by cost (bench.py's multi-GPU deal), every rank's tile set
      rendered on this GPU and reassembled is bitwise the single-call frame.
  C4  scenes/mcprofile.pbrt's layers at 1e7 photons vs the oracle's random walk.
  C5  the 4.06 M-triangle subdivided head with the original tessellation as pointsfile: surface
      irradiance of every point and a 32x32 cheek window at the config's own 512 spp against the oracle
      (at 512 spp a wave's 64 lanes are one pixel's samples: the gather's lane-coherent regime).
"""
import os

import numpy as np
import pytest

import oracle_lib
import parity
import oracle_mc
import oracle_render as orr

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOL = 1e-4
NT = oracle_lib.nthreads()


def _render(torch, ctx, spp, seed, x0, x1, y0, y1):
    out = torch.zeros(((y1 - y0) * (x1 - x0) * 4,), dtype=torch.float32, device="cuda")
    ctx.render_tile(spp, seed, x0, x1, y0, y1, out.data_ptr())
    torch.cuda.synchronize()
    return out.cpu().numpy().reshape(y1 - y0, x1 - x0, 4)


def _check(got, ref):
    """tests/parity.py's criterion: weights bit-exact, XYZ within 1e-4 relative L-inf (no floor)."""
    parity.check_image(got, ref)


def _windows(ctx, W, H, w, h, want):
    """The w x h window (on a w x h grid) nearest the frame centre whose fraction of pixel-centre
    rays hitting skin satisfies want(fraction)."""
    rects = [(x, x + w, y, y + h) for y in range(0, H - h + 1, h) for x in range(0, W - w + 1, w)]
    sss, _ = ctx.tile_costs(rects)
    cand = [(abs((r[0] + r[1]) / 2 - W / 2) + abs((r[2] + r[3]) / 2 - H / 2), r)
            for r, n in zip(rects, sss) if want(n / float(w * h))]
    assert cand, "no window matches"
    return min(cand)[1]


@pytest.fixture(scope="module")
def c2(mpss, oracle):
    import torch
    assert torch.cuda.is_available()
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin.pbrt"))
    assert (sc.xres, sc.yres, sc.spp) == (1024, 1024, 64)
    assert float(sc.integrator["minsampledistance"]) == pytest.approx(0.0015)
    ctx = pbrtscene.build_context(sc)  # desiredlength 512 (CreateLayeredSkinMaterial's default)
    ctx.preprocess(seed=1)
    # the oracle's own tables, irradiance and octree: nothing of the product's feeds its images
    o = orr.OracleScene(sc, orr.tables_from_oracle(sc), ctx.cfg, mpss)
    o.E = o.irradiance(ctx.surface_points(), 1, nthreads=NT)
    o.set_octree(ctx.surface_points(), o.E)
    return torch, sc, ctx, o


def test_c2_tables_at_desired_length_512(c2, oracle):
    """a12/a13 at the benched material: the GPU-built profile (lerponthinslab on) vs the kissfft
    oracle, and the rho_hd table, bit-exact."""
    torch, sc, ctx, o = c2
    tab, rcp, rho, tot = ctx.material_tables(0)
    m = sc.materials[0]
    mua, musp, th, eta = oracle.skin_layers(m["roughness"], m["nmperunit"], m["f_mel"], m["f_eu"], m["f_blood"],
                                            m["f_ohg"], tuple(m["layer_thickness_nm"]), tuple(m["layer_ior"]))
    tab_o, rcp_o, _, tot_o = oracle.compute_profile(mua, musp, eta, th, desired_length=512, lerp=True)
    assert tab.shape == tab_o.shape and tab.shape[1] > 100000
    assert np.array_equal(rcp, rcp_o)
    peak = np.abs(tab_o).max(axis=1, keepdims=True)
    assert np.all(np.abs(tab - tab_o) <= 1e-6 * peak)
    np.testing.assert_allclose(tot, tot_o, rtol=1e-5)
    hd_o, _ = oracle.rho_table(m["roughness"], m["layer_ior"][0])
    assert np.array_equal(rho, hd_o)


def test_c2_surface_points_and_irradiance(c2):
    torch, sc, ctx, o = c2
    pts = ctx.surface_points()
    assert len(pts) > 2_000_000
    assert pts.tobytes() == o.tessellate().tobytes()
    E = o.E  # every point (the fixture's oracle irradiance, from which the oracle's octree is built)
    got = ctx.irradiance()
    assert got.shape == E.shape == (len(pts), 30)
    np.testing.assert_allclose(got, E, rtol=1e-5, atol=1e-6 * float(E.max()))
    assert (got == E).mean() >= 0.99


@pytest.mark.parametrize("where", ["cheek", "silhouette"])
def test_c2_window_parity(c2, where):
    """A window of the benched frame through the production gather (exact_mo = 0) vs the oracle
    (its own tables, irradiance and octree)."""
    torch, sc, ctx, o = c2
    if where == "cheek":
        x0, x1, y0, y1 = _windows(ctx, sc.xres, sc.yres, 32, 32, lambda f: f == 1.0)
    else:
        x0, x1, y0, y1 = _windows(ctx, sc.xres, sc.yres, 37, 29, lambda f: 0.3 < f < 0.7)
    got = _render(torch, ctx, sc.spp, 7, x0, x1, y0, y1)
    ref = o.render_tile(sc.spp, 7, x0, x1, y0, y1, nthreads=NT)
    _check(got, ref)
    assert (ref[..., 1] > 0).mean() > (0.9 if where == "cheek" else 0.2)


def test_c2_full_frame_parity(c2):
    """Every pixel of the benched C2 frame (skin.pbrt 1024x1024, 64 spp, hash sampler, production
    sharded gather) vs the oracle's render of the same frame (multipolesubsurface.cpp:253-304 driven
    by samplerrenderer.cpp:60-167's pixel loop), with tests/parity.py's unfloored 1e-4 relative L-inf.
    The oracle renders from its own profile / rho tables, its own irradiance of all 2.2 M points
    and its own octree: the comparison is end to end."""
    torch, sc, ctx, o = c2
    got = _render(torch, ctx, sc.spp, 7, 0, sc.xres, 0, sc.yres)
    ref = o.render_tile(sc.spp, 7, 0, sc.xres, 0, sc.yres, nthreads=NT)
    st = parity.check_image(got, ref)
    assert 0.03 < (ref[..., 1] > 0).mean() < 0.5  # the head covers ~5 % of the frame, lit background none
    print("C2 full frame: relative L-inf %.3g over %d values" % (st["rel_linf"], st["values"]))


@pytest.fixture(scope="module")
def c3(mpss):
    import torch
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin.pbrt"), xres=2048, yres=2048, spp=256)
    ctx = pbrtscene.build_context(sc)
    ctx.preprocess(seed=1)
    o = orr.OracleScene(sc, orr.tables_from_oracle(sc), ctx.cfg, mpss)
    pts = ctx.surface_points()
    E = o.irradiance(pts, 1, nthreads=NT)
    np.testing.assert_allclose(ctx.irradiance(), E, rtol=1e-5, atol=1e-6 * float(E.max()))
    o.set_octree(pts, E)
    yield torch, sc, ctx, o
    ctx.close()


@pytest.mark.parametrize("where", ["cheek", "silhouette"])
def test_c3_window_parity_256spp(c3, where):
    """C3 at its own 2048x2048 x 256 spp: windows of the frame through the production gather vs the oracle."""
    torch, sc, ctx, o = c3
    assert sc.spp == 256
    if where == "cheek":
        x0, x1, y0, y1 = _windows(ctx, sc.xres, sc.yres, 32, 32, lambda f: f == 1.0)
    else:
        x0, x1, y0, y1 = _windows(ctx, sc.xres, sc.yres, 37, 29, lambda f: 0.3 < f < 0.7)
    got = _render(torch, ctx, sc.spp, 11, x0, x1, y0, y1)
    ref = o.render_tile(sc.spp, 11, x0, x1, y0, y1, nthreads=NT)
    _check(got, ref)
    assert (ref[..., 1] > 0).mean() > (0.9 if where == "cheek" else 0.2)


def test_c3_rank_tiles_reassemble_bitwise(mpss):
    """C3 (2048x2048, 256 spp, 8 ranks): bench.py's cost-balanced deal of 64x64 tiles; each rank's
    tile set rendered separately and reassembled equals one render of the whole frame."""
    import torch
    from mpss import pbrtscene
    from mpss import tiles as tl
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin.pbrt"), xres=2048, yres=2048, spp=256)
    ctx = pbrtscene.build_context(sc)
    ctx.preprocess(seed=1)
    T, world = 64, 8
    tiles = tl.tile_grid(sc.xres, sc.yres, T)
    sss, surf = ctx.tile_costs(tiles)
    px = np.array([(x1 - x0) * (y1 - y0) for x0, x1, y0, y1 in tiles])
    deal = tl.deal_balanced(tl.tile_cost_model(sss, surf, px), world)
    skin = np.asarray(sss) > 0
    per_rank = [int(skin[d].sum()) for d in deal]
    assert max(per_rank) - min(per_rank) <= 1 and min(per_rank) > 0, per_rank
    full = _render(torch, ctx, sc.spp, 11, 0, sc.xres, 0, sc.yres)
    img = np.zeros((1, sc.yres, sc.xres, 4), np.float32)
    bufs, items = [], []
    for d in deal:
        out = torch.zeros((len(d), T * T * 4), dtype=torch.float32, device="cuda")
        tl.render_items(ctx, [(0, t) for t in d], tiles, sc.spp, [11], out, T)
        torch.cuda.synchronize()
        bufs.append(out.cpu().numpy())
        items.append([(0, t) for t in d])
    tl.assemble(img, bufs, items, tiles, T)
    assert np.array_equal(img[0], full)
    assert (full[..., 1] > 0).mean() > 0.03  # the head covers ~5 % of the frame
    ctx.close()


def test_c4_mcprofile_1e7_photons(mpss):
    """C4: scenes/mcprofile.pbrt's layers, 1e7 photons, GPU vs the oracle's walk (identical photon
    streams; statistical bounds as test_mc_gpu.py: totals 4 sigma, 16 coarse rings 5 sigma)."""
    import torch
    assert torch.cuda.is_available()
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "mcprofile.pbrt"))
    _, ps = sc.renderer
    lay = ps.find("layers")
    layers = [tuple(lay[4 * i:4 * i + 4]) for i in range(len(lay) // 4)]
    mfpr, nseg, n = float(ps.one("mfprange", 16.0)), int(ps.one("segments", 1024)), 10_000_000
    ctx = mpss.Context()
    g = ctx.mc_profile(layers, mfpr, nseg, n, seed=89)
    c = oracle_mc.mc_profile(layers, mfp_range=mfpr, nsegments=nseg, nphotons=n, seed=89, nthreads=NT)
    for k in ("total_r", "total_t"):
        p = max(c[k], 1.0 / n)
        sigma = np.sqrt(p * (1 - min(p, 0.999)) / n)
        assert abs(g[k] - c[k]) <= 4 * sigma + 1e-12, (k, g[k], c[k])
    i = np.arange(nseg, dtype=np.float64)
    ext = c["extent"]
    area = np.pi * ((2 * i + 1) * ext / nseg) * (ext / nseg)
    gr = (g["reflectance"] * area).reshape(16, -1).sum(1)
    cr = (c["reflectance"] * area).reshape(16, -1).sum(1)
    sig = np.sqrt(np.maximum(cr, 1.0 / n) / n)
    assert np.all(np.abs(gr - cr) <= 5 * sig), np.abs(gr - cr) / sig
    assert 0.0 < g["total_r"] < 1.0
    ctx.close()


def test_c5_dense_mesh_window(mpss):
    """C5's geometry (head.pbrt subdivided four times: 4.06 M triangles) with the original mesh's
    2.2 M tessellated points as the pointsfile, at 4096x4096 and the config's 512 spp: irradiance of
    every point and a 32x32 cheek window against the oracle (its own BVH over the same 4.06 M
    triangles, its own tables, irradiance and octree)."""
    import torch
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin.pbrt"), xres=4096, yres=4096, spp=512)
    pts = pbrtscene.mesh_points(sc)
    sc.meshes = [pbrtscene.subdivide_mesh(me, 4) for me in sc.meshes]
    assert sum(len(me["indices"]) for me in sc.meshes) > 4_000_000
    ctx = pbrtscene.build_context(sc)
    ctx.set_surface_points(pts)
    ctx.preprocess(seed=3)
    o = orr.OracleScene(sc, orr.tables_from_oracle(sc), ctx.cfg, mpss)
    E = o.irradiance(pts, 3, nthreads=NT)  # every point, over the oracle's own 4.06 M-triangle BVH
    got = ctx.irradiance()
    np.testing.assert_allclose(got, E, rtol=1e-5, atol=1e-6 * float(E.max()))
    assert (got == E).mean() >= 0.99
    o.set_octree(pts, E)
    x0, x1, y0, y1 = _windows(ctx, sc.xres, sc.yres, 32, 32, lambda f: f == 1.0)
    _check(_render(torch, ctx, sc.spp, 5, x0, x1, y0, y1), o.render_tile(sc.spp, 5, x0, x1, y0, y1, nthreads=NT))
    ctx.close()


def test_c5_replay_window(mpss):
    """C5 (4096x4096, 512 spp, 4.06 M triangles) with pbrt's own sampler replayed
    (MPSS_SAMPLER_REFERENCE, 8 emulated cores: 65,536 render tasks of 16x16 pixels): a 32x32 cheek
    window against the oracle fed the same tasks' MT19937 streams. The GPU generates only the
    window's tasks (replay_gen.hip; a whole-frame table would be (4097^2) x 512 x 22 floats)."""
    import torch
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin.pbrt"), xres=4096, yres=4096, spp=512)
    pts = pbrtscene.mesh_points(sc)
    sc.meshes = [pbrtscene.subdivide_mesh(me, 4) for me in sc.meshes]
    ctx = pbrtscene.build_context(sc, sampler=mpss.SAMPLER_REFERENCE, replay_cores=8)
    ctx.set_surface_points(pts)
    ctx.preprocess(seed=0)
    o = orr.OracleScene(sc, orr.tables_from_ctx(ctx, len(sc.materials)), ctx.cfg, mpss)
    o.set_octree(pts, ctx.irradiance())
    x0, x1, y0, y1 = _windows(ctx, sc.xres, sc.yres, 32, 32, lambda f: f == 1.0)
    ctx.set_instrumentation(kernel_timing=True)
    got = _render(torch, ctx, sc.spp, 0, x0, x1, y0, y1)
    win = o.replay_window(x0, x1, y0, y1)
    vals = o.replay_table_window(sc.spp, win, cores=8, li_draws=6, nthreads=NT)
    ref = o.render_tile_replay(sc.spp, vals, x0, x1, y0, y1, nthreads=NT, window=win)
    parity.check_image(got, ref, "c5_replay_window_512spp")
    assert (ref[..., 1] > 0).all()
    assert ctx.render_stats()["n_replay"] >= 1
    ctx.close()

