"""rgbprofile LayeredSkin on the GPU (ComputeRGBMultipoleProfile, multipole.cpp:408-451; Rd =
FromRGB of three lookups, :85-107) against the oracle:

  profile tables     rows c % 3 = the R, G, B profiles of the layers' ToRGBSpectrum mua / musp,
                     GPU build vs the oracle's kissfft build within 1e-6 of each row's peak
  Mo()               the reference-order gather with the RGB functor (exact_mo 1) bit-exact vs the
                     oracle on the same octree, queries and tables; the default sharded gather
                     (three lookups per record, FromRGB into each band group's four bands) within
                     2e-5 of it, as the spectral sharded gather
  image              skin.pbrt window with rgbprofile on: film weights bit-exact, XYZ at 1e-4
"""
import os

import numpy as np
import pytest

import oracle_lib
import oracle_render as orr
import synth
from test_render_parity_gpu import _check, _render_gpu
from test_rgbprofile import rgb_layers

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NB = 30
SKIN = dict(roughness=0.3, nmperunit=40e6, f_mel=0.5, f_eu=0.5, f_blood=0.5, f_ohg=0.5,
            layer_thickness_nm=(0.25e6, 20e6), layer_ior=(1.4, 1.4))


@pytest.mark.parametrize("desired", [64, 512])
def test_rgb_profile_tables(mpss, desired):
    ctx = mpss.Context()
    mid = ctx.add_layeredskin(mpss.default_skin(rgb_profile=1, desired_length=desired, **SKIN))
    tab, rcp, rho, _ = ctx.material_tables(mid)
    mua, musp, th, eta = oracle_lib.skin_layers(0.3, 40e6, 0.5, 0.5, 0.5, 0.5, (0.25e6, 20e6), (1.4, 1.4))
    ra, rs = rgb_layers(mua, musp)
    otab, orcp, _, _ = oracle_lib.compute_profile(ra, rs, eta, th, desired_length=desired)
    assert tab.shape == otab.shape
    for c in range(NB):
        assert np.array_equal(tab[c], tab[c % 3])
    np.testing.assert_array_equal(rcp, orcp)
    for k in range(3):
        np.testing.assert_allclose(tab[k], otab[k], rtol=0, atol=1e-6 * float(np.abs(otab[k]).max()))


def _rgb_patch_mo(mpss, desired=64, **cfg):
    import torch
    ctx = mpss.Context(**cfg)
    mid = ctx.add_layeredskin(mpss.default_skin(rgb_profile=1, desired_length=desired, **SKIN))
    tab, rcp, _, _ = ctx.material_tables(mid)
    p, n, E, area = synth.ellipsoid_cloud(30000, seed=51, black_frac=0.05)
    p = p * np.float32(0.02)  # a patch a few profile reaches across
    ctx.set_irradiance_points(p, n, E, area)
    q = synth.surface_queries(2048, seed=52) * np.float32(0.02)
    qd = torch.from_numpy(np.ascontiguousarray(q, np.float32)).cuda()
    out = torch.zeros((len(q), NB), dtype=torch.float32, device="cuda")
    cnt = torch.zeros((len(q), 4), dtype=torch.int32, device="cuda")
    ctx.mo_batch(mid, len(q), qd.data_ptr(), out.data_ptr(), cnt.data_ptr())
    torch.cuda.synchronize()
    return ctx, mid, (p, n, E, area), q, tab, rcp, out.cpu().numpy(), cnt.cpu().numpy()


@pytest.mark.parametrize("exact_mo,common_grid", [(1, 0), (0, 0), (0, 1)])
def test_rgb_mo_vs_oracle(mpss, exact_mo, common_grid):
    # (the grid needs a table longer than the LDS near field: desiredlength 512, as C2)
    desired = 512 if common_grid else 64
    ctx, mid, (p, n, E, area), q, tab, rcp, got, cnt = _rgb_patch_mo(mpss, desired, exact_mo=exact_mo,
                                                                    mo_common_grid=common_grid)
    info = ctx.gather_info(mid)
    assert info["common_grid"] == (exact_mo == 0 and common_grid == 1)
    max_error = ctx.cfg.max_error
    ref = oracle_lib.Octree(p, n, E, area).mo_rgb(q, tab, rcp, max_error)
    assert (ref > 0).mean() > 0.5
    if exact_mo:
        assert np.array_equal(got, ref)
    elif not common_grid:
        # the same non-negative terms, summed in one running sum per band instead of the recursion's
        # order: both sums are within (n - 1) u of the exact one (n terms, u = 2^-24), so they differ
        # by at most 2 n u relative. n: the records the query visited, summed over the 8 band groups (the
        # counters; an upper bound of any one band's terms). This dense patch gives the longest sums of
        # any test, so the bound is stated rather than the 2e-5 of the smaller spectral cases
        n = (cnt[:, 2] + cnt[:, 3]).astype(np.float64)[:, None]
        tol = 2.0 * n * 2.0 ** -24
        assert np.all(np.abs(got - ref) <= tol * np.abs(ref) + 1e-30), (np.abs(got - ref) / (tol * np.abs(ref) + 1e-30)).max()
        # and typically far inside it (rounding errors of a long sum mostly cancel): the median error is
        # under a tenth of the worst case (round 4 on MI355X: median rel 9.3e-6 on sums of thousands of terms)
        frac = np.abs(got - ref) / (tol * np.abs(ref) + 1e-30)
        assert np.median(frac[ref > 0]) < 0.1, (np.median(frac[ref > 0]), np.median(n))
        assert np.array_equal(got == 0, ref == 0)
    else:
        # the common grid of the three profiles: the same traversal and order as the sharded gather
        # without it (its counters equal), each far R, G, B lookup off by <= 2e-6 of the largest of the
        # three at that distance, or 1e-14 of its peak (gather_info; build_common_grid's rgb scale; a bad
        # cell's lanes read the exact tables). FromRGB's output is .94 (W min + X (mid - min) + Y (max -
        # mid)), weights <= 1.1, so each term's error is <= 6 x that, and max(R, G, B) <= R + G + B:
        # unfloored, per query and band, |got - band| <= 6 (2e-6 S_c + 1e-14 peak mass_c) + the fused
        # FMAs' few ulp of |band|, S_c = sum over the records of (R + G + B)(d2) E_c area -- the reference
        # traversal with each profile in every band (the records do not depend on the table)
        assert info["rel_err"][:3].max() <= 2e-6 and info["rel_err"][:3].max() > 0
        ctx.close()
        ctx0, _, _, _, _, _, band, cnt0 = _rgb_patch_mo(mpss, desired, exact_mo=0, mo_common_grid=0)
        ctx0.close()
        assert np.array_equal(cnt, cnt0)
        assert not np.array_equal(got, band)
        oc = oracle_lib.Octree(p, n, E, area)
        S = sum(oc.mo(q, np.ascontiguousarray(np.repeat(tab[k:k + 1], 30, 0)), np.full(30, rcp[k], np.float32),
                      max_error).astype(np.float64) for k in range(3))
        mass = (E.astype(np.float64) * area.astype(np.float64)[:, None]).sum(axis=0)[None, :]
        bound = 6 * (2e-6 * S + 1e-14 * np.abs(tab[:3]).max() * mass) + 8 * 2.0 ** -24 * np.abs(band)
        err = np.abs(got.astype(np.float64) - band)
        assert np.all(err <= bound), (err / bound).max()
        assert np.array_equal(got == 0, ref == 0)
        return
    ctx.close()


def test_rgb_image_parity(mpss, oracle):
    import torch
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin.pbrt"), xres=48, yres=48, spp=4)
    sc.integrator["minsampledistance"] = 0.008
    for m in sc.materials:
        m["desired_length"] = 128
        m["rgb_profile"] = 1
    ctx = pbrtscene.build_context(sc)
    ctx.preprocess(seed=4)
    o = orr.OracleScene(sc, orr.tables_from_ctx(ctx, len(sc.materials)), ctx.cfg, mpss)
    pts = ctx.surface_points()
    o.set_octree(pts, o.irradiance(pts, 4))
    got = _render_gpu(torch, ctx, sc, 0, sc.xres, 0, sc.yres, 6)
    ref = o.render_tile(sc.spp, 6, 0, sc.xres, 0, sc.yres)
    _check(got, ref)
    assert (ref[..., 1] > 0).mean() > 0.05


def test_rgb_c2_window_parity(mpss, oracle):
    """rgbprofile on at the benched C2 parameters (skin.pbrt 1024x1024, 64 spp, desiredlength 512):
    a 32x32 cheek window through the sharded RGB gather vs the oracle."""
    import torch
    from mpss import pbrtscene
    from test_configs_gpu import _windows
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin.pbrt"))
    for m in sc.materials:
        m["rgb_profile"] = 1
    ctx = pbrtscene.build_context(sc)
    ctx.preprocess(seed=1)
    o = orr.OracleScene(sc, orr.tables_from_ctx(ctx, len(sc.materials)), ctx.cfg, mpss)
    o.set_octree(ctx.surface_points(), ctx.irradiance())
    x0, x1, y0, y1 = _windows(ctx, sc.xres, sc.yres, 32, 32, lambda f: f == 1.0)
    got = _render_gpu(torch, ctx, sc, x0, x1, y0, y1, 7)
    ref = o.render_tile(sc.spp, 7, x0, x1, y0, y1, nthreads=oracle_lib.nthreads())
    _check(got, ref)
    assert (ref[..., 1] > 0).all()
    ctx.close()
