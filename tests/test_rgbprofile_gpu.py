"""rgbprofile LayeredSkin on the GPU (ComputeRGBMultipoleProfile, multipole.cpp:408-451; Rd =
FromRGB of three lookups, :85-107) against the oracle:

  profile tables     rows c % 3 = the R, G, B profiles of the layers' ToRGBSpectrum mua / musp,
                     GPU build vs the oracle's kissfft build within 1e-6 of each row's peak
  Mo()               the reference-order gather with the RGB functor, bit-exact vs the oracle
                     on the same octree, queries and tables
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


def test_rgb_mo_bit_exact(mpss):
    import torch
    ctx = mpss.Context()
    mid = ctx.add_layeredskin(mpss.default_skin(rgb_profile=1, desired_length=64, **SKIN))
    tab, rcp, _, _ = ctx.material_tables(mid)
    p, n, E, area = synth.ellipsoid_cloud(30000, seed=51, black_frac=0.05)
    p = p * np.float32(0.02)  # a patch a few profile reaches across
    ctx.set_irradiance_points(p, n, E, area)
    q = synth.surface_queries(2048, seed=52) * np.float32(0.02)
    qd = torch.from_numpy(np.ascontiguousarray(q, np.float32)).cuda()
    out = torch.zeros((len(q), NB), dtype=torch.float32, device="cuda")
    ctx.mo_batch(mid, len(q), qd.data_ptr(), out.data_ptr())
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    ref = oracle_lib.Octree(p, n, E, area).mo_rgb(q, tab, rcp, ctx.cfg.max_error)
    assert (ref > 0).mean() > 0.5
    assert np.array_equal(got, ref)


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
