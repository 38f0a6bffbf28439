"""LayeredSkin's profile switches on the GPU against the oracle (CreateLayeredSkinMaterial,
layeredskin.cpp:246-255; the constructor's branches at :70-122):

  genprofile false        preparedBSSRDFData = NULL: no Mo() term on the material's surfaces, and its
                          irradiance points lit as points without a MultipoleBSSRDF (Ft = 1, no
                          albedo^mix; multipolesubsurface.cpp:100-107,139-140). Alone, and beside a
                          profiled material whose Mo() gathers those points' irradiance
  showirradiancepoints    the material's profile is ComputeIrradiancePointsProfile(irradiancepointsize)
                          (multipole.cpp:551-567: a disc of 1 / (pi r^2) per band) and its rho table
                          ComputeRoughRhoData (:569-572: zeros, Ft = 1)

Each renders a small skin.pbrt frame through the production path and the oracle (its own tables:
tables_from_oracle, its own irradiance and octree); tests/parity.py's criterion.

genprofile false is parity unpinned: the reference would dereference its NULL MultipoleBSSRDFData
(layeredskin.cpp:184, multipole.cpp rho()/albedo()), so the meaning above is this package's and the
oracle's, and these tests check the two restatements against each other.
"""
import os

import numpy as np
import pytest

import oracle_render as orr
import parity

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _scene(**mat):
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin.pbrt"), xres=64, yres=64, spp=8)
    sc.integrator["minsampledistance"] = 0.008
    for m in sc.materials:
        m["desired_length"] = 128
        m.update(mat)
    return sc


def _split_two_materials(sc, second):
    """The head's triangles dealt alternately to the scene's material and a copy of it with `second`
    applied (two meshes over the same vertices)."""
    me = sc.meshes[0]
    m2 = dict(sc.materials[0])
    m2.update(second)
    sc.materials.append(m2)
    a, b = dict(me), dict(me)
    a["indices"] = me["indices"][0::2]
    b["indices"] = me["indices"][1::2]
    b["material"] = 1
    sc.meshes = [a, b]
    return sc


def _pair_render(mpss, sc, seed=5):
    import torch
    from mpss import pbrtscene
    ctx = pbrtscene.build_context(sc)
    ctx.preprocess(seed=seed)
    o = orr.OracleScene(sc, orr.tables_from_oracle(sc), ctx.cfg, mpss)
    pts = ctx.surface_points()
    assert pts.tobytes() == o.tessellate().tobytes()
    E = o.irradiance(pts, seed)
    got_E = ctx.irradiance()
    np.testing.assert_allclose(got_E, E, rtol=1e-5, atol=1e-6 * float(E.max()))
    o.set_octree(pts, E)
    out = torch.zeros((sc.yres * sc.xres * 4,), dtype=torch.float32, device="cuda")
    ctx.render_tile(sc.spp, 9, 0, sc.xres, 0, sc.yres, out.data_ptr())
    torch.cuda.synchronize()
    got = out.cpu().numpy().reshape(sc.yres, sc.xres, 4)
    ref = o.render_tile(sc.spp, 9, 0, sc.xres, 0, sc.yres)
    return ctx, o, got, ref, pts, E


def test_genprofile_false_has_no_subsurface_term(mpss, oracle):
    sc = _scene(gen_profile=0)
    ctx, o, got, ref, pts, E = _pair_render(mpss, sc)
    parity.check_image(got, ref, "genprofile_false")
    assert (ref[..., 1] > 0).mean() > 0.03  # the surface BSDF's direct light remains (the head: ~5 % of the frame)
    # no Mo() term: the same frame with the profile is brighter wherever skin is lit
    ctx1, o1, got1, ref1, _, _ = _pair_render(mpss, _scene())
    skin = ref1[..., 1] > 0
    assert np.all(got1[..., 1][skin] >= got[..., 1][skin] * (1 - 1e-6))
    assert (got1[..., 1] > got[..., 1] * 1.01).mean() > 0.02
    # no profile to gather with
    import torch
    q = torch.zeros((1, 3), dtype=torch.float32, device="cuda")
    out = torch.zeros((1, 30), dtype=torch.float32, device="cuda")
    with pytest.raises(mpss.MpssError, match="genprofile"):
        ctx.mo_batch(0, 1, q.data_ptr(), out.data_ptr())
    for c in (ctx, ctx1, o, o1):
        c.close()


def test_genprofile_false_beside_a_profiled_material(mpss, oracle):
    """Half the head's triangles carry a genprofile-false copy of the material (its albedo 0.25, which
    its points must ignore): the profiled half's Mo() gathers both halves' points."""
    sc = _split_two_materials(_scene(), dict(gen_profile=0, albedo=[0.25, 0.25, 0.25]))
    ctx, o, got, ref, pts, E = _pair_render(mpss, sc)
    parity.check_image(got, ref, "genprofile_false_beside_profiled")
    assert set(np.unique(pts["material"])) == {0, 1}
    ctx.close()
    o.close()


@pytest.mark.parametrize("size", [0.002, 0.02])
def test_material_showirradiancepoints(mpss, oracle, size):
    sc = _scene(show_irradiance_points=1, irradiance_point_size=size)
    ctx, o, got, ref, pts, E = _pair_render(mpss, sc)
    tab, rcp, rho, _ = ctx.material_tables(0)
    otab, orcp, orho = orr.irradiance_points_tables(size)
    assert tab.shape == (30, 2) and np.array_equal(tab, otab) and np.array_equal(rcp, orcp)
    assert np.array_equal(rho, orho)
    parity.check_image(got, ref, "material_showirradiancepoints_%g" % size)
    assert (ref[..., 1] > 0).mean() > 0.03
    ctx.close()
    o.close()


def test_poisson_finder_keeps_genprofile_false_surfaces(mpss, oracle):
    """FindPoissonPointDistribution picks candidates by GetBSSRDF != NULL (surfacepoints.cpp:202), which a
    LayeredSkin always returns (layeredskin.cpp:170-177) -- genprofile false included. With half the head
    genprofile false, the Poisson points cover both halves, equal to the oracle's (o_poisson_points)."""
    sc = _split_two_materials(_scene(), dict(gen_profile=0))
    sc.integrator["usepoissonpointfinder"] = "true"
    sc.integrator["minsampledistance"] = 0.02
    from mpss import pbrtscene
    ctx = pbrtscene.build_context(sc)
    ctx.preprocess(seed=5)
    got = ctx.surface_points()
    o = orr.OracleScene(sc, orr.tables_from_oracle(sc), ctx.cfg, mpss)
    ref = o.poisson_points(5)
    assert len(got) == len(ref) and len(got) > 100
    assert set(np.unique(got["material"])) == {0, 1}
    assert np.array_equal(got["p"], ref["p"])
    for k in ("u", "v", "material", "area", "ray_eps"):
        assert np.array_equal(got[k], ref[k]), k
    ctx.close()
    o.close()
