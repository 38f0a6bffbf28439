"""FindPoissonPointDistribution ("usepoissonpointfinder", renderers/surfacepoints.cpp:115-284):
random-walk paths from the camera deposit candidate SurfacePoints on BSSRDF surfaces from the
fourth ray on; a candidate is kept unless a kept point lies within minSampleDistance; the
search stops after maxFails (2000, --quick 200) rejections in a row.

CPU: the oracle's restatement against the properties the reference guarantees (Poisson-disk
spacing, points on the surfaces, area pi (minDist/2)^2, unit normals, determinism).
GPU: libmpss (paths traced on the device, acceptance on the host) against the oracle, point by
point. Both follow ONE SurfacePointTask and replay-mode random numbers (the reference runs one
task per core and its point set depends on their interleaving): parity unpinned against
reference output, which would need the reference built and run.
"""
import os

import numpy as np
import pytest

import oracle_render as orr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _scene(mpss, md=0.02, quick=False):
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "tissue.pbrt"))
    sc.integrator["minsampledistance"] = md
    sc.integrator["usepoissonpointfinder"] = "true"
    cfg = mpss.default_config(**pbrtscene.integrator_config(sc, quick_render=int(quick)))
    return sc, cfg


def test_integrator_flag(mpss):
    sc, cfg = _scene(mpss)
    assert cfg.use_poisson_point_finder == 1


@pytest.mark.parametrize("quick", [False, True])
def test_oracle_poisson_properties(mpss, oracle, quick):
    from scipy.spatial import cKDTree
    sc, cfg = _scene(mpss, quick=quick)
    o = orr.OracleScene(sc, orr.tables_from_host(sc, mpss), cfg, mpss)
    md = o.min_dist
    pts = o.poisson_points(3)
    assert len(pts) > (300 if not quick else 20)
    p = pts["p"].astype(np.float64)
    # Poisson-disk: no two kept points closer than minDist (PoissonCheck, DistanceSquared < md^2)
    assert len(cKDTree(p).query_pairs(md * (1 - 1e-6))) == 0
    # on the slab (z = 0, |x|, |y| <= 0.6) or on the block's faces
    on_slab = (np.abs(p[:, 2]) < 1e-5) & (np.abs(p[:, 0]) <= 0.6 + 1e-5) & (np.abs(p[:, 1]) <= 0.6 + 1e-5)
    in_block = (p[:, 0] > -0.05 - 1e-5) & (p[:, 0] < 0.25 + 1e-5) & (np.abs(p[:, 1]) < 0.15 + 1e-5) & \
               (p[:, 2] > -1e-5) & (p[:, 2] < 0.2 + 1e-5)
    assert np.all(on_slab | in_block)
    assert np.all(pts["area"] == np.float32(np.pi) * (np.float32(md) / 2) * (np.float32(md) / 2))
    np.testing.assert_allclose(np.linalg.norm(pts["n"], axis=1), 1, atol=1e-6)
    assert np.all(pts["ray_eps"] > 0) and np.all(pts["material"] == 0)
    # both sides of the one-sided slab collect points: normals face the arriving ray
    nz = pts["n"][on_slab & ~in_block, 2]
    assert (nz > 0.99).any() and (nz < -0.99).any()
    again = o.poisson_points(3)
    assert again.tobytes() == pts.tobytes()
    other = o.poisson_points(4)
    assert other.tobytes() != pts.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("scene,md,bump", [("tissue.pbrt", 0.02, False), ("skin.pbrt", 0.02, False),
                                           ("skin.pbrt", 0.02, True)])
def test_poisson_points_gpu_vs_oracle(mpss, oracle, scene, md, bump):
    """bump: a "bumpmap" float imagemap -- candidates carry Bump(hitGeometry, dgShading).nn
    (surfacepoints.cpp:203-211)."""
    import torch
    import synth
    from mpss import pbrtscene
    assert torch.cuda.is_available()
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", scene), xres=32, yres=32, spp=1)
    sc.integrator["minsampledistance"] = md
    sc.integrator["usepoissonpointfinder"] = "true"
    for m in sc.materials:
        m["desired_length"] = 64
        if bump:
            m["bump_tex"] = dict(texels=synth.texture_texels(40, 30, seed=12), is_float=True, scale=0.05)
    ctx = pbrtscene.build_context(sc)
    ctx.preprocess(seed=5)
    got = ctx.surface_points()
    o = orr.OracleScene(sc, orr.tables_from_ctx(ctx, len(sc.materials)), ctx.cfg, mpss)
    ref = o.poisson_points(5)
    assert len(got) == len(ref) and len(got) > 200
    assert np.array_equal(got["p"], ref["p"])
    np.testing.assert_allclose(got["n"], ref["n"], atol=1e-6)
    for k in ("u", "v", "material", "area", "ray_eps"):
        assert np.array_equal(got[k], ref[k]), k
    # the render path runs on the found points (Preprocess -> irradiance -> octree)
    assert ctx.octree_info()["n_points"] == len(got)
    E = ctx.irradiance()
    np.testing.assert_allclose(E, o.irradiance(got, 5), rtol=1e-5, atol=1e-6 * float(E.max()))
