"""Preprocess's point set built on the GPU (render.hip tess_kernel, one thread per triangle) against
the host build (scene.cpp, tessellate_on_host = 1): the same SurfacePoint records byte for byte,
in the same order (TriangleMesh::TessellateSurfacePoints, trianglemesh.cpp:187-351, per mesh and
triangle in order). The host build is itself bit-exact against the oracle (test_render_parity_gpu,
test_texture_gpu compare the product's points with oracle_render's tessellation)."""
import os

import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUMP = dict(texels=synth.texture_texels(64, 48, seed=8), is_float=True, shift=-0.5, scale=0.02)


def _points(scene, on_host, incenter=0, min_dist=None, bump=False):
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", scene), xres=32, yres=32, spp=1)
    if min_dist is not None:
        sc.integrator["minsampledistance"] = min_dist
    for m in sc.materials:
        m["desired_length"] = 64
        if bump:
            m["bump_tex"] = BUMP
    ctx = pbrtscene.build_context(sc, tessellate_on_host=on_host, incenter=incenter)
    ctx.preprocess(seed=1)
    pts = ctx.surface_points()
    ctx.close()
    return pts


@pytest.mark.parametrize("scene,incenter,min_dist,bump", [("skin.pbrt", 0, None, False),  # C2: 2.2 M points
                                                          ("skin.pbrt", 1, 0.004, False),
                                                          ("skin.pbrt", 0, 0.004, True),
                                                          ("tissue.pbrt", 0, None, False)])
def test_gpu_tessellation_equals_host(mpss, scene, incenter, min_dist, bump):
    gpu = _points(scene, 0, incenter, min_dist, bump)
    host = _points(scene, 1, incenter, min_dist, bump)
    assert len(gpu) == len(host) > 1000
    assert gpu.tobytes() == host.tobytes()
    if scene == "skin.pbrt" and min_dist is None:
        assert len(gpu) > 2_000_000
    assert np.all(np.isfinite(gpu["p"])) and np.all(np.isfinite(gpu["n"])) and np.all(gpu["area"] > 0)
