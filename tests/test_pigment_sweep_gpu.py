"""The fork's actual workload -- one head rendered many times with varied LayeredSkin pigments -- on
the GPU's production path against the oracle, end to end.

The fork sweeps f_blood = H and f_mel = M over 0 ... 0.5, the epidermis thickness E over 0.03 ...
0.33 (x 1e6 nm) and f_eu = B over 0 ... 1 (/root/reference/utilities/csv/
PigmentSamplingValuesWThickness.csv, read by utilities/python/SceneMaker.py:6-62), with f_ohg 0.75,
roughness 0.35 and Kr = Kt = 0 (SceneMaker.py:40-51). The production Mo() gather reads its far field
from a common grid whose error floor was tuned on one material, so its accuracy is
checked here where it is hardest: at the corners of that sweep, the low-absorption corner (H = M = 0,
every band's reach longest) included, and with rgbprofile on at the lowest-absorption corner.

Each case is skin.pbrt (head.pbrt, its camera and area light, 1024x1024 frame, 64 spp,
minsampledistance 0.0015, desiredlength 512) with the corner's material. A 64x64 all-skin window is
rendered by the product (GPU tables, GPU irradiance, GPU octree, the sharded common-grid gather) and
by the oracle from its OWN profile and rho tables (tables_from_oracle), its OWN irradiance of the
same tessellated points (checked first against the GPU's, all 2.2 M of them) and its own octree --
the two sides share only the scene description. Criterion: tests/parity.py (film weights bit-exact,
XYZ within 1e-4 relative L-inf, no floor); the figures go to $MPSS_PARITY_REPORT.
"""
import os

import numpy as np
import pytest

import oracle_lib
import oracle_render as orr
import parity

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NT = oracle_lib.nthreads()

# (H = f_blood, M = f_mel, E = epidermis thickness / 1e6 nm, B = f_eu, rgbprofile): a half fraction
# of the 2^4 corners of the csv's ranges (B = the parity of the other three, so every factor and
# every pair of factors is varied), plus the lowest-absorption corner with rgbprofile on.
CORNERS = [
    (0.0, 0.0, 0.03, 0.0, 0),
    (0.5, 0.0, 0.03, 1.0, 0),
    (0.0, 0.5, 0.03, 1.0, 0),
    (0.5, 0.5, 0.03, 0.0, 0),
    (0.0, 0.0, 0.33, 1.0, 0),
    (0.5, 0.0, 0.33, 0.0, 0),
    (0.0, 0.5, 0.33, 0.0, 0),
    (0.5, 0.5, 0.33, 1.0, 0),
    (0.0, 0.0, 0.03, 0.0, 1),
]


def sweep_scene(H, M, E, B, rgb):
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin.pbrt"))
    for m in sc.materials:
        m.update(roughness=0.35, nmperunit=40e6, f_blood=H, f_mel=M, f_eu=B, f_ohg=0.75,
                 layer_thickness_nm=[E * 1e6, 20e6], layer_ior=[1.4, 1.4], Kr=[0.0, 0.0, 0.0], Kt=[0.0, 0.0, 0.0])
        if rgb:
            m["rgb_profile"] = 1
    return sc


@pytest.mark.parametrize("H,M,E,B,rgb", CORNERS)
def test_pigment_corner_window(mpss, oracle, H, M, E, B, rgb):
    import torch
    from mpss import pbrtscene
    from test_configs_gpu import _windows
    sc = sweep_scene(H, M, E, B, rgb)
    ctx = pbrtscene.build_context(sc)
    ctx.preprocess(seed=1)
    info = ctx.gather_info(0)
    assert info["common_grid"], "the production gather (common grid) must be the one under test"
    o = orr.OracleScene(sc, orr.tables_from_oracle(sc), ctx.cfg, mpss)
    pts = ctx.surface_points()
    assert len(pts) > 2_000_000 and pts.tobytes() == o.tessellate().tobytes()
    E_o = o.irradiance(pts, 1, nthreads=NT)
    E_g = ctx.irradiance()
    np.testing.assert_allclose(E_g, E_o, rtol=1e-5, atol=1e-6 * float(E_o.max()))
    assert (E_g == E_o).mean() >= 0.99
    o.set_octree(pts, E_o)
    x0, x1, y0, y1 = _windows(ctx, sc.xres, sc.yres, 64, 64, lambda f: f == 1.0)
    out = torch.zeros(((y1 - y0) * (x1 - x0) * 4,), dtype=torch.float32, device="cuda")
    ctx.render_tile(sc.spp, 7, x0, x1, y0, y1, out.data_ptr())
    torch.cuda.synchronize()
    got = out.cpu().numpy().reshape(y1 - y0, x1 - x0, 4)
    ref = o.render_tile(sc.spp, 7, x0, x1, y0, y1, nthreads=NT)
    name = "pigment_H%g_M%g_E%g_B%g%s" % (H, M, E, B, "_rgb" if rgb else "")
    st = parity.check_image(got, ref, name)
    # Kr = Kt = 0: no surface BSDF, so every value is the subsurface term alone
    assert (ref[..., 1] > 0).all()
    print("%s: relative L-inf %.3g (at %.2g of the peak), grid rel err max %.3g" %
          (name, st["rel_linf"], st["rel_linf_at_value"], float(info["rel_err"].max())))
    o.close()
    ctx.close()
