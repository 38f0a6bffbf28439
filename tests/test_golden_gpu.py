"""The GPU path against the committed golden fixtures (tests/golden/golden.npz, from the oracle;
see tests/golden/make_golden.py): the GPU-built LayeredSkin profile at desiredlength 512 (the
benched length; 2048^2 FP64 FFTs on the device) within 1e-6 of each band's peak at the stored
entries, its rho table bit-exact, Mo() bit-exact in the reference order and within 2e-5 in the
production sharded gather (the same visit counts), and the small skin.pbrt image within the
render parity tolerance."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def golden():
    return dict(np.load(os.path.join(HERE, "golden", "golden.npz")))


@pytest.fixture(scope="module")
def gen():
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import make_golden
    return make_golden


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available()
    return torch


def test_gpu_profile_512_and_rho(mpss, torch_dev, golden):
    ctx = mpss.Context()
    skin = mpss.default_skin(roughness=0.3, nmperunit=40e6, f_mel=0.5, f_eu=0.5, f_blood=0.5, f_ohg=0.5,
                             layer_thickness_nm=(0.25e6, 20e6), layer_ior=(1.4, 1.4), desired_length=512)
    tab, rcp, rho, tot = ctx.material_tables(ctx.add_layeredskin(skin))
    ctx.close()
    assert tab.shape[1] == int(golden["profile_512_len"])
    assert np.array_equal(rcp, golden["profile_512_rcp"])
    got = tab[:, golden["profile_512_idx"]]
    ref = golden["profile_512"]
    assert np.all(np.abs(got - ref) <= 1e-6 * np.abs(ref).max(axis=1, keepdims=True))
    assert np.allclose(tot, golden["profile_512_total"], rtol=1e-5)
    ulps = np.abs(rho.view(np.int32).astype(np.int64) - golden["rho_hd"].view(np.int32).astype(np.int64))
    assert ulps.max() <= 1 and (ulps == 0).mean() >= 0.999  # GPU rho_hd (rho_gpu.hip)


@pytest.mark.parametrize("mode", [1, 0])
def test_gpu_mo_vs_golden(mpss, torch_dev, golden, gen, mode):
    torch = torch_dev
    (p, n, E, area), q = gen.mo_inputs()
    assert gen.sha(p, n, E, area, q) == str(golden["mo_cloud_sha"])
    ctx = mpss.Context(max_error=float(golden["mo_max_error"]), exact_mo=mode)
    mid = ctx.set_material_tables(golden["profile_64"], golden["profile_64_rcp"], np.zeros(1025, np.float32))
    ctx.set_irradiance_points(p, n, E, area)
    qd = torch.from_numpy(q).cuda()
    out = torch.zeros((len(q), 30), dtype=torch.float32, device="cuda")
    cnt = torch.zeros((len(q), 4), dtype=torch.int32, device="cuda")
    ctx.mo_batch(mid, len(q), qd.data_ptr(), out.data_ptr(), cnt.data_ptr())
    torch.cuda.synchronize()
    got, cnt = out.cpu().numpy(), cnt.cpu().numpy()
    ctx.close()
    ref = golden["mo"]
    if mode == 1:
        assert np.array_equal(got, ref)
        assert np.array_equal(cnt[:, 0], golden["mo_nodes"]) and np.array_equal(cnt[:, 1], golden["mo_points"])
    else:
        scale = np.maximum(np.abs(ref), np.abs(ref).max(axis=1, keepdims=True) * 1e-3)
        assert np.all(np.abs(got - ref) <= 2e-5 * scale + 1e-30)


def test_gpu_image_vs_golden(mpss, torch_dev, golden, gen):
    torch = torch_dev
    from mpss import pbrtscene
    from test_render_parity_gpu import _check
    sc = gen.image_scene()
    ctx = pbrtscene.build_context(sc)
    ctx.preprocess(seed=7)
    assert gen.sha(ctx.surface_points()) == str(golden["image_points_sha"])
    out = torch.zeros((sc.xres * sc.yres * 4,), dtype=torch.float32, device="cuda")
    ctx.render_tile(sc.spp, 9, 0, sc.xres, 0, sc.yres, out.data_ptr())
    torch.cuda.synchronize()
    got = out.cpu().numpy().reshape(sc.yres, sc.xres, 4)
    ctx.close()
    _check(got, golden["image_xyzw"])
