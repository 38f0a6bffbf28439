"""LayeredSkin multipole profile built on the GPU (profile_gpu.hip) vs the product's host build
(material.cpp, itself checked against the kissfft oracle in test_host_parity.py): same
algorithm, FP64 grids and transforms; differences come only from device expf in the dipole
sums and complex division rounding -- bounded at 1e-6 of each channel's peak."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PARAMS = [
    dict(roughness=0.3, nmperunit=40e6, f_mel=0.5, f_eu=0.5, f_blood=0.5, f_ohg=0.5, desired_length=64),
    dict(desired_length=128),                                 # CreateLayeredSkinMaterial defaults
    dict(nmperunit=40e6, desired_length=512, lerp_on_thin_slab=0),
]


@pytest.mark.parametrize("kw", PARAMS)
def test_gpu_profile_matches_host(mpss, kw):
    import torch
    assert torch.cuda.is_available()
    skin = mpss.default_skin(Kt=[0.0] * 30, **kw)
    ctx = mpss.Context(profile_on_host=0)
    mid = ctx.add_layeredskin(skin)
    tab, rcp, rho, tot = ctx.material_tables(mid)
    layers = mpss.host_skin_layers(skin)
    htab, hrcp, htot = mpss.host_build_profile(*layers, desired_length=skin.desired_length,
                                               lerp=bool(skin.lerp_on_thin_slab))
    assert tab.shape == htab.shape
    assert np.array_equal(rcp, hrcp)
    peak = np.abs(htab).max(axis=1, keepdims=True)
    assert np.all(np.abs(tab - htab) <= 1e-6 * peak)
    np.testing.assert_allclose(tot, htot, rtol=1e-6)
    ctx.close()
