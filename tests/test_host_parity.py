"""Product host builders (libmpss, no GPU) vs the CPU oracle on identical inputs.

Bit-exact where both sides run the same IEEE-float formula (skin coefficients, rho table,
octree build); the profile table goes through different FFT implementations (kissfft
restated in the oracle, the product's own radix-2 FFT), so it is compared with a tolerance
scaled to the channel's peak value (FP64 transform rounding, then float output).
"""
import numpy as np
import pytest

import synth

SKIN = dict(roughness=0.3, nmperunit=40e6, f_mel=0.5, f_eu=0.5, f_blood=0.5, f_ohg=0.5,
            layer_thickness_nm=(0.25e6, 20e6), layer_ior=(1.4, 1.4))  # S007Scene.pbrt:35-47


def test_skin_layers_bit_exact(oracle, mpss):
    m = mpss.default_skin(**SKIN)
    pm = mpss.host_skin_layers(m)
    om = oracle.skin_layers(0.3, 40e6, 0.5, 0.5, 0.5, 0.5, (0.25e6, 20e6), (1.4, 1.4))
    for a, b in zip(pm, om):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("params", [dict(), dict(f_mel=0.01, f_blood=0.01, nmperunit=100e6)])
def test_skin_layers_variants(oracle, mpss, params):
    kw = dict(SKIN)
    kw.update(params)
    pm = mpss.host_skin_layers(mpss.default_skin(**kw))
    om = oracle.skin_layers(kw["roughness"], kw["nmperunit"], kw["f_mel"], kw["f_eu"], kw["f_blood"], kw["f_ohg"],
                            kw["layer_thickness_nm"], kw["layer_ior"])
    for a, b in zip(pm, om):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("fixed", [False, True])
def test_rho_table_bit_exact(oracle, mpss, fixed):
    """fixed: LayeredSkin "doublerefsslf" -- FixedFresnelDielectric (reflection.h:315-324)."""
    hd_p, hh_p = mpss.host_rho_table(0.3, 1.4, n=33, sqrt_samples=32, double_ref_sslf=fixed)
    hd_o, hh_o = oracle.rho_table(0.3, 1.4, n_entries=33, sqrt_samples=32, fixed=fixed)
    assert np.array_equal(hd_p, hd_o)
    assert hh_p == hh_o
    if fixed:  # the fixed variant reflects more than the plain one
        hd_n, _ = oracle.rho_table(0.3, 1.4, n_entries=33, sqrt_samples=32)
        assert np.all(hd_o >= hd_n) and np.any(hd_o > hd_n)


@pytest.mark.parametrize("desired", [16, 64])
def test_profile_matches_oracle(oracle, mpss, desired):
    mua, musp, th, eta = oracle.skin_layers(0.3, 40e6, 0.5, 0.5, 0.5, 0.5, (0.25e6, 20e6), (1.4, 1.4))
    tab_o, rcp_o, sp_o, tot_o = oracle.compute_profile(mua, musp, eta, th, desired_length=desired)
    tab_p, rcp_p, tot_p = mpss.host_build_profile(mua, musp, th, eta, desired_length=desired)
    assert tab_p.shape == tab_o.shape
    assert np.array_equal(rcp_p, rcp_o)  # grid spacing is pure float arithmetic
    peak = np.abs(tab_o).max(axis=1, keepdims=True)
    assert np.abs(tab_p - tab_o).max() <= 1e-6 * peak.max()
    assert np.all(np.abs(tab_p - tab_o) <= 1e-6 * peak)
    assert np.allclose(tot_p, tot_o, rtol=1e-5)


def test_octree_build_bit_exact(oracle, mpss):
    p, n, E, area = synth.ellipsoid_cloud(20000, seed=21, black_frac=0.05)
    d_o = oracle.Octree(p, n, E, area).export()
    d_p = mpss.host_octree_export(p, n, E, area)
    for k in ("p", "area", "Et", "depth", "skip", "order"):
        assert np.array_equal(d_p[k], d_o[k]), k
    assert np.array_equal(d_p["leaf_count"], d_o["leaf_count"])
    leaf = d_o["leaf_count"] > 0
    assert np.array_equal(d_p["leaf_first"][leaf], d_o["leaf_first"][leaf])


def test_octree_rejects_coincident_points(mpss):
    p = np.zeros((12, 3), np.float32)
    n = np.tile(np.float32([0, 0, 1]), (12, 1))
    E = np.ones((12, 30), np.float32)
    a = np.ones(12, np.float32)
    with pytest.raises(mpss.MpssError):
        mpss.host_octree_export(p, n, E, a)
