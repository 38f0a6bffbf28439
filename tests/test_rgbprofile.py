"""The rgbprofile LayeredSkin variant in the oracle (CPU): ComputeRGBMultipoleProfile's three
profiles (multipole.cpp:408-451) and the Rd functor MultipoleProfileData::reflectance with
isRGBProfile = Spectrum::FromRGBSpectrum(sampleRGBProfile(...)) (multipole.cpp:85-107) inside Mo.
"""
import numpy as np

import oracle_lib
import synth

NB = 30


def rgb_layers(mua, musp):
    """layeredskin.cpp:85-86: each layer's SampledSpectrum mua / musp as ToRGBSpectrum, replicated
    so band c carries component c % 3 (what the product builds; rows 0..2 are R, G, B)."""
    ra = np.stack([oracle_lib.to_rgb(m) for m in mua])
    rs = np.stack([oracle_lib.to_rgb(m) for m in musp])
    idx = np.arange(NB) % 3
    return ra[:, idx].astype(np.float32), rs[:, idx].astype(np.float32)


def test_rgb_profile_rows_repeat_components():
    mua, musp, th, eta = oracle_lib.skin_layers()
    ra, rs = rgb_layers(mua, musp)
    tab, rcp, _, tot = oracle_lib.compute_profile(ra, rs, eta, th, desired_length=32)
    for c in range(3, NB):
        assert np.array_equal(tab[c], tab[c % 3])
        assert rcp[c] == rcp[c % 3]
    assert (rcp[:3] > 0).all() and len(set(rcp[:3].tolist())) == 3
    assert (tot[:3] > 0).all()


def test_rgb_mo_matches_brute_force():
    """Mo at maxError -> 0 visits every point: Sum_i FromRGB(Rd_rgb(d_i^2)) * E_i * A_i."""
    mua, musp, th, eta = oracle_lib.skin_layers(nmperunit=1e6)
    ra, rs = rgb_layers(mua, musp)
    tab, rcp, _, _ = oracle_lib.compute_profile(ra, rs, eta, th, desired_length=32)
    p, n, E, area = synth.ellipsoid_cloud(1500, seed=41, black_frac=0.1)
    q = synth.surface_queries(20, seed=42)
    t = oracle_lib.Octree(p, n, E, area)
    got = t.mo_rgb(q, tab, rcp, 1e-12)
    L = tab.shape[1]
    want = np.zeros((len(q), NB), np.float64)
    for k, x in enumerate(q):
        d2 = ((p - x) ** 2).sum(axis=1).astype(np.float32)
        for i in np.nonzero(E.any(axis=1))[0]:
            rgb = np.array([oracle_lib.lib().o_sample_profile(np.ascontiguousarray(tab[j]), L, float(rcp[j]),
                                                              float(d2[i])) for j in range(3)], np.float32)
            want[k] += oracle_lib.from_rgb(rgb).astype(np.float64) * E[i] * area[i]
    np.testing.assert_allclose(got, want, rtol=2e-5, atol=1e-30)
    assert (got > 0).any()


def test_rgb_functor_of_grey_is_flat():
    """FromRGB(v, v, v) (reflectance) = 0.94 v rgbRefl2SpectWhite: equal R, G, B lookups give
    the white basis scaled, so a grey profile yields Mo proportional to the white basis band by
    band (for E = 1)."""
    mua, musp, th, eta = oracle_lib.skin_layers()
    ra, rs = rgb_layers(mua, musp)
    tab, rcp, _, _ = oracle_lib.compute_profile(ra, rs, eta, th, desired_length=32)
    grey = np.tile(tab[:1], (NB, 1))
    g_rcp = np.full(NB, rcp[0], np.float32)
    p, n, E, area = synth.ellipsoid_cloud(800, seed=43, black_frac=0.0)
    E = np.ones_like(E)
    q = synth.surface_queries(8, seed=44)
    t = oracle_lib.Octree(p, n, E, area)
    got = t.mo_rgb(q, grey, g_rcp, 0.05)
    white = oracle_lib.from_rgb(np.ones(3, np.float32)) / np.float32(0.94)
    ratio = got / white[None, :]
    np.testing.assert_allclose(ratio, np.broadcast_to(ratio[:, :1], ratio.shape), rtol=1e-5)
