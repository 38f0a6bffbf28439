"""CPU checks of the Monte-Carlo layered profile restatement (oracle/mc.c), the checker of the
product's mc_profile kernel: energy conservation without absorption, Fresnel-free
transmission through an index-matched non-scattering-dominated slab, and agreement with the
multipole model in the regime where diffusion holds (the comparison MonteCarloProfileRenderer
itself prints, mcprofile.cpp:420-440, 499-533)."""
import numpy as np
import pytest

import oracle_mc


def test_energy_conservation_without_absorption():
    for layers in ([(0.0, 1.0, 1.0, 1.0)], [(0.0, 2.0, 1.4, 0.3), (0.0, 0.5, 1.3, 2.0)]):
        o = oracle_mc.mc_profile(layers, mfp_range=2000, nsegments=64, nphotons=20000, seed=3)
        assert o["total_r"] + o["total_t"] == pytest.approx(1.0, abs=1e-12)


def test_deterministic_streams():
    a = oracle_mc.mc_profile([(0.1, 1.0, 1.4, 1.0)], nsegments=128, nphotons=5000, seed=7, nthreads=1)
    b = oracle_mc.mc_profile([(0.1, 1.0, 1.4, 1.0)], nsegments=128, nphotons=5000, seed=7, nthreads=4)
    assert np.array_equal(a["raw_r"], b["raw_r"]) or np.allclose(a["raw_r"], b["raw_r"], rtol=1e-12)


def test_thick_slab_matches_multipole_total(oracle):
    """High-albedo, effectively semi-infinite layer: MC total diffuse reflectance vs the
    multipole/dipole total within 5 % (diffusion is accurate at albedo 0.99)."""
    mua, musp, ior, th = 0.01, 1.0, 1.4, 50.0
    o = oracle_mc.mc_profile([(mua, musp, ior, th)], mfp_range=64, nsegments=256, nphotons=200000, seed=89)
    extent = o["extent"]
    _, _, _, tr, _ = oracle.mpc_profile([(ior, th, mua, musp)], step=extent * 1.01 / 1024, desired_length=1024,
                                        lerp=False, resample=False)
    assert o["total_r"] == pytest.approx(tr, rel=0.05)
