"""Committed golden fixtures (tests/golden/golden.npz, written by tests/golden/make_golden.py from
the CPU oracle): the oracle still reproduces every one of them bit for bit (a drift guard on the
restatement, which is parity-unpinned against reference outputs), and the product's
host builders agree with them on the CPU (profile within 1e-6 of each band's peak: the FFTs
differ; rho table, tessellation bit-exact)."""
import os

import numpy as np
import pytest

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


def test_oracle_reproduces_fixtures(oracle, golden, gen):
    fresh = gen.compute(oracle)
    assert sorted(fresh) == sorted(golden)
    for k, v in fresh.items():
        assert np.array_equal(np.asarray(v), golden[k]), k


def test_product_host_profile_and_rho(mpss, golden, gen):
    skin = mpss.default_skin(roughness=0.3, nmperunit=40e6, f_mel=0.5, f_eu=0.5, f_blood=0.5, f_ohg=0.5,
                             layer_thickness_nm=(0.25e6, 20e6), layer_ior=(1.4, 1.4))
    layers = mpss.host_skin_layers(skin)
    tab, rcp, tot = mpss.host_build_profile(*layers, desired_length=64)
    ref = golden["profile_64"]
    assert tab.shape == ref.shape and np.array_equal(rcp, golden["profile_64_rcp"])
    assert np.all(np.abs(tab - ref) <= 1e-6 * np.abs(ref).max(axis=1, keepdims=True))
    assert np.allclose(tot, golden["profile_64_total"], rtol=1e-5)
    hd, hh = mpss.host_rho_table(0.3, 1.4)
    assert np.array_equal(hd, golden["rho_hd"]) and np.float32(hh) == golden["rho_hh"]


def test_product_host_tessellation(mpss, golden, gen):
    from mpss import pbrtscene
    pts = pbrtscene.mesh_points(gen.image_scene())
    assert len(pts) == int(golden["image_points_n"])
    assert gen.sha(pts) == str(golden["image_points_sha"])


def test_mo_inputs_unchanged(golden, gen):
    (p, n, E, area), q = gen.mo_inputs()
    assert gen.sha(p, n, E, area, q) == str(golden["mo_cloud_sha"])
