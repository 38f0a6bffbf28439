"""Pins the CPU oracle (test infrastructure) against the reference's own self-checks.

The reference has no golden vectors for this path, so each check here is
one of the validation identities its sources contain:
  - MT19937 known answer (core/rng.cpp is the published MT19937ar)
  - kissfft vs brute-force DFT (libkissfft/test/test_vs_dft.c)
  - MPC: pi * integral Rd d(r^2) ~= totalReflectance (src/multipole/test/test.cpp:74-75)
  - rho_hd(cos=1) = normal-incidence Fresnel reflectance for a smooth-ish Beckmann lobe
  - Mo() at maxError -> 0 equals the brute-force sum over all points (diffusionutil.h:175-210)
"""
import numpy as np
import pytest

import synth


def test_mt19937_known_answer(oracle):
    out = np.zeros(5, np.uint32)
    oracle.lib().o_mt_first(5489, 5, out)
    # first outputs of the reference MT19937ar implementation for the default seed 5489
    assert out.tolist() == [3499211612, 581869302, 3890346734, 3586334585, 545404204]


@pytest.mark.parametrize("n", [2048, 1024, 12, 60, 63])
def test_kissfft_vs_dft(oracle, n):
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    xi = np.empty(2 * n)
    xi[0::2], xi[1::2] = x.real, x.imag
    out = np.zeros(2 * n)
    oracle.lib().o_kiss_fft(n, 0, xi, out)
    y = out[0::2] + 1j * out[1::2]
    k = np.arange(n)
    dft = np.exp(-2j * np.pi * (np.outer(k, k) % n) / n) @ x  # exact phase reduction
    assert np.abs(y - dft).max() / np.abs(dft).max() < 1e-13


def test_kissfft_real2d_roundtrip(oracle):
    rng = np.random.default_rng(3)
    r, c = 32, 64
    a = rng.standard_normal((r, c))
    f = np.zeros(r * (c // 2 + 1) * 2)
    oracle.lib().o_kiss_fftndr2(r, c, np.ascontiguousarray(a.ravel()), f)
    fc = (f[0::2] + 1j * f[1::2]).reshape(r, c // 2 + 1)
    assert np.abs(fc - np.fft.rfft2(a)).max() < 1e-12
    back = np.zeros(r * c)
    oracle.lib().o_kiss_fftndri2(r, c, f, back)
    assert np.abs(back.reshape(r, c) / (r * c) - a).max() < 1e-13


def _test_cpp_layers():
    # src/multipole/test/test.cpp:84-116 layer specs (ior, thickness d, mua, musp')
    return [(1.4, 0.025, 0.268088, 19.4879), (1.4, 2.0, 0.268088, 9.74395)]


@pytest.mark.parametrize("layers", [[_test_cpp_layers()[0]], [_test_cpp_layers()[1]], _test_cpp_layers()])
def test_mpc_integral_matches_total_reflectance(oracle, layers):
    mfp = np.mean([1.0 / (l[2] + l[3]) for l in layers])
    step = np.float32(12.0 * mfp / 128)
    d, R, T, tr, tt = oracle.mpc_profile(layers, step, desired_length=128, resample=False)
    assert np.all(np.diff(d) > 0)
    integral = np.pi * np.trapezoid(R.astype(np.float64), d.astype(np.float64))
    assert tr > 0
    assert abs(integral - tr) / tr < 0.05, (integral, tr)


def test_rho_normal_incidence_is_fresnel_r0(oracle):
    hd, hh = oracle.rho_table(0.3, 1.4, n_entries=17, sqrt_samples=64)
    r0 = ((1.4 - 1) / (1.4 + 1)) ** 2
    assert abs(hd[-1] - r0) / r0 < 0.02
    assert np.all(np.diff(hd) < 0)  # rho_hd falls monotonically towards normal incidence
    assert 0 < hh < 1


def test_skin_layers_physical(oracle):
    mua, musp, th, eta = oracle.skin_layers()
    assert mua.shape == (2, 30) and np.all(mua > 0) and np.all(musp > 0)
    assert np.all(np.diff(musp[0]) < 0)  # Rayleigh+Mie scattering falls with wavelength
    assert th.tolist() == [np.float32(0.25e6) / np.float32(40e6), np.float32(20e6) / np.float32(40e6)]


def _brute_mo(p, E, area, q, table, rcp, oracle):
    L = table.shape[1]
    out = np.zeros((len(q), 30), np.float64)
    for i, x in enumerate(q):
        d2 = ((x[None, :] - p) ** 2).sum(1).astype(np.float32)
        for c in range(30):
            rd = np.array([oracle.lib().o_sample_profile(table[c], L, rcp[c], float(v)) for v in d2], np.float32)
            out[i, c] = (rd * E[:, c] * area).sum()
    return out


def test_mo_converges_to_bruteforce(oracle):
    p, n, E, area = synth.ellipsoid_cloud(400, radii=(0.02, 0.025, 0.03), seed=3, black_frac=0.1)
    rng = np.random.default_rng(5)
    L = 256
    x = np.linspace(0, 1, L, dtype=np.float32)
    table = np.stack([np.exp(-x * (3 + 0.1 * c)).astype(np.float32) for c in range(30)])
    rcp = np.full(30, (L - 1) / 0.004, np.float32)
    q = synth.surface_queries(8, radii=(0.02, 0.025, 0.03), seed=9, sort=False)
    t = oracle.Octree(p, n, E, area)
    mo = t.mo(q, table, rcp, 1e-9)
    ref = _brute_mo(p, E, area, q, table, rcp, oracle)
    assert np.allclose(mo, ref, rtol=1e-4, atol=1e-7)
    mo_fast, nn, npt = t.mo(q, table, rcp, 0.5, counters=True)
    assert np.all(nn > 0) and np.all(nn <= t.num_nodes())
    assert np.allclose(mo_fast, ref, rtol=0.2, atol=1e-6)  # hierarchical approximation stays close


def test_octree_export_consistent(oracle):
    p, n, E, area = synth.ellipsoid_cloud(3000, seed=4)
    t = oracle.Octree(p, n, E, area)
    d = t.export()
    N = t.num_nodes()
    assert len(d["depth"]) == N and d["skip"][0] == N
    assert sorted(d["order"].tolist()) == list(range(len(p)))
    # root carries the sum of every point's E*area (InitHierarchy, diffusionutil.h:133-173)
    assert np.allclose(d["Et"][0], (E * area[:, None]).sum(0), rtol=1e-4)
    assert np.isclose(d["area"][0], area.sum(), rtol=1e-5)
