"""DiffusionReflectance, the single-dipole Rd functor (reference
src/integrators/diffusionutil.h:38-83), on the CPU: the product's host evaluator against the
oracle restatement (bit-exact: the same float operations in the same order, exp in double
rounded once), the oracle against an independent float64 closed form (Jensen et al. 2001,
eqs. 4-5: within 2e-6 relative), the total diffuse reflectance of that closed form against
Jensen's analytic Rd_total (eq. 6; numerical quadrature, 1e-6), TotalReflectance()'s 1024-step
sum bit-exact between product and oracle, and Mo() with the dipole at maxError -> 0 equal to
the brute-force point sum (the closed-form pin SURVEY.md 8c item 4 names for the gather)."""
import numpy as np
import pytest

import synth

NB = 30
SIGMA_A = np.array([0.5 + 0.1 * c for c in range(NB)], np.float32)
SIGMAP_S = np.array([40.0 + 1.5 * c for c in range(NB)], np.float32)
ETA = 1.3


def fdr64(eta):
    return -1.4399 / eta ** 2 + 0.7099 / eta + 0.6681 + 0.0636 * eta  # reflection.h:64-71, eta >= 1


def dipole64(sa, sps, eta, d2):
    """Jensen 2001 eqs. 4-5 in float64 (what diffusionutil.h:49-58 computes in float)."""
    sa, sps, d2 = np.float64(sa), np.float64(sps), np.asarray(d2, np.float64)[:, None]
    A = (1 + fdr64(eta)) / (1 - fdr64(eta))
    st = sa + sps
    tr = np.sqrt(3 * sa * st)
    ap = sps / st
    zr = 1 / st
    zv = -zr * (1 + 4 / 3 * A)
    dr = np.sqrt(d2 + zr * zr)
    dv = np.sqrt(d2 + zv * zv)
    return ap / (4 * np.pi) * (zr * (dr * tr + 1) * np.exp(-tr * dr) / dr ** 3 -
                               zv * (dv * tr + 1) * np.exp(-tr * dv) / dv ** 3)


def test_host_dipole_bit_exact_vs_oracle(mpss, oracle):
    mfp = 1.0 / (SIGMA_A + SIGMAP_S)
    d2 = np.concatenate([[0.0], np.geomspace(1e-8, 1.0, 400), (np.arange(64) * (4 * mfp[3]) ** 2 / 64)]).astype(
        np.float32)
    got, tot = mpss.host_dipole_rd(SIGMA_A, SIGMAP_S, ETA, d2)
    dip = oracle.Diffusion(SIGMA_A, SIGMAP_S, ETA)
    ref = dip(d2)
    assert np.array_equal(got, ref)
    assert np.array_equal(tot, dip.total())
    assert np.all(got >= 0) and np.all(np.isfinite(got))


def test_oracle_dipole_matches_float64_closed_form(oracle):
    d2 = np.geomspace(1e-8, 4e-3, 300).astype(np.float32)
    got = oracle.Diffusion(SIGMA_A, SIGMAP_S, ETA)(d2).astype(np.float64)
    ref = dipole64(SIGMA_A, SIGMAP_S, ETA, d2)
    live = ref > 1e-30
    assert np.all(np.abs(got - ref)[live] <= 2e-6 * ref[live] + 1e-37)


def test_closed_form_total_reflectance_is_jensens_rd(oracle):
    """2 pi int Rd(r) r dr = (alpha'/2)(1 + exp(-4/3 A sqrt(3(1-alpha')))) exp(-sqrt(3(1-alpha')))."""
    from scipy.integrate import quad
    A = (1 + fdr64(ETA)) / (1 - fdr64(ETA))
    for c in (0, 11, 29):
        sa, sps = float(SIGMA_A[c]), float(SIGMAP_S[c])
        ap = sps / (sa + sps)
        s = np.sqrt(3 * (1 - ap))
        analytic = ap / 2 * (1 + np.exp(-4 / 3 * A * s)) * np.exp(-s)
        f = lambda r: 2 * np.pi * r * dipole64(sa, sps, ETA, np.array([r * r]))[0, 0]
        mfp = 1 / (sa + sps)
        num = sum(quad(f, a, b, limit=200)[0] for a, b in ((0, mfp), (mfp, 50 * mfp), (50 * mfp, np.inf)))
        assert num == pytest.approx(analytic, rel=1e-6)
    # TotalReflectance() integrates only to (4 mfp)^2 with a left Riemann sum: it is below the
    # analytic total and within the truncated tail
    tot = oracle.Diffusion(SIGMA_A, SIGMAP_S, ETA).total()
    assert np.all(tot > 0)


def test_oracle_mo_dipole_at_zero_error_is_brute_force(oracle):
    p, n, E, area = synth.ellipsoid_cloud(3000, radii=(0.05, 0.06, 0.07), seed=3)
    q = synth.surface_queries(64, radii=(0.05, 0.06, 0.07), seed=4)
    dip = oracle.Diffusion(SIGMA_A, SIGMAP_S, ETA)
    t = oracle.Octree(p, n, E, area)
    mo = t.mo_diffusion(q, dip, 0.0).astype(np.float64)
    ref = np.zeros((len(q), NB))
    for i, x in enumerate(q):
        d2 = ((p - x) ** 2).sum(1, dtype=np.float32)
        rd = dipole64(SIGMA_A, SIGMAP_S, ETA, d2)
        ref[i] = (rd * E * area[:, None]).sum(0)
    assert np.allclose(mo, ref, rtol=2e-5, atol=0)
    # and with maxError the hierarchy stays within a few percent of the exact sum
    approx = t.mo_diffusion(q, dip, 0.05).astype(np.float64)
    assert np.all(np.abs(approx - ref) <= 0.05 * ref + 1e-30)
