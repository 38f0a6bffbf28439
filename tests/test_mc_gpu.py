"""Monte-Carlo layered profile kernel (mpss_mc_profile) vs the CPU oracle (oracle/mc.c).

Both sides draw identical per-photon random streams, so most photons follow identical paths;
paths can part where a double exp/log/sin/cos of the device library differs from glibc in the
last bit, so the comparison is statistical: totals within 4 binomial sigma and coarse ring
bins within 5 sigma. Energy conservation without absorption is exact up to FP64 summation."""
import numpy as np
import pytest

import oracle_mc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(mpss):
    import torch
    assert torch.cuda.is_available()
    return mpss.Context()


def test_energy_conservation(ctx):
    o = ctx.mc_profile([(0.0, 2.0, 1.4, 0.3), (0.0, 0.5, 1.3, 2.0)], mfp_range=2000, nsegments=64, nphotons=50000,
                       seed=3)
    assert o["total_r"] + o["total_t"] == pytest.approx(1.0, abs=1e-9)
    assert o["events"] > 50000


@pytest.mark.parametrize("layers", [
    [(0.01, 1.0, 1.4, 50.0)],
    [(0.2, 3.0, 1.4, 0.25), (0.05, 1.5, 1.4, 5.0)],   # thin epidermis over dermis, skin-like ratios
])
def test_matches_oracle(ctx, layers):
    n = 200000
    g = ctx.mc_profile(layers, mfp_range=16, nsegments=1024, nphotons=n, seed=89)
    c = oracle_mc.mc_profile(layers, mfp_range=16, nsegments=1024, nphotons=n, seed=89)
    for k in ("total_r", "total_t"):
        p = max(c[k], 1.0 / n)
        sigma = np.sqrt(p * (1 - min(p, 0.999)) / n)
        assert abs(g[k] - c[k]) <= 4 * sigma + 1e-12, (k, g[k], c[k])
    # coarse rings: 16 groups of 64 segments, compared as photon fractions
    i = np.arange(1024, dtype=np.float64)
    ext = c["extent"]
    area = np.pi * ((2 * i + 1) * ext / 1024) * (ext / 1024)
    gr = (g["reflectance"] * area).reshape(16, 64).sum(1)
    cr = (c["reflectance"] * area).reshape(16, 64).sum(1)
    sig = np.sqrt(np.maximum(cr, 1.0 / n) / n)
    assert np.all(np.abs(gr - cr) <= 5 * sig), np.abs(gr - cr) / sig


def test_bad_layers(ctx, mpss):
    with pytest.raises(mpss.MpssError):
        ctx.mc_profile([(0.1, 0.0, 1.4, 1.0)], nphotons=10)
    with pytest.raises(mpss.MpssError):
        ctx.mc_profile([(0.1, 1.0, 1.4, 1.0)], nsegments=0, nphotons=10)
