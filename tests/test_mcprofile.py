"""The "mcprofile" renderer's host side (src/renderers/mcprofile.cpp:356-625), no GPU:

* MultipoleReferenceTask (:381-425): mpss.mc_reference (libmpss, host code) vs the oracle's
  MPC restatement (oracle/mpc.c + oracle_mc.mc_reference) -- bit-exact, for scenes/mcprofile.pbrt's
  layers with lerp on, and for a thin single slab where the two lerp settings differ.
* CreateMonteCarloProfileRenderer's parameters and the output file of Render (:544-586): the
  header, six rows, the six r x Rd(r) rows, %g numbers; read back by mcprofile.read_tsv.
The GPU half (the walk, the usemontecarlo material) is test_mcprofile_gpu.py.
"""
import os

import numpy as np
import pytest

import oracle_mc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C4_LAYERS = [(723.6646118164062, 577.9549560546875, 1.399999976158142, 0.0024999999441206455),
             (9.664658546447754, 288.97747802734375, 1.399999976158142, 0.20000000298023224)]


def test_mc_reference_c4_layers_bit_exact(mpss, oracle):
    a = mpss.mc_reference(C4_LAYERS, 16.0, 1024, True)
    b = oracle_mc.mc_reference(C4_LAYERS, 16.0, 1024, True)
    assert np.array_equal(a["reflectance"], b["reflectance"])
    assert np.array_equal(a["transmittance"], b["transmittance"])
    assert (a["total_r"], a["total_t"]) == (b["total_r"], b["total_t"])
    assert 0.0 < a["total_r"] < 1.0 and a["reflectance"][0] > a["reflectance"][-1] >= 0.0


def test_mc_reference_thin_slab_lerp(mpss, oracle):
    """A slab thinner than its lerp threshold: lerponthinslab changes the profile, and both
    settings agree with the oracle bit for bit."""
    lay = [(0.5, 4.0, 1.3, 0.08)]
    out = {}
    for lerp in (False, True):
        a = mpss.mc_reference(lay, 8.0, 64, lerp)
        b = oracle_mc.mc_reference(lay, 8.0, 64, lerp)
        assert np.array_equal(a["reflectance"], b["reflectance"]), lerp
        assert np.array_equal(a["transmittance"], b["transmittance"]), lerp
        assert (a["total_r"], a["total_t"]) == (b["total_r"], b["total_t"])
        out[lerp] = a
    # the unlerped multipole sum goes negative on a slab this thin (-0.24 total transmittance):
    # the artifact lerponthinslab exists for
    assert out[False]["total_t"] != out[True]["total_t"]
    assert not np.array_equal(out[False]["reflectance"], out[True]["reflectance"])


def test_mc_reference_rejects_bad_layers(mpss):
    with pytest.raises(mpss.MpssError):
        mpss.mc_reference([(0.1, 0.0, 1.4, 1.0)], 16.0, 64)
    with pytest.raises(mpss.MpssError):
        mpss.mc_reference(np.zeros((0, 4), np.float32), 16.0, 64)


def test_create_from_params_mcprofile_scene(mpss):
    from mpss import mcprofile, pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "mcprofile.pbrt"))
    kind, ps = sc.renderer
    assert kind == "mcprofile"
    r = mcprofile.create_from_params(ps)
    assert r.layers.shape == (2, 4) and np.allclose(r.layers, C4_LAYERS)
    assert (r.mfp_range, r.segments, r.photons, r.filename) == (16.0, 1024, 100_000_000, "mcprofile.txt")
    ext = r.extent()
    mfp = sum(1.0 / float(np.float32(np.float32(a) + np.float32(b))) for a, b, _, _ in C4_LAYERS)
    assert ext == pytest.approx(16.0 * mfp / 2, rel=1e-12)


def test_tsv_layout_round_trip(mpss, tmp_path):
    from mpss import mcprofile
    n = 8
    r = mcprofile.MonteCarloProfileRenderer([(1.0, 10.0, 1.4, 5.0)], 4.0, n, 1000, str(tmp_path / "p.txt"))
    rng = np.random.default_rng(0)
    prof = {k: rng.random(n) for k in ("reflectance", "transmittance")}
    ref = {lerp: dict(reflectance=rng.random(n), transmittance=rng.random(n), total_r=0.25 + lerp,
                      total_t=1e-3) for lerp in (False, True)}
    r.profile, r.reference = prof, ref
    r.result = dict(totalMCReflectance=0.125, totalMCTransmittance=0.0, totalNoLerpReflectance=0.25,
                    totalNoLerpTransmittance=1e-3, totalLerpReflectance=1.25, totalLerpTransmittance=1e-3)
    (tmp_path / "p.txt").write_text(r.tsv())
    lines = (tmp_path / "p.txt").read_text().splitlines()
    assert len(lines) == 13 and all(len(l.split("\t")) == n + 2 for l in lines)
    assert lines[0].startswith("Name\tTotal\t")
    names = [l.split("\t")[0] for l in lines[1:]]
    six = ["Monte-Carlo Reflectance", "Monte-Carlo Transmittance", "Multipole Reflectance",
           "Multipole Transmittance", "Lerped Reflectance", "Lerped Transmittance"]
    assert names == six + six
    dist, rows = mcprofile.read_tsv(str(tmp_path / "p.txt"))
    ext = r.extent()
    np.testing.assert_allclose(dist, (np.arange(n) + .5) * ext / n, rtol=1e-5)
    (t0, v0), (t1, v1) = rows["Monte-Carlo Reflectance"]
    assert t0 == t1 == 0.125
    np.testing.assert_allclose(v0, prof["reflectance"], rtol=1e-5)
    np.testing.assert_allclose(v1, prof["reflectance"] * dist, rtol=2e-5)
    (t0, v0), _ = rows["Lerped Transmittance"]
    np.testing.assert_allclose(v0, ref[True]["transmittance"], rtol=1e-5)
    assert lines[1].split("\t")[1] == "0.125" and lines[3].split("\t")[1] == "0.25"


def test_layeredskin_usemontecarlo_params(mpss, tmp_path):
    """"bool usemontecarlo" / "string photons" (layeredskin.cpp:250-252) reach mpss_layeredskin;
    defaults false / 10000000."""
    from mpss import pbrtscene
    src = open(os.path.join(ROOT, "scenes", "skin.pbrt")).read()
    d = mpss.default_skin()
    assert (d.use_monte_carlo, d.photons) == (0, 10_000_000)
    txt = src.replace('Material "layeredskin"', 'Material "layeredskin" "bool usemontecarlo" "true" '
                                                '"string photons" "250000"', 1)
    assert txt != src
    p = tmp_path / "mc_skin.pbrt"
    p.write_text(txt)
    base = os.path.join(ROOT, "scenes")
    for f in os.listdir(base):
        if not f.endswith(".pbrt") and not (tmp_path / f).exists():
            os.symlink(os.path.join(base, f), tmp_path / f)
    sc = pbrtscene.load(str(p))
    m = sc.materials[0]
    assert (m["use_monte_carlo"], m["photons"]) == (1, 250_000)
    s = mpss.default_skin(**{k: v for k, v in m.items() if k not in ("Kr", "Kt", "albedo", "albedo_tex",
                                                                      "bump_tex")})
    assert (s.use_monte_carlo, s.photons) == (1, 250_000)
