"""pbrtscene's LayeredSkin parameter parsing (CreateLayeredSkinMaterial, layeredskin.cpp:222-262): the
profile switches reach mpss_layeredskin with the reference's names and defaults (CPU only)."""
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(tmp_path, extra):
    from mpss import pbrtscene
    src = open(os.path.join(ROOT, "scenes", "skin.pbrt")).read()
    src = src.replace('"float f_ohg" 0.5', '"float f_ohg" 0.5 ' + extra)
    p = tmp_path / "s.pbrt"
    p.write_text(src)
    import shutil
    shutil.copy(os.path.join(ROOT, "scenes", "head_mesh.npz"), tmp_path / "head_mesh.npz")
    return pbrtscene.load(str(p))


def test_profile_switch_defaults(mpss):
    s = mpss.default_skin()
    assert s.gen_profile == 1 and s.show_irradiance_points == 0
    assert s.irradiance_point_size == pytest.approx(0.002)


@pytest.mark.parametrize("extra,want", [
    ('"bool genprofile" "false"', dict(gen_profile=0)),
    ('"bool showirradiancepoints" "true" "float irradiancepointsize" 0.01',
     dict(show_irradiance_points=1, irradiance_point_size=0.01)),
    ('"bool rgbprofile" "true" "integer desiredlength" 128', dict(rgb_profile=1, desired_length=128)),
])
def test_profile_switches_parse(mpss, tmp_path, extra, want):
    sc = _load(tmp_path, extra)
    m = sc.materials[0]
    for k, v in want.items():
        assert m[k] == pytest.approx(v), (k, m.get(k))
    s = mpss.default_skin(**{k: v for k, v in m.items() if k not in ("Kr", "Kt", "albedo", "albedo_tex", "bump_tex")})
    for k, v in want.items():
        assert getattr(s, k) == pytest.approx(v)
