"""ImageTexture ("imagemap") on the host: the product's MIPMap build + lookups (texture.cpp /
texture.h, through mpss_host_imagemap_lookup) against the oracle's restatement (oracle/texture.c)
of textures/imagemap.cpp, core/mipmap.h and UVMapping2D; bump-mapped tessellation against the
oracle; the scene loader's Texture directive. All bit-exact: both sides run the same float
operations (the EWA weight table and log2 are double-evaluated transcendentals rounded once).

The reference ships no texture images or golden lookups (S007Scene.pbrt names textures that are
absent from the snapshot), so these lookups are parity-unpinned against the reference itself;
the synthetic images are seeded (synth.texture_texels)."""
import os

import numpy as np
import pytest

import oracle_render as orr
import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = [
    dict(texels=synth.texture_texels(37, 21, seed=1)),                                  # Lanczos resampling
    dict(texels=synth.texture_texels(64, 32, seed=2), wrap="clamp", gamma=2.2, scale=2.0),  # S007's diffuse map
    dict(texels=synth.texture_texels(50, 50, seed=3), wrap="black", shift=-0.5, scale=0.01),
    dict(texels=synth.texture_texels(33, 65, seed=4), trilinear=True, uscale=3.0, vscale=0.5, udelta=0.1),
    dict(texels=synth.texture_texels(40, 24, seed=5), is_float=True, gamma=2.2, maxanisotropy=4.0),
    dict(texels=synth.texture_texels(1, 1, seed=6)),
    dict(texels=None, scale=2.0, gamma=2.2),                                           # file not readable
    dict(texels=None, is_float=True, shift=-0.5, scale=0.01),
]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_imagemap_lookup_bit_exact(mpss, oracle, case):
    tex = CASES[case]
    uvd = synth.random_uvd(4000, seed=10 + case)
    got = mpss.host_imagemap_lookup(tex, uvd)
    ref = orr.imagemap_lookup(tex, uvd)
    assert np.isfinite(ref).all()
    assert np.array_equal(got, ref), "max |diff| %g" % np.abs(got - ref).max()
    if tex.get("is_float"):
        assert not got[:, 1:].any()


def test_imagemap_one_valued(mpss, oracle):
    """An unreadable file: MIPMap(1, 1, powf(scale * (1 + shift), gamma)) (imagemap.cpp:76-81);
    the bilinear (no differentials) lookup returns it exactly."""
    uvd = np.zeros((3, 6), np.float32)
    uvd[:, :2] = [[0.1, 0.2], [0.5, 0.5], [0.9, 0.7]]
    got = mpss.host_imagemap_lookup(dict(texels=None, scale=2.0, gamma=2.2), uvd)
    one = np.float32(np.power(np.float64(np.float32(2.0) * np.float32(1.0)), np.float64(np.float32(2.2))))
    assert np.all(got == one)


def test_imagemap_constant_image_is_preserved(mpss):
    """Filtering a constant image keeps the constant to rounding (EWA weights sum to sumWts)."""
    tex = dict(texels=np.full((16, 16, 3), 0.25, np.float32))
    got = mpss.host_imagemap_lookup(tex, synth.random_uvd(2000, seed=3))
    np.testing.assert_allclose(got, 0.25, rtol=1e-5)


def _bumped_mesh():
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin.pbrt"))
    return sc, sc.meshes[0]


@pytest.mark.parametrize("incenter", [False, True])
def test_bumped_tessellation_bit_exact(mpss, oracle, incenter):
    """TessellateSurfacePoints with a "bumpmap" (BumpMapping::Bump, trianglemesh.cpp:240-245; the
    fork's central differences, material.cpp:47-104) vs the oracle; the bump changes normals only."""
    sc, me = _bumped_mesh()
    bump = dict(texels=synth.texture_texels(48, 40, seed=9), is_float=True, scale=0.05, shift=-0.5)
    sc.materials[0]["bump_tex"] = bump
    sc.integrator["minsampledistance"] = 0.02
    det = np.linalg.det(np.asarray(me["o2w"], np.float64)[:3, :3])
    flip = bool(me["reverse"]) ^ bool(det < 0)
    args = (me["P"], me["indices"], me["o2w"], me["w2o"], 0.02)
    kw = dict(N=me["N"], S=me["S"], uv=me["uv"], flip=flip, incenter=incenter)
    got = mpss.host_tessellate(*args, bump=bump, **kw)
    plain = mpss.host_tessellate(*args, **kw)
    o = orr.OracleScene(sc, orr.tables_from_host(sc, mpss), mpss.default_config(
        min_sample_distance=0.02, max_error=0.1), mpss)
    ref = o.tessellate(incenter)
    o.close()
    assert got.tobytes() == ref.tobytes()
    assert np.array_equal(got["p"], plain["p"]) and np.array_equal(got["u"], plain["u"])
    moved = np.abs(got["n"] - plain["n"]).max(axis=1) > 1e-6
    assert moved.mean() > 0.3  # the bump map really tilts the normals
    assert np.allclose(np.linalg.norm(got["n"], axis=1), 1, atol=1e-5)


def test_scene_loader_imagemap(mpss, tmp_path):
    """Texture "imagemap" in a scene file: a readable TGA becomes texels, an unreadable path the
    one-valued map; layeredskin's last "texture albedo" wins (ParamSet replaces by name)."""
    from mpss import pbrtscene
    img = (synth.texture_texels(6, 4, seed=2) * 255).astype(np.uint8)
    hdr = bytes([0, 0, 2, 0, 0, 0, 0, 0, 0, 0, 0, 0, 6, 0, 4, 0, 24, 0x20])  # top-left origin
    (tmp_path / "diff.tga").write_bytes(hdr + img[:, :, ::-1].tobytes())
    txt = open(os.path.join(ROOT, "scenes", "skin.pbrt")).read()
    txt = txt.replace('Material "layeredskin"',
                      'Texture "bumpy" "float" "imagemap" "string filename" "diff.tga" "float scale" 0.01\n'
                      '    Texture "gone" "color" "imagemap" "string filename" "missing.tga"\n'
                      '    Texture "diff" "color" "imagemap" "string filename" "diff.tga" "string wrap" "clamp"'
                      ' "float gamma" 2.2 "float scale" 2\n    Material "layeredskin" "texture albedo" "gone"'
                      ' "texture albedo" "diff" "texture bumpmap" "bumpy"')
    txt = txt.replace('"string npzfile" "head_mesh.npz"', '"string npzfile" "%s"' % os.path.join(
        ROOT, "scenes", "head_mesh.npz"))
    (tmp_path / "t.pbrt").write_text(txt)
    with pytest.warns(UserWarning):
        sc = pbrtscene.load(str(tmp_path / "t.pbrt"))
    m = sc.materials[0]
    assert m["albedo_tex"]["wrap"] == "clamp" and m["albedo_tex"]["gamma"] == 2.2
    assert m["albedo_tex"]["texels"].shape == (4, 6, 3)
    # ReadImageTGA hands the rows over bottom row first (imageio.cpp:236-247)
    np.testing.assert_allclose(m["albedo_tex"]["texels"], img[::-1] / 255.0, atol=1e-6)
    assert m["bump_tex"]["is_float"] and m["bump_tex"]["scale"] == np.float32(0.01)
