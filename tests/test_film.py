"""ImageFilm::WriteImage and the image writers (film/image.cpp:178-213; core/imageio.cpp:77-104,
156-208, 404-445; core/targa.c:467-618) on the CPU: finalize() bit-exact against a scalar
restatement of the per-pixel loop, and each writer's file read back (PFM and TGA byte layouts
checked field by field, EXR through this package's scanline reader)."""
import struct

import numpy as np
import pytest

from mpss import film, imageio

XYZ2RGB = [[3.240479, -1.537150, -0.498535], [-0.969256, 1.875991, 0.041556], [0.055648, -0.204043, 1.057311]]


def write_image_scalar(xyzw, splat, splat_scale):
    """ImageFilm::WriteImage's loop, one float32 operation at a time."""
    f = np.float32
    h, w, _ = xyzw.shape
    out = np.zeros((h, w, 3), np.float32)
    for y in range(h):
        for x in range(w):
            L = xyzw[y, x]
            rgb = [f(f(f(XYZ2RGB[r][0]) * L[0]) - f(f(-XYZ2RGB[r][1]) * L[1])) for r in range(3)]
            rgb = [f(rgb[r] + f(f(XYZ2RGB[r][2]) * L[2])) for r in range(3)]
            ws = L[3]
            if ws != 0:
                inv = f(f(1) / ws)
                rgb = [max(f(0), f(c * inv)) for c in rgb]
            s = splat[y, x]
            srgb = [f(f(f(XYZ2RGB[r][0]) * s[0]) + f(f(XYZ2RGB[r][1]) * s[1])) for r in range(3)]
            srgb = [f(srgb[r] + f(f(XYZ2RGB[r][2]) * s[2])) for r in range(3)]
            out[y, x] = [f(rgb[r] + f(f(splat_scale) * srgb[r])) for r in range(3)]
    return out


@pytest.mark.parametrize("splat_scale", [1.0, 0.25])
def test_finalize_matches_write_image_loop(splat_scale):
    rng = np.random.default_rng(5)
    xyzw = (rng.standard_normal((9, 13, 4)) * 3).astype(np.float32)
    xyzw[..., 3] = np.abs(xyzw[..., 3])
    xyzw[2, 3, 3] = 0.0  # weightSum == 0: no normalisation, no clamp
    xyzw[4, :, 3] = 0.0
    splat = (rng.standard_normal((9, 13, 3)) * 0.1).astype(np.float32)
    got = film.finalize(xyzw, splat, splat_scale)
    ref = write_image_scalar(xyzw, splat, splat_scale)
    assert np.array_equal(got, ref)
    # no splats (this integrator): the plain form
    assert np.array_equal(film.finalize(xyzw), write_image_scalar(xyzw, np.zeros_like(splat), 1.0))


def test_write_pfm_layout(tmp_path):
    rng = np.random.default_rng(1)
    rgb = rng.random((5, 7, 3)).astype(np.float32)
    p = str(tmp_path / "a.pfm")
    film.write_image(p, rgb)
    data = open(p, "rb").read()
    head = b"PF\n7 5\n-1.000000\n"
    assert data.startswith(head)
    body = np.frombuffer(data[len(head):], "<f4").reshape(5, 7, 3)
    assert np.array_equal(body, rgb[::-1])        # rows bottom to top (imageio.cpp:433-437)
    assert np.array_equal(film.read_pfm(p), rgb)
    # the reference's reader keeps FILE order (ReadImagePFM does not flip)
    assert np.array_equal(imageio.read_pfm_texels(p), rgb[::-1])


def test_write_tga_layout(tmp_path):
    rng = np.random.default_rng(2)
    rgb = (rng.random((6, 4, 3)) * 1.3 - 0.1).astype(np.float32)
    p = str(tmp_path / "a.tga")
    film.write_image(p, rgb)
    d = open(p, "rb").read()
    idl, cmt, typ, cmo, cml, cmd, ox, oy, w, h, bpp, desc = struct.unpack("<BBBHHBHHHHBB", d[:18])
    assert (idl, cmt, typ, cmo, cml, cmd, ox, oy, w, h, bpp, desc) == (0, 0, 2, 0, 0, 0, 0, 0, 4, 6, 24, 0x20)
    assert d[-26:] == b"\0" * 8 + b"TRUEVISION-XFILE.\0"
    px = np.frombuffer(d[18:18 + 6 * 4 * 3], np.uint8).reshape(6, 4, 3)
    exp = film.tga_bytes(rgb)
    assert np.array_equal(px, exp[..., ::-1])     # BGR, top row first
    # TO_BYTE truncates: 255 * v^(1/2.2) within one count of the float64 value, clamped
    v64 = 255 * np.clip(rgb.astype(np.float64), 0, None) ** (1 / 2.2)
    assert np.all(np.abs(exp - np.clip(np.floor(v64), 0, 255)) <= 1)
    assert exp[rgb <= 0].max(initial=0) == 0 and exp[rgb >= 1].min(initial=255) == 255


@pytest.mark.parametrize("compression", ["zip", "none"])
def test_write_exr_round_trip(tmp_path, compression):
    rng = np.random.default_rng(3)
    rgb = (rng.random((37, 21, 3)) * 40).astype(np.float32)
    rgb[0, 0] = [1e-8, 70000.0, 0.0]  # half subnormal / overflow to inf
    p = str(tmp_path / "a.exr")
    film.write_exr(p, rgb, total_res=(64, 48), offset=(5, 3), compression=compression)
    back = imageio.read_exr(p)
    with np.errstate(over="ignore"):
        assert np.array_equal(back, rgb.astype(np.float16).astype(np.float32))
    d = open(p, "rb").read()
    assert b"dataWindow\0box2i\0" + struct.pack("<iiiii", 16, 5, 3, 5 + 21 - 1, 3 + 37 - 1) in d
    assert b"displayWindow\0box2i\0" + struct.pack("<iiiii", 16, 0, 0, 63, 47) in d
    for c in (b"A\0", b"B\0", b"G\0", b"R\0"):
        assert c + struct.pack("<i", 1) in d      # HALF channels (WRITE_RGBA)
    if compression == "zip":
        assert len(d) < 37 * 21 * 4 * 2           # compressed blocks of 16 lines


def test_write_image_dispatch(tmp_path):
    rgb = np.ones((2, 2, 3), np.float32)
    film.write_image(str(tmp_path / "b.PFM"), rgb)
    assert (tmp_path / "b.PFM").read_bytes().startswith(b"PF\n")
    with pytest.raises(ValueError):
        film.write_image(str(tmp_path / "b.png"), rgb)


def test_exrdiff_restatement():
    """exrdiff.cpp:73-109: per-value relative difference thresholds (0.5 %, 5 %) and the mean-delta
    tolerance (-d, percent)."""
    from mpss import film
    a = np.ones((4, 5, 3), np.float32)
    b = a.copy()
    r = film.exrdiff(a, b)
    assert not r["differ"] and r["small"] == 0 and r["avg_delta_pct"] == 0.0
    b[0, 0, 0] = 1.01   # 1 % off: small only
    b[1, 1, 1] = 1.1    # 10 % off: small and big
    r = film.exrdiff(a, b)
    assert r["differ"] and r["small"] == 2 and r["big"] == 1
    assert r["avg_delta_pct"] == pytest.approx(-100 * (0.01 + 0.1) / 60 / (1 + 0.11 / 60), rel=1e-2)
    assert not film.exrdiff(a, b, tol=0.5)["differ"] and film.exrdiff(a, b, tol=0.1)["differ"]
    z = np.zeros_like(a)
    assert film.exrdiff(z, z)["small"] == 0  # zero in both: skipped
