"""ImageFilm finalisation and image files (film/image.cpp:150-213 WriteImage, core/imageio.cpp).

Tiles come back from mpss_render_tile as float4 {sum X, sum Y, sum Z, sum of filter weights}
per pixel (ImageFilm::Pixel). finalize() performs WriteImage's per-pixel XYZToRGB, division by
the weight sum and clamp at 0; write_pfm() is the float PFM writer (imageio.cpp:156-170 path for
".pfm"), write_exr() a minimal uncompressed half-float OpenEXR writer (the reference writes EXR
through OpenEXR's RgbaOutputFile, imageio.cpp).
"""
import struct

import numpy as np

# XYZToRGB, core/spectrum.h
_XYZ2RGB = np.array([[3.240479, -1.537150, -0.498535],
                     [-0.969256, 1.875991, 0.041556],
                     [0.055648, -0.204043, 1.057311]], np.float32)


def xyz_to_rgb(xyz):
    x, y, z = (xyz[..., i].astype(np.float32) for i in range(3))
    m = _XYZ2RGB
    r = m[0, 0] * x + m[0, 1] * y + m[0, 2] * z
    g = m[1, 0] * x + m[1, 1] * y + m[1, 2] * z
    b = m[2, 0] * x + m[2, 1] * y + m[2, 2] * z
    return np.stack([r, g, b], -1).astype(np.float32)


def finalize(xyzw):
    """xyzw: [H, W, 4] float32 -> RGB [H, W, 3] (WriteImage, image.cpp:150-213)."""
    xyzw = np.asarray(xyzw, np.float32)
    rgb = xyz_to_rgb(xyzw[..., :3])
    w = xyzw[..., 3:4]
    safe = np.where(w != 0, w, np.float32(1))
    inv = (np.float32(1) / safe).astype(np.float32)
    out = np.where(w != 0, np.maximum(np.float32(0), rgb * inv), rgb)
    return out.astype(np.float32)


def write_pfm(path, rgb):
    """Float PFM: "PF", width height, scale -1 (little endian), rows bottom to top."""
    rgb = np.asarray(rgb, np.float32)
    h, w, _ = rgb.shape
    with open(path, "wb") as f:
        f.write(b"PF\n%d %d\n-1\n" % (w, h))
        f.write(np.ascontiguousarray(rgb[::-1]).astype("<f4").tobytes())


def read_pfm(path):
    with open(path, "rb") as f:
        assert f.readline().strip() == b"PF"
        w, h = map(int, f.readline().split())
        s = float(f.readline())
        data = np.frombuffer(f.read(), "<f4" if s < 0 else ">f4").reshape(h, w, 3)
    return data[::-1].astype(np.float32)


def write_exr(path, rgb):
    """Scanline, uncompressed, HALF R/G/B OpenEXR (the reference's output format)."""
    rgb = np.asarray(rgb, np.float32)
    h, w, _ = rgb.shape

    def attr(name, typ, data):
        return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(data)) + data

    chans = b"".join(c.encode() + b"\0" + struct.pack("<iB3xii", 1, 0, 1, 1) for c in "BGR") + b"\0"
    hdr = struct.pack("<ii", 20000630, 2)
    hdr += attr("channels", "chlist", chans)
    hdr += attr("compression", "compression", b"\0")
    hdr += attr("dataWindow", "box2i", struct.pack("<iiii", 0, 0, w - 1, h - 1))
    hdr += attr("displayWindow", "box2i", struct.pack("<iiii", 0, 0, w - 1, h - 1))
    hdr += attr("lineOrder", "lineOrder", b"\0")
    hdr += attr("pixelAspectRatio", "float", struct.pack("<f", 1.0))
    hdr += attr("screenWindowCenter", "v2f", struct.pack("<ff", 0.0, 0.0))
    hdr += attr("screenWindowWidth", "float", struct.pack("<f", 1.0))
    hdr += b"\0"
    line_bytes = w * 3 * 2
    table_off = len(hdr)
    first = table_off + 8 * h
    offsets = [first + y * (8 + line_bytes) for y in range(h)]
    half = rgb.astype(np.float16)
    with open(path, "wb") as f:
        f.write(hdr)
        f.write(struct.pack("<%dQ" % h, *offsets))
        for y in range(h):
            row = half[y]
            f.write(struct.pack("<ii", y, line_bytes))
            for c in (2, 1, 0):  # channels in alphabetical order: B, G, R
                f.write(row[:, c].astype("<f2").tobytes())
