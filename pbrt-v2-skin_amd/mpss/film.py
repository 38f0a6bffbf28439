"""ImageFilm finalisation and the image writers (film/image.cpp:178-213 WriteImage,
core/imageio.cpp:77-104 ::WriteImage and its EXR / TGA / PFM writers).

Tiles come back from mpss_render_tile as float4 {sum X, sum Y, sum Z, sum of filter weights}
per pixel (ImageFilm::Pixel, image.h:69-78). finalize() is ImageFilm::WriteImage's per-pixel
pass: XYZToRGB, then, for a non-zero weight sum, multiplication by 1 / weightSum and max(0, .),
then the splat term splatScale * XYZToRGB(splatXYZ) (zero for this integrator: nothing splats).
write_image() dispatches on the suffix like ::WriteImage:

  .exr  WriteImageEXR (imageio.cpp:156-178): RgbaOutputFile with WRITE_RGBA, i.e. HALF channels
        A (= 1), B, G, R, ZIP compression (RgbaOutputFile's default), INCREASING_Y, display
        window (0,0)-(totalXRes-1, totalYRes-1) and data window at the crop offset;
  .tga  WriteImageTGA (imageio.cpp:185-208): BGR bytes uint8(Clamp(255 powf(v, 1/2.2), 0, 255)),
        uncompressed true colour, top-to-bottom descriptor bit, TRUEVISION-XFILE footer
        (targa.c:467-553, 567-618);
  .pfm  WriteImagePFM (imageio.cpp:404-445): "PF\\n", "%d %d\\n", "%f\\n" of -1 (little endian),
        rows bottom to top.
"""
import struct
import zlib

import numpy as np

# XYZToRGB, core/spectrum.h:51-55
_XYZ2RGB = np.array([[3.240479, -1.537150, -0.498535],
                     [-0.969256, 1.875991, 0.041556],
                     [0.055648, -0.204043, 1.057311]], np.float32)


def xyz_to_rgb(xyz):
    """rgb[0] = 3.240479f*x - 1.537150f*y - 0.498535f*z, ... in float, left to right."""
    x, y, z = (np.asarray(xyz)[..., i].astype(np.float32) for i in range(3))
    m = _XYZ2RGB
    out = []
    for r in range(3):
        acc = (m[r, 0] * x).astype(np.float32)
        acc = (acc + (m[r, 1] * y).astype(np.float32)).astype(np.float32)
        acc = (acc + (m[r, 2] * z).astype(np.float32)).astype(np.float32)
        out.append(acc)
    return np.stack(out, -1).astype(np.float32)


def finalize(xyzw, splat_xyz=None, splat_scale=1.0):
    """xyzw: [H, W, 4] float32 (Lxyz, weightSum) -> RGB [H, W, 3] (ImageFilm::WriteImage)."""
    xyzw = np.asarray(xyzw, np.float32)
    rgb = xyz_to_rgb(xyzw[..., :3])
    w = xyzw[..., 3:4]
    safe = np.where(w != 0, w, np.float32(1))
    inv = (np.float32(1) / safe).astype(np.float32)
    out = np.where(w != 0, np.maximum(np.float32(0), (rgb * inv).astype(np.float32)), rgb).astype(np.float32)
    splat = xyz_to_rgb(np.zeros_like(xyzw[..., :3]) if splat_xyz is None else splat_xyz)
    return (out + (np.float32(splat_scale) * splat).astype(np.float32)).astype(np.float32)


def write_image(path, rgb, total_res=None, offset=(0, 0)):
    """::WriteImage (imageio.cpp:77-104): by suffix (.exr, .tga, .pfm; upper case too)."""
    low = path[-4:].lower() if len(path) >= 5 else ""
    if low == ".exr":
        return write_exr(path, rgb, total_res, offset)
    if low == ".tga":
        return write_tga(path, rgb)
    if low == ".pfm":
        return write_pfm(path, rgb)
    raise ValueError("Can't determine image file type from suffix of filename %r" % path)


def write_pfm(path, rgb):
    """WriteImagePFM: "PF", width height, "%f" of the scale -1 (little endian), rows bottom to top."""
    rgb = np.asarray(rgb, np.float32)
    h, w, _ = rgb.shape
    with open(path, "wb") as f:
        f.write(b"PF\n%d %d\n%s\n" % (w, h, (b"%f" % -1.0)))
        f.write(np.ascontiguousarray(rgb[::-1]).astype("<f4").tobytes())


def read_pfm(path):
    """The image write_pfm wrote, row 0 = the top row."""
    with open(path, "rb") as f:
        assert f.readline().strip() == b"PF"
        w, h = map(int, f.readline().split())
        s = float(f.readline())
        data = np.frombuffer(f.read(), "<f4" if s < 0 else ">f4").reshape(h, w, 3)
    return data[::-1].astype(np.float32)


def tga_bytes(rgb):
    """TO_BYTE (imageio.cpp:195): uint8(Clamp(255.f * powf(v, 1.f/2.2f), 0.f, 255.f)); powf in double
    rounded once (the package's transcendental convention)."""
    v = np.asarray(rgb, np.float32)
    with np.errstate(invalid="ignore"):
        p = np.power(v.astype(np.float64), np.float64(np.float32(1.0) / np.float32(2.2))).astype(np.float32)
    x = (np.float32(255) * p).astype(np.float32)
    x = np.where(x < 0, np.float32(0), np.where(x > 255, np.float32(255), x))  # Clamp; NaN passes
    x = np.nan_to_num(x, nan=0.0)  # uint8(NaN) is undefined in C; 0 here
    return x.astype(np.uint8)


def write_tga(path, rgb):
    """WriteImageTGA -> tga_write_bgr(…, 24): 18-byte header, BGR rows top to bottom, footer."""
    b = tga_bytes(rgb)
    h, w, _ = b.shape
    hdr = struct.pack("<BBBHHBHHHHBB", 0, 0, 2, 0, 0, 0, 0, 0, w, h, 24, 0x20)
    with open(path, "wb") as f:
        f.write(hdr)
        f.write(np.ascontiguousarray(b[..., ::-1]).tobytes())
        f.write(b"\0" * 8 + b"TRUEVISION-XFILE.\0")


def _predict_interleave(raw):
    """OpenEXR ZIP/RLE pre-pass: split even/odd bytes, then byte deltas + 128."""
    a = np.frombuffer(raw, np.uint8)
    t = np.concatenate([a[0::2], a[1::2]]).astype(np.int32)
    d = t.copy()
    d[1:] = (t[1:] - t[:-1] + 128) & 0xFF
    return d.astype(np.uint8).tobytes()


def write_exr(path, rgb, total_res=None, offset=(0, 0), compression="zip"):
    """WriteImageEXR: scanline HALF A/B/G/R (alpha 1), ZIP (16 lines a block) or NONE."""
    rgb = np.asarray(rgb, np.float32)
    h, w, _ = rgb.shape
    tx, ty = total_res if total_res is not None else (w, h)
    ox, oy = offset
    comp = {"none": 0, "zip": 3}[compression]
    lpb = 16 if comp == 3 else 1

    def attr(name, typ, data):
        return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(data)) + data

    chans = b"".join(c.encode() + b"\0" + struct.pack("<iB3xii", 1, 0, 1, 1) for c in "ABGR") + b"\0"
    hdr = struct.pack("<ii", 20000630, 2)
    hdr += attr("channels", "chlist", chans)
    hdr += attr("compression", "compression", bytes([comp]))
    hdr += attr("dataWindow", "box2i", struct.pack("<iiii", ox, oy, ox + w - 1, oy + h - 1))
    hdr += attr("displayWindow", "box2i", struct.pack("<iiii", 0, 0, tx - 1, ty - 1))
    hdr += attr("lineOrder", "lineOrder", b"\0")
    hdr += attr("pixelAspectRatio", "float", struct.pack("<f", 1.0))
    hdr += attr("screenWindowCenter", "v2f", struct.pack("<ff", 0.0, 0.0))
    hdr += attr("screenWindowWidth", "float", struct.pack("<f", 1.0))
    hdr += b"\0"
    with np.errstate(over="ignore"):
        half = rgb.astype(np.float16)  # Rgba(float): round to nearest even, overflow to inf
    alpha = np.ones((h, w), np.float16)
    blocks = []
    for y0 in range(0, h, lpb):
        raw = b"".join(plane[y].astype("<f2").tobytes()
                       for y in range(y0, min(h, y0 + lpb))
                       for plane in (alpha, half[..., 2], half[..., 1], half[..., 0]))
        data = raw
        if comp == 3:
            z = zlib.compress(_predict_interleave(raw))
            data = z if len(z) < len(raw) else raw
        blocks.append(struct.pack("<ii", oy + y0, len(data)) + data)
    offs, pos = [], len(hdr) + 8 * len(blocks)
    for b in blocks:
        offs.append(pos)
        pos += len(b)
    with open(path, "wb") as f:
        f.write(hdr)
        f.write(struct.pack("<%dQ" % len(offs), *offs))
        for b in blocks:
            f.write(b)


def exrdiff(im1, im2, tol=0.0):
    """pbrt's exrdiff tool (src/tools/exrdiff.cpp:73-109) on two RGB(A) images as WriteImageEXR
    stores them (HALF channels, alpha 1): per channel value, skipping alpha and values that are 0
    in both, d = |a - b| / a counts as a small difference above 0.5 % and a big one above 5 %;
    avgDelta = (avg1 - avg2) / min(avg1, avg2) of the channel sums over 3 W H. The images "differ"
    (exrdiff exits 1) when tol == 0 and any small/big difference exists, or when tol > 0 and
    100 |avgDelta| > tol (tol in percent, the tool's -d). Returns the tool's report as a dict."""
    a = np.asarray(im1, np.float32)[..., :3].astype(np.float16).astype(np.float32)
    b = np.asarray(im2, np.float32)[..., :3].astype(np.float16).astype(np.float32)
    if a.shape != b.shape:
        raise ValueError("resolutions don't match: %s vs %s" % (a.shape, b.shape))
    h, w, _ = a.shape
    live = ~((a == 0) & (b == 0))
    av, bv = a[live].astype(np.float64), b[live].astype(np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        d = (np.abs(a[live] - b[live]) / a[live]).astype(np.float32)  # fabsf(...) / im1[i] in float
    small, big = int((d > 0.005).sum()), int((d > 0.05).sum())
    n3 = 3.0 * w * h
    avg1, avg2 = av.sum() / n3, bv.sum() / n3
    delta = (avg1 - avg2) / min(avg1, avg2)
    mse = float(((av - bv) ** 2).sum() / n3)
    differ = (tol == 0.0 and (big > 0 or small > 0)) or (tol > 0.0 and 100.0 * abs(delta) > tol)
    return {"differ": bool(differ), "small": small, "big": big, "small_pct": 100.0 * small / n3,
            "big_pct": 100.0 * big / n3, "avg1": avg1, "avg2": avg2, "avg_delta_pct": 100.0 * delta,
            "mse": mse, "rms_pct": 100.0 * np.sqrt(mse), "tol_pct": tol}
