"""ReadImage for environment maps (core/imageio.cpp:54-75): the texel array, in the row order
the reference hands to the MIPMap, for the three formats it reads.

  .exr  ReadImageEXR (imageio.cpp:120-150): R, G, B read through OpenEXR HALF slices (float
        channels are rounded to half), missing channels 0, rows top to bottom. Scanline files
        with NONE, RLE, ZIPS or ZIP compression are decoded here; PIZ/PXR24/B44/DWA and tiled
        files raise (the reference links OpenEXR, this package does not).
  .pfm  ReadImagePFM (imageio.cpp:318-395): rows in FILE order (no flip), |scale| != 1
        multiplies, a negative scale means little endian; "Pf" replicates the grey value.
  .tga  ReadImageTGA (imageio.cpp:214-256): 8-bit channels / 255, rows bottom to top after the
        top-to-bottom flip; types 2, 3, 10, 11 (no colour maps).

Returns an (H, W, 3) float32 array: row 0 is the texel row t = 0 of the radiance map.
"""
import struct
import zlib

import numpy as np


def read_image(path):
    low = path.lower()
    if low.endswith(".exr"):
        return read_exr(path)
    if low.endswith(".pfm"):
        return read_pfm_texels(path)
    if low.endswith(".tga"):
        return read_tga(path)
    raise ValueError("can't determine image file type from suffix of filename %r" % path)


# ------------------------------------------------------------------ PFM
def read_pfm_texels(path):
    data = open(path, "rb").read()
    pos = 0
    words = []
    while len(words) < 4:  # readWord: skip whitespace, read to the next whitespace, consume it
        while pos < len(data) and data[pos:pos + 1].isspace():
            pos += 1
        start = pos
        while pos < len(data) and not data[pos:pos + 1].isspace():
            pos += 1
        words.append(data[start:pos].decode("ascii"))
        pos += 1
    kind, w, h, scale = words[0], int(words[1]), int(words[2]), float(words[3])
    if kind not in ("PF", "Pf"):
        raise ValueError("error reading PFM file %r" % path)
    nch = 3 if kind == "PF" else 1
    n = nch * w * h
    arr = np.frombuffer(data, "<f4" if scale < 0 else ">f4", count=n, offset=pos).astype(np.float32)
    if abs(np.float32(scale)) != 1.0:
        arr = (arr * np.float32(abs(scale))).astype(np.float32)
    arr = arr.reshape(h, w, nch)
    if nch == 1:
        arr = np.repeat(arr, 3, axis=2)
    return np.ascontiguousarray(arr)


# ------------------------------------------------------------------ TGA
def read_tga(path):
    d = open(path, "rb").read()
    idlen, cmtype, itype = d[0], d[1], d[2]
    w, h = struct.unpack("<HH", d[12:16])
    bpp, desc = d[16], d[17]
    if cmtype != 0 or itype not in (2, 3, 10, 11):
        raise ValueError("TGA %r: only uncompressed / RLE true-colour or grey images are supported" % path)
    nb = bpp // 8
    pos = 18 + idlen
    npx = w * h
    if itype in (2, 3):
        px = np.frombuffer(d, np.uint8, count=npx * nb, offset=pos).reshape(npx, nb)
    else:
        out = bytearray()
        while len(out) < npx * nb:
            c = d[pos]
            pos += 1
            cnt = (c & 0x7F) + 1
            if c & 0x80:
                out += d[pos:pos + nb] * cnt
                pos += nb
            else:
                out += d[pos:pos + nb * cnt]
                pos += nb * cnt
        px = np.frombuffer(bytes(out[:npx * nb]), np.uint8).reshape(npx, nb)
    img = px.reshape(h, w, nb)
    if desc & 0x10:  # right to left
        img = img[:, ::-1]
    if not (desc & 0x20):  # bottom to top: flip to top to bottom
        img = img[::-1]
    img = img[::-1]  # the reader's loop walks y = height-1 .. 0
    if nb == 1:
        g = img[..., 0].astype(np.float32) / np.float32(255)
        return np.ascontiguousarray(np.stack([g, g, g], -1))
    rgb = np.stack([img[..., 2], img[..., 1], img[..., 0]], -1).astype(np.float32) / np.float32(255)
    return np.ascontiguousarray(rgb.astype(np.float32))


# ------------------------------------------------------------------ OpenEXR (scanline subset)
_PIX = {0: (np.dtype("<u4"), 4), 1: (np.dtype("<f2"), 2), 2: (np.dtype("<f4"), 4)}
_LINES = {0: 1, 1: 1, 2: 1, 3: 16}


def _undo_predictor_interleave(t):
    t = np.frombuffer(t, np.uint8).astype(np.int32)
    t = ((np.cumsum(t - 128) + 128) & 0xFF).astype(np.uint8)  # t[i] = t[i-1] + t[i] - 128
    n = len(t)
    half = (n + 1) // 2
    out = np.empty(n, np.uint8)
    out[0::2] = t[:half]
    out[1::2] = t[half:]
    return out.tobytes()


def _rle_decode(src, expect):
    out = bytearray()
    i = 0
    while i < len(src) and len(out) < expect:
        c = struct.unpack("b", src[i:i + 1])[0]
        i += 1
        if c < 0:
            out += src[i:i - c]
            i += -c
        else:
            out += src[i:i + 1] * (c + 1)
            i += 1
    return bytes(out)


def read_exr(path):
    d = open(path, "rb").read()
    magic, ver = struct.unpack("<ii", d[:8])
    if magic != 20000630:
        raise ValueError("%r is not an OpenEXR file" % path)
    if ver & 0x200:
        raise ValueError("EXR %r: tiled files are not supported" % path)
    if ver & 0x1000:
        raise ValueError("EXR %r: multi-part files are not supported" % path)
    pos = 8
    hdr = {}
    while d[pos] != 0:
        e = d.index(b"\0", pos)
        name = d[pos:e].decode()
        e2 = d.index(b"\0", e + 1)
        typ = d[e + 1:e2].decode()
        size = struct.unpack("<i", d[e2 + 1:e2 + 5])[0]
        hdr[name] = (typ, d[e2 + 5:e2 + 5 + size])
        pos = e2 + 5 + size
    pos += 1
    chans = []
    cl = hdr["channels"][1]
    i = 0
    while cl[i] != 0:
        e = cl.index(b"\0", i)
        nm = cl[i:e].decode()
        ptype, _lin, xs, ys = struct.unpack("<iB3xii", cl[e + 1:e + 17])
        if xs != 1 or ys != 1:
            raise ValueError("EXR %r: subsampled channels are not supported" % path)
        chans.append((nm, ptype))
        i = e + 17
    comp = hdr["compression"][1][0]
    if comp not in _LINES:
        raise ValueError("EXR %r: compression %d is not supported (NONE, RLE, ZIPS, ZIP only)" % (path, comp))
    x0, y0, x1, y1 = struct.unpack("<iiii", hdr["dataWindow"][1])
    w, h = x1 - x0 + 1, y1 - y0 + 1
    lpb = _LINES[comp]
    nblocks = (h + lpb - 1) // lpb
    offsets = struct.unpack("<%dQ" % nblocks, d[pos:pos + 8 * nblocks])
    planes = {nm: np.zeros((h, w), np.float32) for nm, _ in chans}
    for off in offsets:
        yb, size = struct.unpack("<ii", d[off:off + 8])
        raw = d[off + 8:off + 8 + size]
        nl = min(lpb, y1 - yb + 1)
        expect = sum(_PIX[pt][1] for _, pt in chans) * w * nl
        if size < expect:
            if comp == 1:
                raw = _undo_predictor_interleave(_rle_decode(raw, expect))
            elif comp in (2, 3):
                raw = _undo_predictor_interleave(zlib.decompress(raw))
        if len(raw) != expect:
            raise ValueError("EXR %r: corrupt block at line %d" % (path, yb))
        p = 0
        for li in range(nl):
            for nm, pt in chans:
                dt, nbt = _PIX[pt]
                row = np.frombuffer(raw, dt, count=w, offset=p)
                planes[nm][yb - y0 + li] = row.astype(np.float32)
                p += nbt * w

    def half_slice(nm):  # Slice(HALF, ...): every channel type converts to half; missing -> 0.0
        if nm not in planes:
            return np.zeros((h, w), np.float32)
        return planes[nm].astype(np.float16).astype(np.float32)

    return np.ascontiguousarray(np.stack([half_slice("R"), half_slice("G"), half_slice("B")], -1))
