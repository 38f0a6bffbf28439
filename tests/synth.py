"""Seeded synthetic inputs shared by the parity tests and bench.py."""
import numpy as np

NB = 30


def smooth_spectra(n, seed=1, black_frac=0.0):
    """E_c = s * (0.5 + 0.5 sin(0.1 c + phi)), s ~ U[0,1)."""
    rng = np.random.default_rng(seed)
    s = rng.random(n, dtype=np.float32)
    phi = rng.random(n, dtype=np.float32) * np.float32(6.2831853)
    c = np.arange(NB, dtype=np.float32)
    E = (s[:, None] * (np.float32(0.5) + np.float32(0.5) * np.sin(np.float32(0.1) * c[None, :] + phi[:, None])))
    E = E.astype(np.float32)
    if black_frac > 0:
        E[rng.random(n) < black_frac] = 0.0
    return E


def ellipsoid_cloud(n, radii=(0.25, 0.3, 0.35), seed=7, black_frac=0.05):
    """Irradiance points on an ellipsoid surface: p, n, E, area."""
    rng = np.random.default_rng(seed)
    v = rng.standard_normal((n, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    r = np.asarray(radii)
    p = (v * r).astype(np.float32)
    nrm = v / (r * r)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    area_total = 4 * np.pi * (np.prod(r) ** (2 / 3))
    area = np.full(n, area_total / n, np.float32) * (0.5 + rng.random(n).astype(np.float32))
    return p, nrm.astype(np.float32), smooth_spectra(n, seed + 1, black_frac), area.astype(np.float32)


def surface_queries(q, radii=(0.25, 0.3, 0.35), seed=11, jitter=0.0, sort=True):
    rng = np.random.default_rng(seed)
    v = rng.standard_normal((q, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    p = v * np.asarray(radii)
    if jitter:
        p += rng.standard_normal((q, 3)) * jitter
    p = p.astype(np.float32)
    if sort:  # Morton order: neighbouring queries share octree paths, like a pixel's samples
        p = p[np.argsort(morton3(p), kind="stable")]
    return np.ascontiguousarray(p)


def morton3(p, bits=10):
    """30-bit Morton code of points quantised over their bounding box."""
    lo = p.min(0)
    span = np.maximum(p.max(0) - lo, 1e-30)
    q = np.minimum(((p - lo) / span * (1 << bits)).astype(np.uint64), (1 << bits) - 1)
    code = np.zeros(len(p), np.uint64)
    for b in range(bits):
        for a in range(3):
            code |= ((q[:, a] >> np.uint64(b)) & np.uint64(1)) << np.uint64(3 * b + a)
    return code


def texture_texels(w, h, seed=3, lo=0.05, hi=1.0):
    """A (h, w, 3) RGB image like a skin diffuse map: smooth colour bands plus per-texel noise,
    values in [lo, hi) (ReadImage's float texels)."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    base = np.stack([0.5 + 0.4 * np.sin(x / max(w, 1) * 6.3 + k + y / max(h, 1) * 2.1) for k in range(3)], -1)
    img = lo + (hi - lo) * np.clip(0.8 * base + 0.2 * rng.random((h, w, 3)), 0, 0.999)
    return img.astype(np.float32)


def random_uvd(n, seed=5, scale=0.02, outside=0.1):
    """(n, 6) lookup points u, v, dudx, dvdx, dudy, dvdy: u, v partly outside [0, 1) (wrap
    modes), differentials log-uniform over ~4 decades of `scale`, a share of them zero
    (the irradiance / tessellation lookups) and a share strongly anisotropic."""
    rng = np.random.default_rng(seed)
    uv = rng.uniform(-outside, 1 + outside, (n, 2))
    d = rng.standard_normal((n, 4)) * scale * np.exp(rng.uniform(-4.5, 4.5, (n, 1)))
    d[rng.random(n) < 0.15] = 0.0
    an = rng.random(n) < 0.15
    d[an, 2:] *= 1e-3
    return np.concatenate([uv, d], 1).astype(np.float32)
