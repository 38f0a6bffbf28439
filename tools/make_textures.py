"""Synthetic skin textures for scenes/skin_textured.pbrt (the fork's S007 scene drives LayeredSkin's
"albedo" and "bumpmap" with imagemaps, scenes/BasicMeshScenes/S007Scene.pbrt:31-34,49-50, whose
image files are not in the reference snapshot). Deterministic: value noise of a fixed seed.

    python tools/make_textures.py   -> scenes/textures/skin_albedo.tga, skin_bump.tga

albedo: 512x512 RGB, a pale skin tone modulated by low-frequency blotches and small freckles;
bump: 256x256 grey, pores / fine wrinkles (the float imagemap takes the texel's average).
Both 8-bit uncompressed TGA (ReadImageTGA, imageio.cpp:214-256)."""
import os
import struct

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def value_noise(n, cells, rng):
    g = rng.random((cells + 1, cells + 1))
    x = np.linspace(0, cells, n, endpoint=False)
    i = x.astype(int)
    f = x - i
    f = f * f * (3 - 2 * f)
    a = g[i][:, i] * (1 - f)[None, :] + g[i][:, i + 1] * f[None, :]
    b = g[i + 1][:, i] * (1 - f)[None, :] + g[i + 1][:, i + 1] * f[None, :]
    return a * (1 - f)[:, None] + b * f[:, None]


def fbm(n, rng, octaves):
    out = np.zeros((n, n))
    amp, tot = 1.0, 0.0
    for o in range(octaves):
        out += amp * value_noise(n, 4 << o, rng)
        tot += amp
        amp *= 0.5
    return out / tot


def write_tga(path, rgb8):
    h, w, _ = rgb8.shape
    hdr = struct.pack("<BBBHHBHHHHBB", 0, 0, 2, 0, 0, 0, 0, 0, w, h, 24, 0x20)  # top-left origin
    with open(path, "wb") as f:
        f.write(hdr)
        f.write(np.ascontiguousarray(rgb8[..., ::-1]).tobytes())


def main():
    rng = np.random.default_rng(0x5EED)
    n = 512
    base = np.array([0.80, 0.62, 0.52])
    blot = fbm(n, rng, 5)
    freck = np.clip((fbm(n, rng, 7) - 0.62) * 6.0, 0, 1)
    alb = base[None, None, :] * (0.85 + 0.3 * blot[..., None]) * (1 - 0.35 * freck[..., None] * np.array([0.5, 0.8, 0.9]))
    write_tga(os.path.join(ROOT, "scenes", "textures", "skin_albedo.tga"),
              np.clip(np.round(alb * 255), 0, 255).astype(np.uint8))
    m = 256
    bump = 0.5 + 0.35 * (fbm(m, rng, 6) - 0.5) + 0.15 * (value_noise(m, 96, rng) - 0.5)
    g = np.clip(np.round(bump * 255), 0, 255).astype(np.uint8)
    write_tga(os.path.join(ROOT, "scenes", "textures", "skin_bump.tga"), np.repeat(g[..., None], 3, axis=2))


if __name__ == "__main__":
    main()
