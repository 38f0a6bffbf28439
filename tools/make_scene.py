"""Convert the reference's head mesh (scenes/geometry/head.pbrt, a pbrt "trianglemesh" shape with
P / N / S / uv / indices) into scenes/head_mesh.npz, the geometry of the reconstructed
skin.pbrt (the scene files named by BASELINE.json are absent from the
reference snapshot; skin.pbrt = this mesh + S007Scene.pbrt's camera, light and layeredskin).

Run in the build container only (the GPU box has no /root/reference):
    python tools/make_scene.py [/root/reference/scenes/geometry/head.pbrt]
The arrays are stored exactly as parsed into float32 / int32 (pbrt's ParamSet parses numbers
with atof and stores floats, core/pbrtparse.yy).
"""
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def parse_trianglemesh(path):
    txt = open(path).read()
    out = {}
    for m in re.finditer(r'"(point|normal|vector|float|integer)\s+(\w+)"\s*\[([^\]]*)\]', txt):
        typ, name, body = m.groups()
        vals = body.split()
        if typ == "integer":
            out[name] = np.array([int(v) for v in vals], np.int32)
        else:
            out[name] = np.array([float(v) for v in vals], np.float64).astype(np.float32)
    return out


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/scenes/geometry/head.pbrt"
    d = parse_trianglemesh(src)
    P = d["P"].reshape(-1, 3)
    idx = d["indices"].reshape(-1, 3)
    N = d["N"].reshape(-1, 3)
    S = d["S"].reshape(-1, 3)
    uv = d["uv"].reshape(-1, 2)
    assert len(N) == len(P) and len(S) == len(P) and len(uv) == len(P)
    assert idx.min() >= 0 and idx.max() < len(P)
    dst = os.path.join(ROOT, "scenes", "head_mesh.npz")
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    np.savez_compressed(dst, P=P, N=N, S=S, uv=uv, indices=idx)
    print("wrote %s: %d vertices, %d triangles" % (dst, len(P), len(idx)))


if __name__ == "__main__":
    main()
