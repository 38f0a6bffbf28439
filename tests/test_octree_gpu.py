"""The irradiance octree built on the GPU (octree_gpu.hip, the default) against the host build
(octree_on_host = 1: SubsurfaceOctreeNode::Insert in point order, diffusionutil.h:94-173) and the
oracle's restatement: the device arrays the gather reads (pre-order NodeHdr records, Et rows,
point records, point order) are compared bit for bit.
"""
import os

import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

NODE = np.dtype([("p", "<f4", 3), ("sum_area", "<f4"), ("bmin", "<f4", 3), ("bmax", "<f4", 3), ("skip", "<i4"),
                 ("leaf_first", "<i4"), ("leaf_count", "<i4"), ("depth", "<i4"), ("flags", "<u4"), ("pad", "<u4")])


def _export(mpss, on_host, p, n, E, area):
    ctx = mpss.Context(octree_on_host=on_host)
    ctx.set_irradiance_points(p, n, E, area)
    return ctx.octree_info(), ctx.octree_export()


def _same(a, b):
    for k in ("nodes", "node_et", "pt_hdr", "pt_e", "pt_index"):
        assert a[k].shape == b[k].shape, k
        assert a[k].tobytes() == b[k].tobytes(), k


def _clustered(n, seed):
    """Dense clumps at a few centres (deep subtrees), spread points and exact duplicates of <= 8."""
    rng = np.random.default_rng(seed)
    centres = rng.random((6, 3)).astype(np.float32)
    p = centres[rng.integers(0, 6, n)] + (rng.standard_normal((n, 3)) * 1e-4).astype(np.float32)
    p[: n // 4] = rng.random((n // 4, 3)).astype(np.float32)
    p[n // 4: n // 4 + 7] = p[n // 4 + 7]  # 8 coincident points fit one leaf
    nrm = np.tile(np.float32([0, 0, 1]), (n, 1))
    E = synth.smooth_spectra(n, seed=seed, black_frac=0.1)
    area = (rng.random(n) * 1e-4 + 1e-6).astype(np.float32)
    return p.astype(np.float32), nrm, E, area


CLOUDS = {
    "ellipsoid": lambda: synth.ellipsoid_cloud(50000, seed=21, black_frac=0.05),
    "clustered": lambda: _clustered(30000, 5),
    "one_leaf": lambda: synth.ellipsoid_cloud(8, seed=3, black_frac=0.25),
    "one_split": lambda: synth.ellipsoid_cloud(9, seed=4, black_frac=0.0),
    "all_black": lambda: synth.ellipsoid_cloud(1000, seed=6, black_frac=1.0),
}


@pytest.mark.parametrize("cloud", sorted(CLOUDS))
def test_gpu_build_matches_host_build(mpss, cloud):
    p, n, E, area = CLOUDS[cloud]()
    ig, g = _export(mpss, 0, p, n, E, area)
    ih, h = _export(mpss, 1, p, n, E, area)
    assert ig == ih
    _same(g, h)


def test_gpu_build_matches_oracle(mpss, oracle):
    p, n, E, area = synth.ellipsoid_cloud(40000, seed=22, black_frac=0.05)
    _, g = _export(mpss, 0, p, n, E, area)
    o = oracle.Octree(p, n, E, area).export()
    nodes = g["nodes"].view(NODE).reshape(-1)
    assert len(nodes) == len(o["p"])
    assert np.array_equal(nodes["p"], o["p"])
    assert np.array_equal(nodes["sum_area"], o["area"])
    assert np.array_equal(g["node_et"][:, :30], o["Et"])
    assert not g["node_et"][:, 30:].any()
    assert np.array_equal(nodes["depth"], o["depth"])
    assert np.array_equal(nodes["skip"], o["skip"])
    assert np.array_equal(nodes["leaf_count"], o["leaf_count"])
    leaf = o["leaf_count"] > 0
    assert np.array_equal(nodes["leaf_first"][leaf], o["leaf_first"][leaf])
    assert (nodes["leaf_first"][~leaf] == -1).all()
    # the device keeps each leaf's non-black points first (in slot order), then the black ones
    black = ~E.any(axis=1)
    want = np.empty_like(o["order"])
    for f, c in zip(o["leaf_first"][leaf], o["leaf_count"][leaf]):
        ids = o["order"][f:f + c]
        want[f:f + c] = np.concatenate([ids[~black[ids]], ids[black[ids]]])
        assert (nodes["pad"][nodes["leaf_first"] == f] & 0xffff).max() == (~black[ids]).sum()
    assert np.array_equal(g["pt_index"], want)
    assert np.array_equal(g["pt_hdr"][:, :3], p[want])
    assert np.array_equal(np.signbit(g["pt_hdr"][:, 3]), black[want])
    assert np.array_equal(np.abs(g["pt_hdr"][:, 3]), area[want])
    assert np.array_equal(g["pt_e"][:, :30], E[want])


def _leaf_code_bounds(nodes, max_error):
    """ensure_leaf_r2's bound (mo_kernel.hip leaf_r2_kernel, in double) as the leaf code the gather
    compares: its float's high 16 bits rounded up -- with a 1e-6 margin either way for the device's
    double sqrt. Interior nodes and leaves without area: +inf (code 0x7f80)."""
    b0, b1 = nodes["bmin"].astype(np.float64), nodes["bmax"].astype(np.float64)
    c = nodes["p"].astype(np.float64)
    diag = np.sqrt(((b1 - b0) ** 2).sum(axis=1))
    corner = np.sqrt((np.maximum(np.abs(c - b0), np.abs(c - b1)) ** 2).sum(axis=1))
    with np.errstate(invalid="ignore", divide="ignore"):
        opn = np.sqrt(nodes["sum_area"].astype(np.float64) / max_error) * (1 + 1e-6)
    R = np.maximum(opn + corner, diag)
    live = (nodes["leaf_first"] >= 0) & (nodes["sum_area"] > 0) & np.isfinite(c).all(axis=1)
    r2 = np.where(live, R * R * (1 + 1e-6), np.inf)

    def code(x):
        return (x.astype(np.float32).view(np.uint32).astype(np.uint64) + 0xffff) >> 16
    return code(r2 * (1 - 1e-6)), code(r2 * (1 + 1e-6))


def test_leaf_codes_in_node_headers(mpss):
    """NodeHdr::pad's high half (ensure_leaf_r2): the leaf's near-field bound as the 16-bit code the
    sharded gather's LDS-only leaf test compares (code < lim's code => bound < lim), next to the
    live-point count in the low half."""
    p, n, E, area = synth.ellipsoid_cloud(40000, seed=23, black_frac=0.05)
    ctx = mpss.Context()
    ctx.set_irradiance_points(p, n, E, area)
    nodes = ctx.octree_export()["nodes"].view(NODE).reshape(-1)
    got = (nodes["pad"] >> 16).astype(np.uint64)
    lo, hi = _leaf_code_bounds(nodes, float(ctx.cfg.max_error))
    assert np.all((got >= lo) & (got <= hi))
    assert np.all(got[nodes["leaf_first"] < 0] == 0x7f80)
    leaf = nodes["leaf_first"] >= 0
    assert np.all((nodes["pad"][leaf] & 0xffff) <= 8) and np.all(got[leaf] < 0x7f80)


def test_gpu_build_rejects_coincident_points(mpss):
    p = np.zeros((12, 3), np.float32)
    n = np.tile(np.float32([0, 0, 1]), (12, 1))
    ctx = mpss.Context()
    with pytest.raises(mpss.MpssError):
        ctx.set_irradiance_points(p, n, np.ones((12, 30), np.float32), np.ones(12, np.float32))


def test_preprocess_gpu_build_matches_host_build(mpss):
    """The render path's Preprocess (device irradiance handed to the device build) on skin.pbrt."""
    from mpss import pbrtscene
    out = []
    for on_host in (0, 1):
        sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin.pbrt"), xres=64, yres=64, spp=4)
        sc.integrator["minsampledistance"] = 0.004
        for m in sc.materials:
            m["desired_length"] = 64
        ctx = pbrtscene.build_context(sc, octree_on_host=on_host)
        ctx.preprocess(seed=3)
        out.append((ctx.octree_info(), ctx.octree_export()))
    assert out[0][0] == out[1][0]
    assert out[0][0]["n_points"] > 50000
    _same(out[0][1], out[1][1])
