"""CPU checks of the per-pixel path (no GPU): the oracle's render restatement against itself
(tile invariance, determinism, film coverage) and against reference semantics that have a
closed form, plus the product's host tessellation against the oracle's (bit-exact)."""
import os

import numpy as np
import pytest

import oracle_render as orr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def small(mpss, oracle):
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin.pbrt"), xres=48, yres=48, spp=4)
    sc.integrator["minsampledistance"] = 0.01
    for m in sc.materials:
        m["desired_length"] = 64
    cfg = mpss.default_config(**pbrtscene.integrator_config(sc))
    tabs = orr.tables_from_host(sc, mpss)
    o = orr.OracleScene(sc, tabs, cfg, mpss)
    pts = o.tessellate()
    E = o.irradiance(pts, 1)
    o.set_octree(pts, E)
    return sc, o, pts, E


def test_host_tessellation_bit_exact(mpss, small):
    sc, o, pts, _ = small
    me = sc.meshes[0]
    det = np.linalg.det(me["o2w"][:3, :3].astype(np.float64))
    got = mpss.host_tessellate(me["P"], me["indices"], me["o2w"], me["w2o"], 0.01, N=me["N"], S=me["S"],
                               uv=me["uv"], flip=bool(me["reverse"]) ^ bool(det < 0))
    assert len(got) == len(pts)
    assert got.tobytes() == pts.tobytes()


@pytest.mark.parametrize("incenter", [False, True])
def test_host_tessellation_small_cases(mpss, oracle, incenter):
    """Edge cases of the tessellator: a triangle smaller than minDist (sent back whole), a long
    sliver (edge factors >> centre factor) and a mesh without N/S/uv."""
    P = np.array([[0, 0, 0], [1e-3, 0, 0], [0, 1e-3, 0], [0, 0, 0], [2.0, 0, 0], [0, 0.05, 0],
                  [0, 0, 0], [0.3, 0.1, 0], [0.1, 0.3, 0.05]], np.float32)
    idx = np.arange(9, dtype=np.int32).reshape(3, 3)
    eye = np.eye(4, dtype=np.float32)
    got = mpss.host_tessellate(P, idx, eye, eye, 0.02, incenter=incenter)
    assert got["area"].min() > 0
    # total area is preserved by the tessellation (up to float rounding)
    tri_area = 0.5 * np.linalg.norm(np.cross(P[idx[:, 1]] - P[idx[:, 0]], P[idx[:, 2]] - P[idx[:, 0]]), axis=1)
    assert got["area"].sum() == pytest.approx(tri_area.sum(), rel=1e-4)
    from mpss import pbrtscene
    sc = pbrtscene.Scene()
    sc.xres = sc.yres = 8
    sc.materials = [{}]
    sc.meshes = [dict(P=P, N=None, S=None, uv=None, indices=idx, o2w=eye, w2o=eye, reverse=False, material=0)]
    cfg = mpss.default_config(min_sample_distance=0.02)
    o = orr.OracleScene(sc, [(np.ones((30, 4), np.float32), np.ones(30, np.float32), np.zeros(5, np.float32))],
                        cfg, mpss)
    ref = o.tessellate(incenter=incenter)
    assert got.tobytes() == ref.tobytes()


def test_oracle_preprocess_sane(small):
    sc, o, pts, E = small
    assert len(pts) > 10000
    assert np.all(np.isfinite(E)) and np.all(E >= 0)
    lit = E.sum(1) > 0
    assert 0.1 < lit.mean() < 0.9
    # a lit point's irradiance is bounded by the light's power over the distance: E <= L * solid angle * albedo
    assert E.max() < 3200 * 2 * np.pi


def test_oracle_tile_invariance_and_determinism(small):
    sc, o, _, _ = small
    full = o.render_tile(sc.spp, 3, 0, sc.xres, 0, sc.yres, nthreads=4)
    again = o.render_tile(sc.spp, 3, 0, sc.xres, 0, sc.yres, nthreads=2)
    assert np.array_equal(full, again)
    tiled = np.zeros_like(full)
    T = 20
    for y0 in range(0, sc.yres, T):
        for x0 in range(0, sc.xres, T):
            x1, y1 = min(x0 + T, sc.xres), min(y0 + T, sc.yres)
            tiled[y0:y1, x0:x1] = o.render_tile(sc.spp, 3, x0, x1, y0, y1, nthreads=4)
    assert np.array_equal(full, tiled)
    w = full[..., 3]
    assert w.min() >= sc.spp and w.max() <= 4 * sc.spp
    assert np.all(np.isfinite(full))
    Y = full[..., 1] / w
    assert (Y > 0).mean() > 0.02 and (Y == 0).mean() > 0.2


def test_film_edge_semantics():
    """ImageFilm::AddSample's pixel range for the 0.5-wide box filter: the float sample
    position x + u can round onto either pixel edge; such samples reach the neighbour too."""
    def extent(X, res):
        d = np.float32(X) - np.float32(0.5)
        lo = int(np.ceil(d - np.float32(0.5)))
        hi = int(np.floor(d + np.float32(0.5)))
        return max(lo, 0), min(hi, res - 1)
    assert extent(np.float32(5) + np.float32(0.25), 100) == (5, 5)
    assert extent(np.float32(5) + np.float32(0.0), 100) == (4, 5)
    big = np.float32(1000) + np.float32(1 - 2 ** -24)  # rounds up to 1001
    assert big == np.float32(1001) and extent(big, 2000) == (1000, 1001)
    assert extent(np.float32(0), 100) == (0, 0)


def test_windowed_replay_table_and_render(small):
    """o_replay_render_table_window keeps exactly the whole-extent table's rows of its window (a
    task's RNG(taskNum) stream is its own, so skipping the tasks outside changes nothing), and a
    tile rendered from the windowed table equals the tile rendered from the whole table."""
    sc, o, _, _ = small
    full = o.replay_table(sc.spp, cores=8, li_draws=6, nthreads=4)
    x0, x1, y0, y1 = 13, 31, 7, 29
    win = o.replay_window(x0, x1, y0, y1)
    assert win == (12, 32, 6, 30)
    part = o.replay_table_window(sc.spp, win, cores=8, li_draws=6, nthreads=4)
    assert np.array_equal(part, full[win[2]:win[3], win[0]:win[1]])
    a = o.render_tile_replay(sc.spp, full, x0, x1, y0, y1, nthreads=4)
    b = o.render_tile_replay(sc.spp, part, x0, x1, y0, y1, nthreads=4, window=win)
    assert np.array_equal(a, b) and (a[..., 1] > 0).any()
    # a window touching the frame edge keeps the extent's last row / column (xres, yres)
    win = o.replay_window(sc.xres - 5, sc.xres, sc.yres - 4, sc.yres)
    assert win == (sc.xres - 6, sc.xres + 1, sc.yres - 5, sc.yres + 1)
    part = o.replay_table_window(sc.spp, win, cores=8, li_draws=6, nthreads=4)
    assert np.array_equal(part, full[win[2]:, win[0]:])


def test_cpu_baseline_task_split(small):
    """bench.py's CPU baseline runs SamplerRenderer::Render's task split: RoundUpPow2(max(32 cores,
    W H / 256)) sub-windows (Sampler::ComputeSubWindow) that tile the image exactly once."""
    sc, o, _, _ = small
    assert orr.render_task_count(1024, 1024, 8) == 4096
    assert orr.render_task_count(1024, 1024, 256) == 8192
    assert orr.render_task_count(48, 48, 4) == 128
    cover = np.zeros((sc.yres, sc.xres), np.int32)
    n = orr.render_task_count(sc.xres, sc.yres, 4)
    for k in range(n):
        x0, x1, y0, y1 = orr.sub_window(k, n, 0, sc.xres, 0, sc.yres)
        cover[y0:y1, x0:x1] += 1
    assert np.all(cover == 1)
    # a bounded run renders whole tasks only
    import ctypes as C
    order = np.arange(n, dtype=np.int32)
    tasks, el = C.c_long(), C.c_double()
    px = orr._lib().o_cpu_baseline(o.h, sc.spp, 3, 4, 4, 30.0, order.ctypes.data, n, C.byref(tasks), C.byref(el))
    assert tasks.value == n and px == sc.xres * sc.yres and el.value > 0
