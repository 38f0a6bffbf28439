"""Several LayeredSkin materials and concurrent callers (include/mpss.h thread-safety contract).

* Two layeredskin materials with different pigments on one head (the mesh split in two): every
  BSSRDF hit evaluates Mo() with its own material's profile (multipolesubsurface.cpp:267-280),
  checked against the oracle, which does the same per hit.
* 8 host threads x 2 materials, each thread on its own HIP stream, calling mpss_render_tile and
  mpss_mo_batch at the same time (SamplerRendererTask calls Li from every worker thread,
  parallel.cpp:800-878): every result bit-identical to the same call made serially.
"""
import os
import threading

import numpy as np
import pytest

import oracle_lib
import oracle_render as orr

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NT = oracle_lib.nthreads()


def _two_material_scene(res=64, spp=8):
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin.pbrt"), xres=res, yres=res, spp=spp)
    sc.integrator["minsampledistance"] = 0.008
    m0 = dict(sc.materials[0])
    m0["desired_length"] = 128
    m1 = dict(m0)
    m1.update(f_mel=0.05, f_blood=0.2, f_ohg=0.9)  # paler, redder skin: different Rd and band groups
    sc.materials = [m0, m1]
    me = sc.meshes[0]
    idx = np.asarray(me["indices"])
    P = np.asarray(me["P"])
    cx = P[idx].mean(axis=1)[:, 0]
    left = cx < np.median(cx)
    a, b = dict(me), dict(me)
    a["indices"], a["material"] = idx[left], 0
    b["indices"], b["material"] = idx[~left], 1
    sc.meshes = [a, b]
    return sc


@pytest.fixture(scope="module")
def two(mpss, oracle):
    import torch
    assert torch.cuda.is_available()
    from mpss import pbrtscene
    sc = _two_material_scene()
    ctx = pbrtscene.build_context(sc)
    ctx.preprocess(seed=2)
    o = orr.OracleScene(sc, orr.tables_from_ctx(ctx, 2), ctx.cfg, mpss)
    return torch, sc, ctx, o


def _render(torch, ctx, spp, seed, x0, x1, y0, y1, stream=None):
    out = torch.zeros(((y1 - y0) * (x1 - x0) * 4,), dtype=torch.float32, device="cuda")
    ctx.render_tile(spp, seed, x0, x1, y0, y1, out.data_ptr(), None if stream is None else stream.cuda_stream)
    return out


def test_two_materials_have_different_profiles(two):
    torch, sc, ctx, o = two
    t0, r0, _, _ = ctx.material_tables(0)
    t1, r1, _, _ = ctx.material_tables(1)
    assert not np.array_equal(t0, t1)


def test_two_materials_match_oracle(two):
    torch, sc, ctx, o = two
    pts = ctx.surface_points()
    assert set(np.unique(pts["material"])) == {0, 1}
    E = o.irradiance(pts, 2, nthreads=NT)
    np.testing.assert_allclose(ctx.irradiance(), E, rtol=1e-5, atol=1e-6 * float(E.max()))
    o.set_octree(pts, E)
    got = _render(torch, ctx, sc.spp, 5, 0, sc.xres, 0, sc.yres).cpu().numpy().reshape(sc.yres, sc.xres, 4)
    ref = o.render_tile(sc.spp, 5, 0, sc.xres, 0, sc.yres, nthreads=NT)
    assert np.array_equal(got[..., 3], ref[..., 3])
    peak = float(np.abs(ref[..., :3]).max())
    bound = 1e-4 * np.maximum(np.abs(ref[..., :3]), 1e-3 * peak)
    worst = float((np.abs(got[..., :3] - ref[..., :3]) / bound).max())
    assert worst <= 1.0, worst
    # the hits of each material really use their own profile: rendering with material 1's
    # profile swapped for material 0's changes the image (the oracle's view of the swap)
    o2 = orr.OracleScene(sc, [orr.tables_from_ctx(ctx, 1)[0]] * 2, ctx.cfg, ctx_mpss())
    o2.set_octree(pts, E)
    wrong = o2.render_tile(sc.spp, 5, 0, sc.xres, 0, sc.yres, nthreads=NT)
    assert np.abs(wrong[..., :3] - ref[..., :3]).max() > 10 * bound.max()


def ctx_mpss():
    import mpss
    return mpss


def test_concurrent_callers_bit_identical_to_serial(two):
    torch, sc, ctx, o = two
    rng = np.random.default_rng(4)
    q = ctx.surface_points()["p"][rng.integers(0, len(ctx.surface_points()), 20000)].astype(np.float32)
    qd = torch.from_numpy(np.ascontiguousarray(q)).cuda()
    strips = [(0, sc.xres, 8 * k, 8 * k + 8) for k in range(8)]

    def job(k, stream):
        x0, x1, y0, y1 = strips[k]
        img = _render(torch, ctx, sc.spp, 9, x0, x1, y0, y1, stream)
        mo = torch.zeros((len(q), 30), dtype=torch.float32, device="cuda")
        ctx.mo_batch(k % 2, len(q), qd.data_ptr(), mo.data_ptr(), None,
                     None if stream is None else stream.cuda_stream)
        return img, mo

    serial = []
    for k in range(8):
        img, mo = job(k, None)
        torch.cuda.synchronize()
        serial.append((img.cpu().numpy(), mo.cpu().numpy()))
    results = [None] * 8
    errors = []
    barrier = threading.Barrier(8)

    def worker(k):
        try:
            s = torch.cuda.Stream()
            barrier.wait()
            with torch.cuda.stream(s):
                out = [job(k, s) for _ in range(3)]
            s.synchronize()
            results[k] = [(a.cpu().numpy(), b.cpu().numpy()) for a, b in out]
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errors, errors
    for k in range(8):
        for img, mo in results[k]:
            assert np.array_equal(img, serial[k][0]), k
            assert np.array_equal(mo, serial[k][1]), k
    # the two materials' gathers differ (so the test exercises both profiles)
    assert not np.array_equal(serial[0][1], serial[1][1])


def test_octree_rebuild_while_rendering(mpss, oracle):
    """mpss.h: a call that replaces the octree (mpss_set_irradiance_points) waits until the renders
    in flight have queued their kernels, then for those kernels. 4 threads render strips on their own
    streams while the main thread swaps the octree between two irradiance sets: no fault, and every
    strip equals that strip rendered serially on one of the two octrees, bit for bit."""
    import torch
    from mpss import pbrtscene
    sc = _two_material_scene(res=48, spp=4)
    ctx = pbrtscene.build_context(sc)
    ctx.preprocess(seed=3)
    pts = ctx.surface_points()
    E1 = np.ascontiguousarray(ctx.irradiance())
    E2 = np.ascontiguousarray(E1 * np.float32(0.5))
    cloud = [np.ascontiguousarray(pts[k], np.float32) for k in ("p", "n")]
    area = np.ascontiguousarray(pts["area"], np.float32)

    def use(E):
        ctx.set_irradiance_points(cloud[0], cloud[1], E, area)

    strips = [(0, sc.xres, 12 * k, 12 * k + 12) for k in range(4)]
    refs = []
    for E in (E1, E2):
        use(E)
        refs.append([_render(torch, ctx, sc.spp, 7, *r).cpu().numpy() for r in strips])
        torch.cuda.synchronize()
    assert not np.array_equal(refs[0][1], refs[1][1])  # the two octrees render differently
    results = [[] for _ in strips]
    errors = []
    start = threading.Barrier(len(strips) + 1)

    def worker(k):
        try:
            s = torch.cuda.Stream()
            start.wait()
            with torch.cuda.stream(s):
                for _ in range(6):
                    out = _render(torch, ctx, sc.spp, 7, *strips[k], s)
                    s.synchronize()
                    results[k].append(out.cpu().numpy())
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=worker, args=(k,)) for k in range(len(strips))]
    for t in th:
        t.start()
    start.wait()
    for i in range(4):
        use(E1 if i % 2 else E2)
    for t in th:
        t.join(timeout=120)
    assert not errors, errors
    for k in range(len(strips)):
        assert len(results[k]) == 6
        for img in results[k]:
            assert np.array_equal(img, refs[0][k]) or np.array_equal(img, refs[1][k]), k
    use(E1)  # last: every render from now on sees E1
    assert np.array_equal(_render(torch, ctx, sc.spp, 7, *strips[0]).cpu().numpy(), refs[0][0])
    ctx.close()
