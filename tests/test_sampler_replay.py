"""The reference sampler in the oracle (oracle/render.c o_replay_*), on the CPU.

pbrt draws each render task's sample values from RNG(task) = MT19937 (core/rng.cpp):
SamplerRenderer::Render's task split (samplerrenderer.cpp:191-225) and ComputeSubWindow over the
film's sample extent (core/sampler.cpp:55-78, film/image.cpp:150-166), LDSampler ->
LDPixelSample (lowdiscrepancy.cpp:69-82, montecarlo.cpp:200-250) with LDShuffleScrambled1D/2D and
Shuffle (montecarlo.h:183-189, 314-333), and Li's BSDFSample(rng) draws per camera hit
(integrator.cpp:177-185). Checked here:
  - the oracle's MT19937 against numpy's (RandomState uses init_genrand for integer seeds);
  - the oracle's whole sample table against an independent pure-Python restatement, on scenes
    where every camera ray hits (6 draws each) or none does;
  - net structure: a pixel's spp image samples occupy distinct 1/spp strata in both axes, and
    each light array's spp x n values occupy distinct strata too;
  - the table depends on the emulated core count (the task split), as in the reference;
  - IrradianceTask's RNG(47 k) scrambles against the Python restatement.
"""
import numpy as np
import pytest

import oracle_render as orr

NB = 30
ONE_M_EPS = np.float32(float.fromhex("0x1.fffffep-1"))  # OneMinusEpsilon, pbrt.h


def vdc(n, scr):
    n = int(n) & 0xffffffff
    n = ((n << 16) | (n >> 16)) & 0xffffffff
    n = (((n & 0x00ff00ff) << 8) | ((n & 0xff00ff00) >> 8)) & 0xffffffff
    n = (((n & 0x0f0f0f0f) << 4) | ((n & 0xf0f0f0f0) >> 4)) & 0xffffffff
    n = (((n & 0x33333333) << 2) | ((n & 0xcccccccc) >> 2)) & 0xffffffff
    n = (((n & 0x55555555) << 1) | ((n & 0xaaaaaaaa) >> 1)) & 0xffffffff
    n ^= scr
    return min(np.float32((n >> 8) & 0xffffff) / np.float32(1 << 24), ONE_M_EPS)


def sobol2(n, scr):
    v = 1 << 31
    while n:
        if n & 1:
            scr ^= v
        n >>= 1
        v ^= v >> 1
    return min(np.float32((scr >> 8) & 0xffffff) / np.float32(1 << 24), ONE_M_EPS)


class MT:
    def __init__(self, seed):
        self.rs = np.random.RandomState(seed)

    def u32(self):
        return int(self.rs.randint(0, 2 ** 32, dtype=np.uint64))


def shuffle(samp, count, dims, rng):
    for i in range(count):
        other = i + rng.u32() % (count - i)
        for j in range(dims):
            samp[dims * i + j], samp[dims * other + j] = samp[dims * other + j], samp[dims * i + j]


def ld1d(n, npix, rng):
    scr = rng.u32()
    s = [vdc(i, scr) for i in range(n * npix)]
    for i in range(npix):
        sub = s[i * n:(i + 1) * n]
        shuffle(sub, n, 1, rng)
        s[i * n:(i + 1) * n] = sub
    shuffle(s, npix, n, rng)
    return s


def ld2d(n, npix, rng):
    s0, s1 = rng.u32(), rng.u32()
    s = []
    for i in range(n * npix):
        s += [vdc(i, s0), sobol2(i, s1)]
    for i in range(npix):
        sub = s[2 * i * n:2 * (i + 1) * n]
        shuffle(sub, n, 2, rng)
        s[2 * i * n:2 * (i + 1) * n] = sub
    shuffle(s, npix, 2 * n, rng)
    return s


def sub_window(num, count, xs, xe, ys, ye):
    f = np.float32
    dx, dy = xe - xs, ye - ys
    nx, ny = count, 1
    while (nx & 1) == 0 and 2 * dx * ny < dy * nx:
        nx >>= 1
        ny <<= 1
    xo, yo = num % nx, num // nx

    def lerp(t, a, b):
        return int(np.floor(f(f(f(1) - t) * f(a)) + f(t * f(b))))
    tx0, tx1 = f(xo) / f(nx), f(xo + 1) / f(nx)
    ty0, ty1 = f(yo) / f(ny), f(yo + 1) / f(ny)
    return lerp(tx0, xs, xe), lerp(tx1, xs, xe), lerp(ty0, ys, ye), lerp(ty1, ys, ye)


def round_pow2(v):
    r = 1
    while r < v:
        r <<= 1
    return r


def python_table(W, H, spp, ns, cores, li_draws):
    """The reference loop for a scene where every camera ray hits (li_draws per sample) or none."""
    K = 2 + 5 * sum(ns)
    offs = np.cumsum([2] + [5 * n for n in ns])[:-1]
    T = round_pow2(max(32 * cores, (W * H) // 256))
    vals = np.zeros((H + 1, W + 1, spp, K), np.float32)
    n1 = [n for n in ns for _ in (0, 1)] + [1, 1]
    n2 = [n for n in ns for _ in (0, 1)]
    for task in range(T):
        x0, x1, y0, y1 = sub_window(task, T, 0, W + 1, 0, H + 1)
        if x0 == x1 or y0 == y1:
            continue
        rng = MT(task)
        for y in range(y0, y1):
            for x in range(x0, x1):
                image = ld2d(1, spp, rng)
                ld2d(1, spp, rng)  # lens
                ld1d(1, spp, rng)  # time
                one = [ld1d(n, spp, rng) for n in n1]
                two = [ld2d(n, spp, rng) for n in n2]
                for i in range(spp):
                    vals[y, x, i, 0:2] = image[2 * i:2 * i + 2]
                    for l, n in enumerate(ns):
                        for j in range(n):
                            o = offs[l] + 5 * j
                            vals[y, x, i, o:o + 2] = two[2 * l][2 * (n * i + j):2 * (n * i + j) + 2]
                            vals[y, x, i, o + 2] = one[2 * l + 1][n * i + j]
                            vals[y, x, i, o + 3:o + 5] = two[2 * l + 1][2 * (n * i + j):2 * (n * i + j) + 2]
                for _ in range(spp * li_draws):
                    rng.u32()
    return vals


def _scene(mpss, hits, W=20, H=12, spp=4, ns=(2, 1)):
    """A camera (identity world-to-camera, looking down +z) in front of a huge quad that fills the
    view (hits) or behind it (no hit); a sphere light and an infinite light."""
    from mpss import pbrtscene
    sc = pbrtscene.Scene()
    sc.xres, sc.yres, sc.spp, sc.fov = W, H, spp, 60.0
    sc.materials = [{"desired_length": 16}]
    z = 10.0 if hits else -10.0
    P = np.array([[-1e3, -1e3, z], [1e3, -1e3, z], [1e3, 1e3, z], [-1e3, 1e3, z]], np.float32)
    eye = np.eye(4, dtype=np.float32)
    sc.meshes = [dict(P=P, N=None, S=None, uv=None, indices=np.array([[0, 1, 2], [0, 2, 3]], np.int32), o2w=eye,
                      w2o=eye, reverse=False, material=0)]
    sc.lights = [dict(center=[0.0, 0.0, -5.0], radius=0.5, L=[1.0, 1.0, 1.0], nsamples=ns[0]),
                 dict(kind="infinite", L=[0.3, 0.3, 0.3], scale=[1, 1, 1], nsamples=ns[1], l2w=eye, w2l=eye)]
    tables = [(np.ones((NB, 16), np.float32), np.ones(NB, np.float32), np.zeros(1025, np.float32))]
    return sc, orr.OracleScene(sc, tables, mpss.default_config(), mpss)


def test_mt19937_matches_numpy(oracle):
    for seed in (0, 1, 47 * 5, 2 ** 31 + 7):
        out = np.zeros(700, np.uint32)
        oracle.lib().o_mt_first(seed, 700, out)
        ref = np.random.RandomState(seed).randint(0, 2 ** 32, size=700, dtype=np.uint64).astype(np.uint32)
        assert np.array_equal(out, ref)


@pytest.mark.parametrize("hits,li_draws,cores", [(True, 6, 1), (False, 6, 1), (True, 0, 1), (True, 6, 2)])
def test_oracle_table_matches_python_restatement(mpss, oracle, hits, li_draws, cores):
    sc, o = _scene(mpss, hits)
    got = o.replay_table(4, cores=cores, li_draws=li_draws)
    ref = python_table(sc.xres, sc.yres, 4, (2, 1), cores, li_draws if hits else 0)
    assert got.shape == ref.shape
    assert np.array_equal(got, ref)


def test_table_net_structure_and_core_dependence(mpss, oracle):
    sc, o = _scene(mpss, True, W=33, H=17, spp=8, ns=(4, 2))
    t = o.replay_table(8, cores=1)
    spp = 8
    for y in range(0, 18, 5):
        for x in range(0, 34, 7):
            for c in (0, 1):  # image u, v: one per stratum of width 1/spp
                assert len(set(np.floor(t[y, x, :, c] * spp).astype(int))) == spp
            for off, n in ((2, 4), (22, 2)):  # light positions: spp * n strata
                u = t[y, x, :, off:off + 5 * n:5].ravel()
                assert len(set(np.floor(u * spp * n).astype(int))) == spp * n
    assert not np.array_equal(t, o.replay_table(8, cores=4))  # another task split, other streams


def test_irradiance_scrambles_match_python(oracle):
    n, nl, cores = 5000, 2, 1
    scr = np.zeros((n, nl, 2), np.uint32)
    orr._lib().o_replay_irradiance_scr(n, nl, cores, scr.ctypes.data)
    T = round_pow2(max(32 * cores, n // 4096))
    ref = np.zeros_like(scr)
    for k in range(T):
        i0, i1 = k * n // T, (k + 1) * n // T
        rng = MT(47 * k)
        for i in range(i0, i1):
            for l in range(nl):
                ref[i, l] = rng.u32(), rng.u32()
                rng.u32()
    assert np.array_equal(scr, ref)


def test_sobol2_closed_form_equals_the_loop():
    """pbrt_math.h sobol2: the superset-sum transform + bit reversal equals Sobol02's column loop
    (montecarlo.h:292-302) for every 16-bit index and random 32-bit ones."""
    def loop(n, scr):
        v = 1 << 31
        while n:
            if n & 1:
                scr ^= v
            n >>= 1
            v ^= v >> 1
        return scr

    def closed(n, scr):
        for k, m in ((1, 0x55555555), (2, 0x33333333), (4, 0x0F0F0F0F), (8, 0x00FF00FF), (16, 0x0000FFFF)):
            n ^= (n >> k) & m
        return int("{:032b}".format(n)[::-1], 2) ^ scr

    rng = np.random.default_rng(7)
    ns = list(range(1 << 16)) + [int(x) for x in rng.integers(0, 1 << 32, 4096, dtype=np.uint64)]
    scr = [int(x) for x in rng.integers(0, 1 << 32, len(ns), dtype=np.uint64)]
    assert all(loop(n, s) == closed(n, s) for n, s in zip(ns, scr))
