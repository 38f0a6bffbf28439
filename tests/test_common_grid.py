"""The common grid of the sharded Mo() gather (mpss_config.mo_common_grid; mo_band.h CommonGrid),
host half, on the CPU: the LDS split, the resampled pair rows and the range they serve, against a
numpy restatement of multipole.cpp:60-73's sampleProfile (every served knot within 2e-6 of the
band's own value, or 1e-14 of the band's peak in the far tails).

The gather itself (LDS and own-table lanes bit-identical to the per-band gather, row lanes within
the bound) is checked on the GPU by tests/test_mo_gpu.py and the image tests."""
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "golden.npz")
NEAR_FIELDS = (5088, 10236)  # mpss_config.mo_near_field: the default layout and the one-workgroup one
ABS_TOL = 1e-14  # mo_kernel.h kCgAbsTol


def _groups(rcp):
    """make_band_groups (mo_band.h): bands by increasing rcp, runs of 4, 4, 4, 4, 4, 4, 3, 3."""
    order = np.argsort(rcp, kind="stable")
    return [list(order[i * 4:(i + 1) * 4]) for i in range(6)] + [list(order[24:27]), list(order[27:30])]


def _band_at(T, f, L):
    """Band lerp at fractional index f (double), the last segment continued one row past the end."""
    s = np.minimum(np.floor(f).astype(np.int64), L - 2)
    t = f - s
    return (1.0 - t) * T[s] + t * T[s + 1]


def _R(T, r, u, L):
    """Band table T on a group grid of relative spacing r at integer u (build_common's R_j(u))."""
    f = u * r
    v = _band_at(T, f, L)
    return np.where((f - r > L - 1) | (u >= L), 0.0, v)


def _lerp_at(T, f, L):
    """A band's own lookup at fractional index f (0 past its end)."""
    s = np.minimum(np.floor(f).astype(np.int64), L - 2)
    t = f - s
    return np.where(f > L - 1, 0.0, (1.0 - t) * T[np.maximum(s, 0)] + t * T[np.maximum(s, 0) + 1])


def _check_layout(tab, rcp, cg, tol=2e-6, groups=None, near_field=5088, rgb=False):
    """Groups, the LDS split, the pair rows against numpy, and that every band knot the rows serve
    is within tol of the band's own value (unfloored) -- for the rgbprofile's R, G, B (rgb) within tol
    of the largest of the three at that distance, the scale of FromRGB's outputs."""
    lds_floats = 4 * (near_field + 3)
    L = tab.shape[1]
    T64 = tab.astype(np.float64)
    for g, bands in enumerate(groups or _groups(rcp)):
        slots = cg["bands"][g]
        assert sorted(b for b in slots if b >= 0) == sorted(int(b) for b in bands)
        rg = np.float32(rcp[bands].min())
        assert cg["rg"][g] == rg
        r = np.array([np.float64(rcp[c]) / np.float64(rg) if c >= 0 else 0.0 for c in slots])
        # every lane with u < u0lim has s_j < klim_j for every band: the split fits the LDS
        need = sum(int(np.ceil(cg["u0lim"][g] * rj)) + 2 for rj in r if rj > 0)
        assert 0 < need <= lds_floats
        u0, u1, ub, r0 = cg["u0lim"][g], cg["u1lim"][g], int(cg["ubase"][g]), int(cg["row0"][g])
        if u1 <= u0:
            continue
        us = cg["u1start"][g]  # the rows serve u in [u1start, u1lim); they begin at the near field's end
        assert us >= u0 and us < u1
        assert ub == max(0, int(np.floor(u0)) - 1)
        # row coordinate v: u below ua, ua + (u - ua) / H above it (H = 1 / hinv, ua a multiple of 64)
        H = int(round(1.0 / cg["hinv"][g]))
        assert H in (1, 2, 4) and np.float32(1.0 / H) == cg["hinv"][g]
        ua = int(cg["ua"][g]) if H > 1 else int(u1)
        assert H == 1 or (ua % 64 == 0 and ub < ua < u1 and (int(u1) - ua) % H == 0)
        v1 = ua + (int(u1) - ua) // H
        n = v1 - ub + 1  # (one pad row: a lane's v may round up to v(u1lim))
        rows = cg["rows"][r0:r0 + n].astype(np.float64)
        assert len(rows) == n and n <= 65537
        v = np.arange(ub, ub + n + 1, dtype=np.int64)
        upos = np.where(v <= ua, v, ua + H * (v - ua)).astype(np.float64)
        bad = np.isnan(rows[:, 0])
        # cells with a knot off by more than the bound, before u1start, or within a step of a band's end
        # (must: the cells meeting [u_end - 1, u_end + 2]; may: with a rounding margin either way)
        served_bad = upos[1:] <= np.floor(us)
        must = np.zeros(n, bool)
        for j, c in enumerate(slots):
            if c >= 0:
                ue = (L - 1) / r[j]
                served_bad |= (upos[1:] > ue - 1 - 1e-6) & (upos[:-1] <= ue + 2 + 1e-6)
                must |= (upos[1:] > ue - 1 + 1e-6) & (upos[:-1] <= ue + 2 - 1e-6)
        # every cell within a step of a band's end is flagged (the combine has no range test)
        assert np.all(bad[must & (upos[:-1] >= np.floor(us))]), g
        for j, c in enumerate(slots):
            if c < 0:
                assert np.all(rows[:, 2 * j:2 * j + 2] == 0)
                continue
            want0 = _R(T64[c], r[j], upos[:-1], L).astype(np.float32)
            want1 = _R(T64[c], r[j], upos[1:], L).astype(np.float32)
            got0 = rows[:, 2 * j].astype(np.float32)
            np.testing.assert_array_equal(got0[~bad] if j == 0 else got0, want0[~bad] if j == 0 else want0)
            np.testing.assert_array_equal(rows[:, 2 * j + 1].astype(np.float32), want1)
            # the knots in the rows' cells (from the first row's, u >= ubase), each in its cell (row) k; the
            # lanes read those with u in [u1start, u1lim)
            k = np.arange(max(0, int(np.floor(ub * r[j])) - 1), L - 1)
            uk = k / r[j]
            sel = (uk >= ub) & (uk < u1)
            k, uk = k[sel], uk[sel]
            served = uk >= us
            vk = np.where(uk < ua, uk, ua + (uk - ua) / H)
            ci = np.floor(vk).astype(np.int64) - ub
            t = vk - np.floor(vk)
            approx = (1 - t) * want0[ci].astype(np.float64) + t * want1[ci].astype(np.float64)
            err = np.abs(approx - T64[c, k])
            # kCgRelTol of the band's value (rgb: of the largest of R, G, B there), or kCgAbsTol = 1e-14
            # of its peak where that is larger
            scale = np.abs(T64[c, k])
            if rgb:
                for q, cq in enumerate(slots):
                    if cq >= 0 and q != j:
                        scale = np.maximum(scale, np.abs(_lerp_at(T64[cq], uk * r[q], L)))
            bound = np.maximum(tol * scale, ABS_TOL * np.abs(T64[c]).max())
            over = (err > bound * (1 + 1e-9)) & served
            # every knot off by more than the bound lies in a flagged cell (its lanes read the exact tables)
            assert np.all(bad[ci[over]]), (g, c, (err[served & ~bad[ci]] / bound[served & ~bad[ci]]).max())
            served_bad[ci[err > bound * (1 - 1e-9)]] = True
        # and a flagged cell is one of those (the flags are not spent on good cells; the pad row's cell
        # lies past u1lim)
        assert np.all(served_bad[:-1][bad[:-1]]), (g, np.flatnonzero(bad[:-1] & ~served_bad[:-1])[:5])


@pytest.mark.parametrize("near_field", NEAR_FIELDS)
def test_common_grid_of_golden_profile(mpss, near_field):
    """desiredlength 64 skin profile (tests/golden): layout and pair rows vs numpy, the served range
    within the bound."""
    z = np.load(GOLDEN)
    tab, rcp = z["profile_64"], z["profile_64_rcp"]
    cg = mpss.host_common_grid(tab, rcp, near_field=near_field)
    _check_layout(tab, rcp, cg, near_field=near_field)
    assert cg["rel_err"].max() <= 2e-6


@pytest.mark.parametrize("near_field", NEAR_FIELDS)
def test_common_grid_of_the_benched_skin_profile(mpss, near_field):
    """C2's material (skin.pbrt, desiredlength 512), for both LDS layouts (5088: the default the
    render path uses): rows for 7 of the 8 groups, over more than one doubling of distance past the
    near field for each, every served knot within the bound."""
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin.pbrt"))
    m = sc.materials[0]
    kw = {k: v for k, v in m.items() if k not in ("Kr", "Kt", "albedo", "albedo_tex", "bump_tex")}
    tab, rcp, _ = mpss.host_build_profile(*mpss.host_skin_layers(mpss.default_skin(**kw)), 512)
    cg = mpss.host_common_grid(tab, rcp, near_field=near_field)
    assert cg["ok"]
    span = np.log2(np.maximum(cg["u1lim"], 1) / cg["u0lim"])
    assert (span > 1.0).sum() >= 7, span
    assert cg["rel_err"].max() <= 2e-6 and cg["l1_err"].max() <= 1e-8
    assert len(cg["rows"]) <= 8 * 65537
    _check_layout(tab, rcp, cg, near_field=near_field)


@pytest.mark.parametrize("near_field", NEAR_FIELDS)
def test_common_grid_of_the_rgb_profile(mpss, near_field):
    """rgbprofile at C2's length (desiredlength 512): the R, G, B profiles in slots 0..2 of every
    group, grid = G's (the longest reach). B reaches ~15x less far in d^2, its knots that much denser
    than the grid; each knot's error is bounded against the largest of R, G, B at that distance (the
    scale of FromRGB's outputs, build_common_grid's rgb), so the rows serve all three from (about) the
    near field's end to ~67 k of G's 120 k steps."""
    import oracle_lib
    from test_rgbprofile import rgb_layers
    mua, musp, th, eta = oracle_lib.skin_layers(0.3, 40e6, 0.5, 0.5, 0.5, 0.5, (0.25e6, 20e6), (1.4, 1.4))
    ra, rs = rgb_layers(mua, musp)
    tab, rcp, _, _ = oracle_lib.compute_profile(ra, rs, eta, th, desired_length=512)
    cg = mpss.host_common_grid(tab, rcp, rgb=True, near_field=near_field)
    assert cg["ok"]
    assert np.all(cg["bands"] == np.array([0, 1, 2, -1]))
    assert np.all(cg["rg"] == np.float32(rcp[:3].min()))
    # (5088 layout: u0lim 1174, rows from 1319; 10236: both 2364 -- with each component's own value as
    # the scale, round 4's bound, B kept the rows off until 4185)
    assert np.all(cg["u1start"] >= cg["u0lim"]) and np.all(cg["u1start"] < 1.2 * cg["u0lim"])
    assert np.all(cg["u1lim"] - cg["u1start"] > 60000)
    rows = cg["rows"].reshape(8, -1, 8)
    assert np.all(rows[:, :, 6:] == 0)  # the empty slot
    assert cg["rel_err"][:3].max() <= 2e-6 and cg["l1_err"][:3].max() <= 5e-8
    _check_layout(tab, rcp, cg, groups=[[0, 1, 2]] * 8, near_field=near_field, rgb=True)


def test_common_grid_of_a_rough_table(mpss):
    """A table that is rough on the groups' grids (30 % noise): the good rows serve only knots within the
    bound -- here only where a resampled band has fallen under 5e-5 of its peak (kCgAbsTol / kCgRelTol);
    where its noise is resolvable every cell is flagged (its lanes read the exact tables)."""
    rng = np.random.default_rng(5)
    L = 4096
    x = np.arange(L) / L
    tab = np.stack([np.exp(-x * (3 + c)) * (1 + 0.3 * rng.random(L)) for c in range(30)]).astype(np.float32)
    rcp = ((L - 1) / np.linspace(0.01, 0.05, 30)).astype(np.float32)
    cg = mpss.host_common_grid(tab, rcp)
    _check_layout(tab, rcp, cg)
    for g in range(8):
        us, u1, ub, r0 = cg["u1start"][g], cg["u1lim"][g], int(cg["ubase"][g]), int(cg["row0"][g])
        if u1 <= cg["u0lim"][g]:
            continue
        H = int(round(1.0 / cg["hinv"][g]))
        ua = float(cg["ua"][g]) if H > 1 else float(u1)
        for c in cg["bands"][g]:
            if c < 0 or rcp[c] == cg["rg"][g]:
                continue
            r = np.float64(rcp[c]) / np.float64(cg["rg"][g])
            k = np.arange(L - 1)
            uk = k / r
            served = (uk >= us) & (uk < u1)
            vk = np.where(uk < ua, uk, ua + (uk - ua) / H)
            row = cg["rows"][r0 + np.floor(vk[served]).astype(np.int64) - ub, 0]
            good = ~np.isnan(row)
            assert np.all(np.abs(tab[c, :L - 1][served][good]) < ABS_TOL / 2e-6 * np.abs(tab[c]).max())


def test_common_grid_equal_spacing_is_exact(mpss):
    """Bands sharing one spacing: the group grid is every band's own, the rows are the tables."""
    L = 30000
    x = np.arange(L) / L
    tab = np.stack([np.exp(-x * (4 + 0.2 * c)) for c in range(30)]).astype(np.float32)
    rcp = np.full(30, (L - 1) / 0.004, np.float32)
    cg = mpss.host_common_grid(tab, rcp)
    assert cg["ok"] and cg["rel_err"].max() == 0
    _check_layout(tab, rcp, cg, tol=0.0)
    ub, r0 = int(cg["ubase"][0]), int(cg["row0"][0])
    c = cg["bands"][0][0]
    assert np.array_equal(cg["rows"][r0:r0 + 100, 0], tab[c, ub:ub + 100])


@pytest.mark.parametrize("bad", ["zero_rcp", "short"])
def test_common_grid_declines_degenerate_tables(mpss, bad):
    L = 3 if bad == "short" else 100
    tab = np.ones((30, L), np.float32)
    rcp = np.full(30, 10.0, np.float32)
    if bad == "zero_rcp":
        rcp[3] = 0.0
    cg = mpss.host_common_grid(tab, rcp)
    assert not cg["ok"] and len(cg["rows"]) == 0
