"""Mo() gather on the GPU (libmpss HIP kernel) vs the CPU oracle: bit-exact.

The kernel follows the reference recursion's summation order (diffusionutil.h:175-210) and
rounds every product/sum like the scalar code, so equality is exact, not a tolerance.
Counters (octree nodes entered, leaf points evaluated) must match the oracle's
instrumented recursion too (they feed the algorithmic-bytes figure).
The spectrally sharded kernel (exact_mo=0) with per-band tables (mo_common_grid=0) and the packet
kernel (exact_mo=2) must agree bit for bit with each other; the packet kernel evaluates the same terms
with one running sum per band; it is held to 2e-5 relative of the reference order (all terms are
>= 0, so the reassociation error is bounded by n*eps of the result) and must visit exactly the same
pruned node/point sets as the exact kernel. The default sharded gather reads each band group's far
field from its resampled common grid (mo_common_grid=1, accepted per material by a measured error
bound): same traversal, the same 2e-5 bound against the reference order.
"""
import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu

RADII = (0.25, 0.3, 0.35)


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch


@pytest.fixture(scope="module")
def skin_profile(oracle):
    mua, musp, th, eta = oracle.skin_layers(0.3, 40e6, 0.5, 0.5, 0.5, 0.5, (0.25e6, 20e6), (1.4, 1.4))
    tab, rcp, _, _ = oracle.compute_profile(mua, musp, eta, th, desired_length=512)
    return tab, rcp


@pytest.fixture(scope="module")
def wide_profile():
    """A synthetic smooth profile whose extent spans many octree levels (stresses Rd lookups)."""
    L = 4096
    x = np.linspace(0, 1, L, dtype=np.float32)
    tab = np.stack([(np.exp(-x * (4 + 0.2 * c)) * (1 + 0.01 * c)).astype(np.float32) for c in range(30)])
    rcp = np.array([(L - 1) / (0.004 * (1 + 0.03 * c)) for c in range(30)], np.float32)
    return tab, rcp


def run_gpu(mpss, torch, cloud, table, rcp, q, max_error, exact=True, mode=None, **cfg):
    p, n, E, area = cloud
    ctx = mpss.Context(max_error=max_error, exact_mo=int(exact) if mode is None else mode, **cfg)
    mid = ctx.set_material_tables(table, rcp, np.zeros(1025, np.float32))
    ctx.set_irradiance_points(p, n, E, area)
    qd = torch.from_numpy(q).cuda()
    out = torch.zeros((len(q), 30), dtype=torch.float32, device="cuda")
    cnt = torch.zeros((len(q), 4), dtype=torch.int32, device="cuda")
    ctx.mo_batch(mid, len(q), qd.data_ptr(), out.data_ptr(), cnt.data_ptr())
    torch.cuda.synchronize()
    mo_plain = torch.zeros_like(out)
    ctx.mo_batch(mid, len(q), qd.data_ptr(), mo_plain.data_ptr())
    torch.cuda.synchronize()
    info = ctx.octree_info()
    ctx.close()
    return out.cpu().numpy(), cnt.cpu().numpy(), mo_plain.cpu().numpy(), info


@pytest.mark.parametrize("max_error", [0.05, 0.1, 0.5])
def test_mo_bit_exact_skin_profile(oracle, mpss, torch_dev, skin_profile, max_error):
    cloud = synth.ellipsoid_cloud(200000, radii=RADII, seed=7, black_frac=0.05)
    q = synth.surface_queries(6000, radii=RADII, seed=13)
    table, rcp = skin_profile
    mo, cnt, mo_plain, info = run_gpu(mpss, torch_dev, cloud, table, rcp, q, max_error)
    t = oracle.Octree(*cloud)
    ref, nn, npt = t.mo(q, table, rcp, max_error, counters=True)
    assert info["n_nodes"] == t.num_nodes()
    assert np.array_equal(mo, ref)
    assert np.array_equal(mo_plain, ref)  # the counting variant changes nothing
    assert np.array_equal(cnt[:, 0], nn) and np.array_equal(cnt[:, 1], npt)
    assert np.any(ref > 0)


@pytest.mark.parametrize("jitter", [0.0, 0.01])
def test_mo_bit_exact_wide_profile(oracle, mpss, torch_dev, wide_profile, jitter):
    cloud = synth.ellipsoid_cloud(50000, radii=RADII, seed=17, black_frac=0.1)
    q = synth.surface_queries(4001, radii=RADII, seed=19, jitter=jitter)  # odd count: half-wave tail
    table, rcp = wide_profile
    mo, cnt, _, _ = run_gpu(mpss, torch_dev, cloud, table, rcp, q, 0.1)
    ref, nn, npt = oracle.Octree(*cloud).mo(q, table, rcp, 0.1, counters=True)
    assert np.array_equal(mo, ref)
    assert np.array_equal(cnt[:, 0], nn) and np.array_equal(cnt[:, 1], npt)
    assert (ref > 0).mean() > 0.5


def test_mo_edge_cases(oracle, mpss, torch_dev, wide_profile):
    table, rcp = wide_profile
    # tiny clouds: single point, exactly 8 points (one leaf), 9 points (first split)
    for npts in (1, 8, 9, 100):
        cloud = synth.ellipsoid_cloud(npts, radii=(0.002, 0.002, 0.002), seed=npts, black_frac=0.0)
        q = np.concatenate([synth.surface_queries(63, radii=(0.002, 0.002, 0.002), seed=5, sort=False),
                            cloud[0][:1],                        # query exactly on a point (d2 = 0)
                            np.float32([[10.0, 10.0, 10.0]])])   # far outside every node
        mo, cnt, _, _ = run_gpu(mpss, torch_dev, cloud, table, rcp, np.ascontiguousarray(q), 0.05)
        ref, nn, npt = oracle.Octree(*cloud).mo(q, table, rcp, 0.05, counters=True)
        assert np.array_equal(mo, ref), npts
        assert np.array_equal(cnt[:, 0], nn)
    # all-black cloud: root is black, Mo = 0 after one node visit
    p, n, E, area = synth.ellipsoid_cloud(64, seed=3)
    mo, cnt, _, _ = run_gpu(mpss, torch_dev, (p, n, np.zeros_like(E), area), table, rcp,
                            synth.surface_queries(16, seed=2), 0.05)
    assert np.all(mo == 0) and np.all(cnt[:, 0] == 1)


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_mo_batch_sizes(mpss, torch_dev, wide_profile, mode):
    """q = 0 launches nothing and leaves the output alone; q above 2^30 and an empty point set
    are refused (MPSS_ERR_INVALID) before any launch; one query and 64 + 1 queries (a wave plus a
    one-lane tail) equal the same queries inside a larger batch."""
    table, rcp = wide_profile
    p, n, E, area = synth.ellipsoid_cloud(3000, radii=RADII, seed=31, black_frac=0.05)
    ctx = mpss.Context(max_error=0.1, exact_mo=mode)
    mid = ctx.set_material_tables(table, rcp, np.zeros(1025, np.float32))
    with pytest.raises(mpss.MpssError):
        ctx.set_irradiance_points(p[:0], n[:0], E[:0], area[:0])
    ctx.set_irradiance_points(p, n, E, area)
    q = synth.surface_queries(1100, radii=RADII, seed=37)
    qd = torch_dev.from_numpy(q).cuda()
    out = torch_dev.full((len(q), 30), -1.0, dtype=torch_dev.float32, device="cuda")
    ctx.mo_batch(mid, 0, qd.data_ptr(), out.data_ptr())
    torch_dev.cuda.synchronize()
    assert bool((out == -1.0).all())
    with pytest.raises(mpss.MpssError):
        ctx.mo_batch(mid, (1 << 30) + 1, qd.data_ptr(), out.data_ptr())
    ctx.mo_batch(mid, len(q), qd.data_ptr(), out.data_ptr())
    torch_dev.cuda.synchronize()
    full = out.cpu().numpy()
    for lo, m in ((0, 1), (700, 65)):
        part = torch_dev.zeros((m, 30), dtype=torch_dev.float32, device="cuda")
        ctx.mo_batch(mid, m, qd[lo:lo + m].contiguous().data_ptr(), part.data_ptr())
        torch_dev.cuda.synchronize()
        assert np.array_equal(part.cpu().numpy(), full[lo:lo + m]), (lo, m)
    ctx.close()


def test_layeredskin_material_on_device(oracle, mpss, torch_dev):
    """mpss_add_layeredskin builds the tables itself; they must match the oracle's."""
    ctx = mpss.Context(max_error=0.1)
    skin = mpss.default_skin(roughness=0.3, nmperunit=40e6, f_mel=0.5, f_eu=0.5, f_blood=0.5, f_ohg=0.5, Kt=[0.0] * 30,
                             desired_length=64)
    mid = ctx.add_layeredskin(skin)
    tab, rcp, rho, tot = ctx.material_tables(mid)
    ctx.close()
    mua, musp, th, eta = oracle.skin_layers(0.3, 40e6, 0.5, 0.5, 0.5, 0.5, (0.25e6, 20e6), (1.4, 1.4))
    tab_o, rcp_o, _, tot_o = oracle.compute_profile(mua, musp, eta, th, desired_length=64)
    assert np.array_equal(rcp, rcp_o)
    assert np.abs(tab - tab_o).max() <= 1e-6 * np.abs(tab_o).max()
    hd_o, _ = oracle.rho_table(0.3, 1.4)
    assert np.array_equal(rho, hd_o)


U = 2.0 ** -24


def _sum_bound(ref, nn, npt):
    """Per query and band, unfloored: the fast kernels form the reference's terms exactly and sum them in
    another order (a leaf's points first, one running sum per band), so each sum lies within 2 (n - 1) u
    of the exact one (n: the records the reference visits, u = 2^-24); the terms are non-negative."""
    n = (nn + npt).astype(np.float64)[:, None]
    return (4 * U + 2 * n * U) * np.abs(ref)


def _grid_bound(ref, nn, npt, table, cloud):
    """_sum_bound for the common-grid gather: every term's lookup within kCgRelTol (2e-6, 3e-6 here for a
    lerp between knots) of its value or kCgAbsTol (1e-14) of the band's peak (a bad cell's lanes read the
    exact tables), the fused lerp within a few ulp. The relative parts scale the result, and the absolute
    part is at most 1e-14 peak_c times the E_c * area of all points."""
    _, _, E, area = cloud
    peak = np.abs(table).max(axis=1).astype(np.float64)[None, :]
    mass = (E.astype(np.float64) * area.astype(np.float64)[:, None]).sum(axis=0)[None, :]
    return 3e-6 * np.abs(ref) + _sum_bound(ref, nn, npt) + 1e-14 * peak * mass


def _within(got, ref, bound):
    err = np.abs(got.astype(np.float64) - ref.astype(np.float64))
    return bool(np.all(err <= bound)), float((err / np.maximum(bound, 1e-300)).max())


@pytest.mark.parametrize("max_error", [0.05, 0.1])
def test_mo_packet_matches_reference_order(oracle, mpss, torch_dev, skin_profile, wide_profile, max_error):
    for (table, rcp), npts in ((skin_profile, 200000), (wide_profile, 50000)):
        cloud = synth.ellipsoid_cloud(npts, radii=RADII, seed=23, black_frac=0.05)
        q = synth.surface_queries(6001, radii=RADII, seed=29)
        fast, cnt_f, plain_f, _ = run_gpu(mpss, torch_dev, cloud, table, rcp, q, max_error, mode=2)
        band, cnt_b, plain_b, _ = run_gpu(mpss, torch_dev, cloud, table, rcp, q, max_error, mode=0,
                                          mo_common_grid=0)
        cg, cnt_g, plain_g, _ = run_gpu(mpss, torch_dev, cloud, table, rcp, q, max_error, mode=0)
        exact, cnt_e, _, _ = run_gpu(mpss, torch_dev, cloud, table, rcp, q, max_error, exact=True)
        ref, nn, npt = oracle.Octree(*cloud).mo(q, table, rcp, max_error, counters=True)
        assert np.array_equal(exact, ref)
        ok, worst = _within(fast, ref, _sum_bound(ref, nn, npt))
        assert ok, worst
        assert np.array_equal(cnt_f[:, 2:], cnt_e[:, 2:])  # same pruned traversal per query
        assert np.array_equal(fast == 0, ref == 0)
        # spectral sharding: same terms, same order per band -> bit-identical to the packet kernel
        assert np.array_equal(band, fast) and np.array_equal(plain_b, fast) and np.array_equal(plain_f, fast)
        # per-group pruning never visits more than the all-band traversal, per group
        assert np.all(cnt_b[:, 2] <= 8 * cnt_f[:, 2]) and np.all(cnt_b[:, 2] > 0)
        # the common grid: the same traversal, its far lookups resampled
        assert np.array_equal(cnt_g, cnt_b) and np.array_equal(plain_g, cg)
        ok, worst = _within(cg, ref, _grid_bound(ref, nn, npt, table, cloud))
        assert ok, worst
        assert np.array_equal(cg == 0, ref == 0)


def test_mo_packet_edge_cases(oracle, mpss, torch_dev, wide_profile):
    table, rcp = wide_profile
    for npts in (1, 9, 100):
        cloud = synth.ellipsoid_cloud(npts, radii=(0.002, 0.002, 0.002), seed=npts, black_frac=0.0)
        q = np.ascontiguousarray(np.concatenate([
            synth.surface_queries(61, radii=(0.002, 0.002, 0.002), seed=5, sort=False),
            cloud[0][:1], np.float32([[10.0, 10.0, 10.0]])]))  # 63 queries: ragged last packet
        fast, _, _, _ = run_gpu(mpss, torch_dev, cloud, table, rcp, q, 0.05, mode=2)
        band, _, _, _ = run_gpu(mpss, torch_dev, cloud, table, rcp, q, 0.05, mode=0, mo_common_grid=0)
        cg, _, _, _ = run_gpu(mpss, torch_dev, cloud, table, rcp, q, 0.05, mode=0)
        ref, nn, npt = oracle.Octree(*cloud).mo(q, table, rcp, 0.05, counters=True)
        assert _within(fast, ref, _sum_bound(ref, nn, npt))[0], npts
        assert np.array_equal(band, fast), npts
        assert _within(cg, ref, _grid_bound(ref, nn, npt, table, cloud))[0], npts


@pytest.mark.parametrize("cfg", [dict(mo_band_dealing=1), dict(mo_work_stealing=0), dict(mo_near_field=10236),
                                 dict(mo_band_dealing=1, mo_work_stealing=0, mo_near_field=10236)])
def test_mo_gather_choices_are_bit_identical(oracle, mpss, torch_dev, skin_profile, cfg):
    """The per-band gather (mo_common_grid 0) deals bands into adjacent-reach groups, lets
    workgroups steal other groups' units and keeps 5088 profile entries per band in LDS; snake-round
    groups (mo_band_dealing 1), per-XCD groups (mo_work_stealing 0) and the one-workgroup-per-CU near
    field (mo_near_field 10236) evaluate the same non-zero terms in the same order, so every sum
    must match bit for bit (and the oracle)."""
    cloud = synth.ellipsoid_cloud(120000, radii=RADII, seed=23, black_frac=0.05)
    q = synth.surface_queries(20000, radii=RADII, seed=29)
    table, rcp = skin_profile
    _, _, base, _ = run_gpu(mpss, torch_dev, cloud, table, rcp, q, 0.1, mode=0, mo_common_grid=0)
    packet, _, _, _ = run_gpu(mpss, torch_dev, cloud, table, rcp, q, 0.1, mode=2)
    _, _, alt, _ = run_gpu(mpss, torch_dev, cloud, table, rcp, q, 0.1, mode=0, mo_common_grid=0, **cfg)
    assert np.array_equal(base, alt)
    assert np.array_equal(base, packet)  # one running sum per band, the packet kernel's order
    ref, nn, npt = oracle.Octree(*cloud).mo(q, table, rcp, 0.1, counters=True)
    ok, worst = _within(base, ref, _sum_bound(ref, nn, npt))
    assert ok, worst
    assert np.any(ref > 0)


@pytest.mark.parametrize("cfg", [dict(), dict(mo_work_stealing=0), dict(mo_band_dealing=1), dict(mo_near_field=10236)])
def test_mo_common_grid_vs_oracle(oracle, mpss, torch_dev, skin_profile, cfg):
    """The default gather with the skin profile's common grid (accepted: mpss_get_gather_info) vs the
    reference-order oracle, 2e-5 relative as the per-band gather; the choices that do not change a bit
    with per-band tables do not change one with the common grid either (work stealing), and a
    different band dealing builds its own grid within the same bound."""
    cloud = synth.ellipsoid_cloud(120000, radii=RADII, seed=23, black_frac=0.05)
    q = synth.surface_queries(20000, radii=RADII, seed=29)
    table, rcp = skin_profile
    ctx = mpss.Context(max_error=0.1, **cfg)
    mid = ctx.set_material_tables(table, rcp, np.zeros(1025, np.float32))
    info = ctx.gather_info(mid)
    ctx.close()
    # every dealing gets rows: adjacent-reach groups (the default) from the near field's end; snake
    # rounds mix reaches 1:400 within a group, so their rows serve the stretch past the end of the
    # short-reach bands (CommonGrid::u1start), where only bands the grid follows are live
    assert info["common_grid"]
    assert info["l1_err"].max() <= 1e-7 and info["rel_err"].max() <= 2e-6
    _, _, cg, _ = run_gpu(mpss, torch_dev, cloud, table, rcp, q, 0.1, mode=0, **cfg)
    _, _, band, _ = run_gpu(mpss, torch_dev, cloud, table, rcp, q, 0.1, mode=0, mo_common_grid=0, **cfg)
    ref, nn, npt = oracle.Octree(*cloud).mo(q, table, rcp, 0.1, counters=True)
    # unfloored, per query and band, from the grid's guarantee (_grid_bound)
    ok, worst = _within(cg, ref, _grid_bound(ref, nn, npt, table, cloud))
    assert ok, worst
    if cfg.get("mo_band_dealing", 0) == 0:
        assert not np.array_equal(cg, band)  # the grid is in use (snake: its rows may lie past this cloud)
    if cfg.get("mo_work_stealing") == 0:
        _, _, base, _ = run_gpu(mpss, torch_dev, cloud, table, rcp, q, 0.1, mode=0)
        assert np.array_equal(base, cg)


def test_mo_gather_rejects_bad_choices(mpss, torch_dev):
    for cfg in (dict(mo_near_field=4096), dict(mo_band_dealing=2), dict(mo_common_grid=2)):
        with pytest.raises(mpss.MpssError):
            mpss.Context(**cfg)
