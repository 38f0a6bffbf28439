"""Mo() with the closed-form single dipole on the GPU (row a21; reference
src/integrators/diffusionutil.h:38-83 used through Mo, :175-210, as dipolesubsurface.cpp:171-172
does).

1. A dipole material (mpss_add_dipole_material) runs the reference-order gather with the closed
   form per band: against the oracle's Mo with DiffusionReflectance, 1e-6 relative (exp is
   evaluated in double by OCML and by glibc and rounded once; everything else is the same
   float sequence), and the same node/point visit counts.
2. maxError -> 0: the GPU gather equals the brute-force sum of the closed form over every point.
3. The production sharded gather with a profile TABULATED from the closed form (uniform in d^2,
   the layout of MultipoleProfileData) against the brute-force closed-form sum at maxError -> 0:
   the only difference is the table's linear interpolation (bounded here at 2e-3).
"""
import numpy as np
import pytest

import synth

pytestmark = pytest.mark.gpu

NB = 30
RADII = (0.05, 0.06, 0.07)
SIGMA_A = np.array([0.5 + 0.1 * c for c in range(NB)], np.float32)
SIGMAP_S = np.array([40.0 + 1.5 * c for c in range(NB)], np.float32)
ETA = 1.3


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch


@pytest.fixture(scope="module")
def scene():
    cloud = synth.ellipsoid_cloud(6000, radii=RADII, seed=21)
    q = synth.surface_queries(1024, radii=RADII, seed=22)
    return cloud, q


def brute(mpss, cloud, q):
    p, _, E, area = cloud
    out = np.zeros((len(q), NB))
    for i, x in enumerate(q):
        d2 = ((p - x) ** 2).sum(1, dtype=np.float32)
        rd, _ = mpss.host_dipole_rd(SIGMA_A, SIGMAP_S, ETA, d2)
        out[i] = (rd.astype(np.float64) * E * area[:, None]).sum(0)
    return out


def gpu_mo(mpss, torch, cloud, q, max_error, table=None, mode=1):
    ctx = mpss.Context(max_error=max_error, exact_mo=mode)
    if table is None:
        mid = ctx.add_dipole_material(SIGMA_A, SIGMAP_S, ETA)
    else:
        mid = ctx.set_material_tables(table[0], table[1], np.zeros(1025, np.float32))
    ctx.set_irradiance_points(*cloud)
    qd = torch.from_numpy(q).cuda()
    out = torch.zeros((len(q), NB), dtype=torch.float32, device="cuda")
    cnt = torch.zeros((len(q), 4), dtype=torch.int32, device="cuda")
    ctx.mo_batch(mid, len(q), qd.data_ptr(), out.data_ptr(), cnt.data_ptr())
    torch.cuda.synchronize()
    res = out.cpu().numpy(), cnt.cpu().numpy()
    ctx.close()
    return res


@pytest.mark.parametrize("max_error", [0.05, 0.2])
def test_dipole_material_vs_oracle(mpss, oracle, torch_dev, scene, max_error):
    cloud, q = scene
    got, cnt = gpu_mo(mpss, torch_dev, cloud, q, max_error)
    t = oracle.Octree(*cloud)
    ref, nn, npt = t.mo_diffusion(q, oracle.Diffusion(SIGMA_A, SIGMAP_S, ETA), max_error, counters=True)
    scale = np.maximum(np.abs(ref), np.abs(ref).max(axis=1, keepdims=True) * 1e-3)
    assert np.all(np.abs(got - ref) <= 1e-6 * scale + 1e-37)
    assert np.mean(got == ref) > 0.99
    assert np.array_equal(cnt[:, 0], nn) and np.array_equal(cnt[:, 1], npt)


def test_dipole_material_zero_error_is_brute_force(mpss, torch_dev, scene):
    cloud, q = scene
    q = q[::8]
    got, _ = gpu_mo(mpss, torch_dev, cloud, q, 0.0)
    ref = brute(mpss, cloud, q)
    assert np.allclose(got, ref, rtol=2e-5, atol=0)


def test_tabulated_dipole_through_sharded_gather(mpss, torch_dev, scene):
    cloud, q = scene
    q = q[::8]
    p = cloud[0]
    L = 65536
    d2max = float(((p.max(0) - p.min(0)) ** 2).sum()) * 1.01
    spacing = np.float32(d2max / (L - 1))
    grid = (np.arange(L, dtype=np.float64) * spacing).astype(np.float32)
    rd, _ = mpss.host_dipole_rd(SIGMA_A, SIGMAP_S, ETA, grid)
    table = np.ascontiguousarray(rd.T)
    rcp = np.full(NB, 1.0 / spacing, np.float32)
    got, _ = gpu_mo(mpss, torch_dev, cloud, q, 1e-6, table=(table, rcp), mode=0)
    ref = brute(mpss, cloud, q)
    assert np.allclose(got, ref, rtol=2e-3, atol=0)
