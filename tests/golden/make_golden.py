"""Regenerates tests/golden/golden.npz from the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY. The reference ships no golden vectors for this path and could not be
built or run here, so these fixtures are the oracle's own outputs, frozen: they
pin the restatement against drift (tests/test_golden.py regenerates and compares bit for bit)
and give the GPU tests fixed expected values (tests/test_golden_gpu.py). Inputs:

  profile_512   LayeredSkin of S007Scene.pbrt:35-47 (roughness 0.3, nmperunit 40e6, layers
                0.25e6 / 20e6 nm, ior 1.4, f_mel = f_eu = f_blood = f_ohg = 0.5) at desiredlength
                512 with lerponthinslab (multipole.cpp:241-295): every 61st entry and the first 512
                of each band, rcp[30], totalReflectance[30]
  profile_64    the same material at desiredlength 64, whole table
  rho           rho_hd[1025] and rho_hh of Microfacet(1, Fresnel(1, 1.4), Beckmann(0.3)),
                256^2 samples per entry (multipole.cpp:466-549)
  mo            Mo() (diffusionutil.h:175-210) of 4096 Morton-ordered surface queries over a
                50,000-point ellipsoid cloud (tests/synth.py, seeds 31/32; the cloud's SHA-256 is
                stored) with profile_64 at maxError 0.05; per-query node / point visit counts
  image         skin.pbrt at 32x32, 4 spp, minsampledistance 0.01, desiredlength 64, oracle
                tables: tessellation SHA-256, irradiance (seed 7) SHA-256, film XYZW (seed 9)

Run:  python tests/golden/make_golden.py   (about 15 s on 8 cores)
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "pbrt-v2-skin_amd"), ROOT]

SKIN = (0.3, 40e6, 0.5, 0.5, 0.5, 0.5, (0.25e6, 20e6), (1.4, 1.4))
SUB = 61


def sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def profile_sub_index(L):
    return np.unique(np.concatenate([np.arange(min(L, 512)), np.arange(0, L, SUB)])).astype(np.int64)


def mo_inputs():
    import synth
    cloud = synth.ellipsoid_cloud(50000, seed=31, black_frac=0.05)
    q = synth.surface_queries(4096, seed=32)
    return cloud, q


def image_scene():
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin.pbrt"), xres=32, yres=32, spp=4)
    sc.integrator["minsampledistance"] = 0.01
    for m in sc.materials:
        m["desired_length"] = 64
    return sc


def oracle_tables(oracle, desired):
    mua, musp, th, eta = oracle.skin_layers(*SKIN)
    tab, rcp, _, tot = oracle.compute_profile(mua, musp, eta, th, desired_length=desired)
    return tab, rcp, tot


def compute(oracle):
    import mpss
    import oracle_render as orr
    out = {}
    tab, rcp, tot = oracle_tables(oracle, 512)
    idx = profile_sub_index(tab.shape[1])
    out.update(profile_512_len=np.int64(tab.shape[1]), profile_512_idx=idx, profile_512=tab[:, idx],
               profile_512_rcp=rcp, profile_512_total=tot)
    tab64, rcp64, tot64 = oracle_tables(oracle, 64)
    out.update(profile_64=tab64, profile_64_rcp=rcp64, profile_64_total=tot64)
    hd, hh = oracle.rho_table(0.3, 1.4)
    out.update(rho_hd=hd, rho_hh=np.float32(hh))
    (p, n, E, area), q = mo_inputs()
    mo, nn, npt = oracle.Octree(p, n, E, area).mo(q, tab64, rcp64, 0.05, counters=True)
    out.update(mo_cloud_sha=np.array(sha(p, n, E, area, q)), mo=mo, mo_nodes=nn, mo_points=npt,
               mo_max_error=np.float32(0.05))
    sc = image_scene()
    from mpss import pbrtscene
    cfg = mpss.default_config(**pbrtscene.integrator_config(sc))
    o = orr.OracleScene(sc, [(tab64, rcp64, hd)], cfg, mpss)
    pts = o.tessellate()
    E = o.irradiance(pts, 7)
    o.set_octree(pts, E)
    img = o.render_tile(sc.spp, 9, 0, sc.xres, 0, sc.yres)
    o.close()
    out.update(image_points_sha=np.array(sha(pts)), image_points_n=np.int64(len(pts)),
               image_irradiance_sha=np.array(sha(E)), image_xyzw=img)
    return out


if __name__ == "__main__":
    import oracle_lib
    oracle_lib.build()
    data = compute(oracle_lib)
    path = os.path.join(HERE, "golden.npz")
    np.savez_compressed(path, **data)
    print("wrote %s (%d KB)" % (path, os.path.getsize(path) // 1024))
