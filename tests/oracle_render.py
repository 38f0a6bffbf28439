"""ctypes front-end to the oracle's per-pixel path (oracle/render.c).

TEST INFRASTRUCTURE ONLY: used by tests/ as the parity checker and by bench.py's
cpu_baseline leg; never by the product package.
"""
import ctypes as C
import os
import time

import numpy as np

import oracle_lib

NB = 30
f32p = oracle_lib.f32p
vp = C.c_void_p

SURFACE_POINT = np.dtype([("p", "<f4", 3), ("n", "<f4", 3), ("u", "<f4"), ("v", "<f4"), ("material", "<u4"),
                          ("area", "<f4"), ("ray_eps", "<f4")])


def _lib():
    L = oracle_lib.lib()
    if getattr(L, "_render_sigs", False):
        return L
    L.o_scene_create.restype = vp
    L.o_scene_create.argtypes = [C.c_int, C.c_int, f32p, f32p]
    L.o_scene_add_material.restype = C.c_int
    L.o_scene_add_material.argtypes = [vp, f32p, f32p, f32p, C.c_float, C.c_float, C.c_float, C.c_int, f32p,
                                       C.c_int, C.c_int, f32p, C.c_int, f32p]
    L.o_scene_set_material_rgb.restype = C.c_int
    L.o_scene_set_material_rgb.argtypes = [vp, C.c_int, C.c_int]
    L.o_scene_set_material_no_bssrdf.restype = C.c_int
    L.o_scene_set_material_no_bssrdf.argtypes = [vp, C.c_int, C.c_int]
    L.o_scene_add_mesh.restype = C.c_int
    L.o_scene_add_mesh.argtypes = [vp, C.c_int, f32p, vp, vp, vp, C.c_int, oracle_lib.i32p, f32p, f32p, C.c_int,
                                   C.c_int]
    L.o_scene_add_sphere_light.restype = C.c_int
    L.o_scene_add_sphere_light.argtypes = [vp, f32p, C.c_float, f32p, C.c_int]
    L.o_scene_add_infinite_light.restype = C.c_int
    L.o_scene_add_infinite_light.argtypes = [vp, f32p, C.c_int, f32p, f32p, C.c_int, C.c_int, vp]
    L.o_poisson_points.restype = C.c_long
    L.o_poisson_points.argtypes = [vp, C.c_float, C.c_int, C.c_uint32, vp, C.c_long]
    L.o_tessellate.restype = C.c_long
    L.o_tessellate.argtypes = [vp, C.c_float, C.c_int, vp, C.c_long]
    L.o_irradiance.argtypes = [vp, C.c_int, vp, C.c_uint32, C.c_int, f32p]
    L.o_scene_set_octree.argtypes = [vp, C.c_int, f32p, f32p, f32p, f32p, C.c_float]
    L.o_render_tile.argtypes = [vp, C.c_int, C.c_uint32, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, f32p]
    L.o_scene_free.argtypes = [vp]
    L.o_scene_set_material_texture.restype = C.c_int
    L.o_scene_set_material_texture.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, vp, C.c_float, C.c_float,
                                               C.c_float, C.c_int, C.c_int, C.c_float, C.c_float, C.c_float,
                                               C.c_float, C.c_float]
    L.o_imagemap_lookup.restype = C.c_int
    L.o_imagemap_lookup.argtypes = [C.c_int, C.c_int, vp, C.c_int, C.c_float, C.c_float, C.c_float, C.c_int, C.c_int,
                                    C.c_float, C.c_float, C.c_float, C.c_float, C.c_float, C.c_int, f32p, f32p]
    L.o_replay_render_table.restype = C.c_int
    L.o_replay_render_table.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, vp]
    L.o_replay_irradiance_scr.argtypes = [C.c_int, C.c_int, C.c_int, vp]
    L.o_irradiance_replay.argtypes = [vp, C.c_int, vp, vp, C.c_int, f32p]
    L.o_render_tile_replay.argtypes = [vp, C.c_int, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, f32p]
    L.o_replay_render_table_window.restype = C.c_int
    L.o_replay_render_table_window.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int] + [C.c_int] * 4 + [vp]
    L.o_render_tile_replay_window.argtypes = [vp, C.c_int, vp, C.c_int] + [C.c_int] * 9 + [f32p]
    L.o_cpu_baseline.restype = C.c_long
    L.o_cpu_baseline.argtypes = [vp, C.c_int, C.c_uint32, C.c_int, C.c_int, C.c_double, vp, C.c_int,
                                 C.POINTER(C.c_long), C.POINTER(C.c_double)]
    L.o_render_task_count.restype = C.c_int
    L.o_render_task_count.argtypes = [C.c_int, C.c_int, C.c_int]
    L.o_sub_window.argtypes = [C.c_int] * 6 + [vp]
    L._render_sigs = True
    return L


_WRAP = {"repeat": 0, "black": 1, "clamp": 2}


def _tex_args(tex):
    """(W, H, texels, keep-alive array, params after texels) of an mpss.imagemap kwargs dict."""
    arr = None if tex.get("texels") is None else np.ascontiguousarray(tex["texels"], np.float32)
    H, W = (0, 0) if arr is None else arr.shape[:2]
    rest = [float(tex.get("shift", 0.0)), float(tex.get("scale", 1.0)), float(tex.get("gamma", 1.0)),
            _WRAP[tex.get("wrap", "repeat")], int(bool(tex.get("trilinear", False))),
            float(tex.get("maxanisotropy", 8.0)), float(tex.get("uscale", 1.0)), float(tex.get("vscale", 1.0)),
            float(tex.get("udelta", 0.0)), float(tex.get("vdelta", 0.0))]
    return W, H, (None if arr is None else arr.ctypes.data), arr, rest


def imagemap_lookup(tex, uvd):
    """The oracle's ImageTexture::Evaluate (oracle/texture.c) at uvd (n, 6) = u, v, dudx, dvdx,
    dudy, dvdy; tex = mpss.imagemap kwargs dict."""
    W, H, ptr, arr, rest = _tex_args(tex)
    uvd = np.ascontiguousarray(uvd, np.float32).reshape(-1, 6)
    out = np.zeros((len(uvd), 3), np.float32)
    _lib().o_imagemap_lookup(W, H, ptr, int(bool(tex.get("is_float", False))), *rest, len(uvd), uvd, out)
    return out


_TEXKEYS = ("Kr", "Kt", "albedo", "albedo_tex", "bump_tex")


def _opt(a):
    return None if a is None else np.ascontiguousarray(a, np.float32)


def tables_from_ctx(ctx, n):
    return [ctx.material_tables(i)[:3] for i in range(n)]


def tables_from_oracle(sc):
    """Material tables built by the oracle itself (oracle/skin.c + mpc.c + kissfft.c, oracle/rho.c):
    LayeredSkin's layers (layeredskin.cpp:47-89), ComputeMultipoleProfile at the material's
    desiredlength with lerponthinslab (multipole.cpp:241-295), rgbprofile's three RGB profiles
    (multipole.cpp:408-451: rows c % 3), and ComputeRhoDataFromBxDF (multipole.cpp:521-549). With
    these and the oracle's own irradiance, an image comparison shares nothing with the product but
    the scene description."""
    import oracle_lib
    out = []
    for m in sc.materials:
        if not m.get("gen_profile", 1):  # preparedBSSRDFData = NULL: nothing is read (o_mat.no_bssrdf)
            out.append((np.zeros((NB, 2), np.float32), np.ones(NB, np.float32), np.zeros(2, np.float32)))
            continue
        if m.get("show_irradiance_points"):
            out.append(irradiance_points_tables(m.get("irradiance_point_size", 0.002)))
            continue
        th = tuple(m.get("layer_thickness_nm", (0.25e6, 20e6)))
        ior = tuple(m.get("layer_ior", (1.4, 1.4)))
        rough = m.get("roughness", 0.3)
        mua, musp, thk, eta = oracle_lib.skin_layers(rough, m.get("nmperunit", 40e6), m.get("f_mel", 0.5),
                                                     m.get("f_eu", 0.5), m.get("f_blood", 0.5), m.get("f_ohg", 0.5),
                                                     th, ior)
        if m.get("rgb_profile"):
            ra = np.stack([oracle_lib.to_rgb(x) for x in mua])
            rs = np.stack([oracle_lib.to_rgb(x) for x in musp])
            idx = np.arange(NB) % 3
            mua, musp = ra[:, idx].astype(np.float32), rs[:, idx].astype(np.float32)
        tab, rcp, _, _ = oracle_lib.compute_profile(mua, musp, eta, thk, desired_length=int(m.get("desired_length", 512)),
                                                    lerp=bool(m.get("lerp_on_thin_slab", 1)))
        rho, _ = oracle_lib.rho_table(rough, ior[0], fixed=bool(m.get("double_ref_sslf", 0)))
        out.append((tab, rcp, rho))
    return out


def irradiance_points_tables(radius):
    """ComputeIrradiancePointsProfile(radius) (multipole.cpp:551-567) and ComputeRoughRhoData
    (:569-572), restated: each band {1/area, 1/area} with area = float(M_PI * r * r) (a double
    product), dsqSpacing = r * r (float), rcp = 1 / dsqSpacing; rho_hd = {0, 0}."""
    r = np.float32(radius)
    area = np.float32(np.float64(np.pi) * np.float64(r) * np.float64(r))
    v = np.float32(1.0) / area
    rcp = np.float32(1.0) / (r * r)
    return (np.full((NB, 2), v, np.float32), np.full(NB, rcp, np.float32), np.zeros(2, np.float32))


def tables_from_host(sc, mpss):
    """Material tables from the product's host builders (CPU only; no device needed)."""
    out = []
    for m in sc.materials:
        kw = {k: v for k, v in m.items() if k not in _TEXKEYS}
        skin = mpss.default_skin(**kw)
        tab, rcp, _ = mpss.host_build_profile(*mpss.host_skin_layers(skin), desired_length=skin.desired_length,
                                              lerp=bool(skin.lerp_on_thin_slab))
        rho, _ = mpss.host_rho_table(skin.roughness, skin.layer_ior[0], double_ref_sslf=bool(skin.double_ref_sslf))
        out.append((tab, rcp, rho))
    return out


class OracleScene:
    """The oracle's copy of a pbrtscene.Scene. Material tables (Rd profile, rho_hd) come
    from the product (its context or its host builders), so this checks the per-pixel path
    in isolation; the tables themselves are checked against the oracle in
    test_host_parity.py. cfg: an mpss.Config (or anything with the same fields)."""

    def __init__(self, sc, tables, cfg, mpss):
        L = _lib()
        r2c, c2w = sc.raster_to_camera()
        self.sc = sc
        self.h = L.o_scene_create(sc.xres, sc.yres, np.ascontiguousarray(r2c, np.float32),
                                  np.ascontiguousarray(c2w, np.float32))
        self._keep = []
        for mid, m in enumerate(sc.materials):
            kw = {k: v for k, v in m.items() if k not in _TEXKEYS}
            skin = mpss.default_skin(**kw)
            Kr = mpss.host_from_rgb(m["Kr"]) if "Kr" in m else np.ones(NB, np.float32)
            Kt = mpss.host_from_rgb(m["Kt"]) if "Kt" in m else np.ones(NB, np.float32)
            alb = mpss.host_from_rgb(m["albedo"]) if "albedo" in m else np.ones(NB, np.float32)
            tab, rcp, rho = tables[mid]
            L.o_scene_add_material(self.h, Kr, Kt, alb, cfg.mix, skin.roughness, skin.layer_ior[0],
                                   int(skin.double_ref_sslf), rho, len(rho), int(skin.use_monte_carlo),
                                   np.ascontiguousarray(tab, np.float32), tab.shape[1], rcp)
            if skin.rgb_profile and skin.gen_profile and not skin.show_irradiance_points:
                assert L.o_scene_set_material_rgb(self.h, mid, 1) == 0
            if not skin.gen_profile:
                assert L.o_scene_set_material_no_bssrdf(self.h, mid, 1) == 0
            for which, key in ((0, "albedo_tex"), (1, "bump_tex")):
                if m.get(key) is not None:
                    W, H, ptr, arr, rest = _tex_args(m[key])
                    assert L.o_scene_set_material_texture(self.h, mid, which, W, H, ptr, *rest) == 0
        for me in sc.meshes:
            N, S, uv = _opt(me["N"]), _opt(me["S"]), _opt(me["uv"])
            self._keep += [N, S, uv]
            det = np.linalg.det(me["o2w"][:3, :3].astype(np.float64))
            flip = int(bool(me["reverse"]) ^ bool(det < 0))
            L.o_scene_add_mesh(self.h, len(me["P"]), np.ascontiguousarray(me["P"], np.float32),
                               None if N is None else N.ctypes.data, None if S is None else S.ctypes.data,
                               None if uv is None else uv.ctypes.data, len(me["indices"]),
                               np.ascontiguousarray(me["indices"], np.int32), me["o2w"], me["w2o"], flip,
                               me["material"])
        for li in sc.lights:
            ns = li["nsamples"] if not cfg.quick_render else max(1, li["nsamples"] // 4)
            if li.get("kind") == "infinite":
                Lsc = (oracle_lib.from_rgb(li["L"]) * oracle_lib.from_rgb(li["scale"])).astype(np.float32)
                from mpss import pbrtscene
                tex = pbrtscene.infinite_texels(li)
                H, W = (0, 0) if tex is None else tex.shape[:2]
                rc = L.o_scene_add_infinite_light(self.h, Lsc, ns, np.ascontiguousarray(li["l2w"], np.float32),
                                                  np.ascontiguousarray(li["w2l"], np.float32), W, H,
                                                  None if tex is None else tex.ctypes.data)
                assert rc >= 0
                continue
            L.o_scene_add_sphere_light(self.h, np.ascontiguousarray(li["center"], np.float32), li["radius"],
                                       mpss.host_from_rgb(li["L"]), ns)
        self.max_error = cfg.max_error * (4 if cfg.quick_render else 1)
        self.min_dist = cfg.min_sample_distance * (4 if cfg.quick_render else 1)
        self.quick = bool(cfg.quick_render)

    def close(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib().o_scene_free(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def tessellate(self, incenter=False):
        L = _lib()
        n = L.o_tessellate(self.h, self.min_dist, int(incenter), None, 0)
        out = np.zeros(n, SURFACE_POINT)
        L.o_tessellate(self.h, self.min_dist, int(incenter), out.ctypes.data, n)
        return out

    def poisson_points(self, seed, cap=1 << 22, min_dist=None):
        """FindPoissonPointDistribution (one task, replay-mode random numbers)."""
        out = np.zeros(cap, SURFACE_POINT)
        md = self.min_dist if min_dist is None else min_dist
        n = _lib().o_poisson_points(self.h, md, int(self.quick), seed, out.ctypes.data, cap)
        if n < 0:
            raise RuntimeError("o_poisson_points failed (%d)" % n)
        return out[:n]

    def irradiance(self, pts, seed, nthreads=None):
        pts = np.ascontiguousarray(pts, SURFACE_POINT)
        E = np.zeros((len(pts), NB), np.float32)
        _lib().o_irradiance(self.h, len(pts), pts.ctypes.data, seed, nthreads or os.cpu_count(), E)
        return E

    # ---- the reference sampler (oracle/render.c o_replay_*)
    def replay_table(self, spp, cores=8, li_draws=6, nthreads=None):
        """Sample values of the whole sample extent: (yres+1, xres+1, spp, K) float32."""
        L = _lib()
        K = L.o_replay_render_table(self.h, spp, cores, li_draws, 1, None)
        vals = np.zeros((self.sc.yres + 1, self.sc.xres + 1, spp, K), np.float32)
        L.o_replay_render_table(self.h, spp, cores, li_draws, nthreads or os.cpu_count(), vals.ctypes.data)
        return vals

    def replay_window(self, x0, x1, y0, y1):
        """The sample-extent pixels a tile's film needs: the tile plus a one-pixel border."""
        return (max(x0 - 1, 0), min(x1 + 1, self.sc.xres + 1), max(y0 - 1, 0), min(y1 + 1, self.sc.yres + 1))

    def replay_table_window(self, spp, window, cores=8, li_draws=6, nthreads=None):
        """replay_table restricted to window = (vx0, vx1, vy0, vy1) of the sample extent (only the
        render tasks whose sub-window meets it run): (vy1-vy0, vx1-vx0, spp, K) float32."""
        L = _lib()
        vx0, vx1, vy0, vy1 = window
        K = L.o_replay_render_table(self.h, spp, cores, li_draws, 1, None)
        vals = np.zeros((vy1 - vy0, vx1 - vx0, spp, K), np.float32)
        L.o_replay_render_table_window(self.h, spp, cores, li_draws, nthreads or os.cpu_count(), vx0, vx1, vy0, vy1,
                                       vals.ctypes.data)
        return vals

    def irradiance_replay(self, pts, cores=8, nthreads=None, n_total=None):
        """IrradianceTask with the reference sampler's RNG(47 k) scrambles; pts may be a prefix of
        n_total points (the task split depends on the whole point count)."""
        pts = np.ascontiguousarray(pts, SURFACE_POINT)
        n_total = n_total or len(pts)
        scr = np.zeros((n_total, max(1, len(self.sc.lights)), 2), np.uint32)
        _lib().o_replay_irradiance_scr(n_total, len(self.sc.lights), cores, scr.ctypes.data)
        scr = np.ascontiguousarray(scr[:len(pts)])
        E = np.zeros((len(pts), NB), np.float32)
        _lib().o_irradiance_replay(self.h, len(pts), pts.ctypes.data, scr.ctypes.data, nthreads or os.cpu_count(), E)
        return E

    def render_tile_replay(self, spp, vals, x0, x1, y0, y1, nthreads=None, window=None):
        """vals: replay_table (whole extent) or, with window, replay_table_window(window)."""
        vals = np.ascontiguousarray(vals, np.float32)
        out = np.zeros(((y1 - y0) * (x1 - x0) * 4,), np.float32)
        if window is None:
            _lib().o_render_tile_replay(self.h, spp, vals.ctypes.data, vals.shape[-1], x0, x1, y0, y1,
                                        nthreads or os.cpu_count(), out)
        else:
            _lib().o_render_tile_replay_window(self.h, spp, vals.ctypes.data, vals.shape[-1], *window, x0, x1, y0, y1,
                                               nthreads or os.cpu_count(), out)
        return out.reshape(y1 - y0, x1 - x0, 4)

    def set_octree(self, pts, E):
        p = np.ascontiguousarray(pts["p"], np.float32)
        n = np.ascontiguousarray(pts["n"], np.float32)
        a = np.ascontiguousarray(pts["area"], np.float32)
        _lib().o_scene_set_octree(self.h, len(pts), p, n, np.ascontiguousarray(E, np.float32), a, self.max_error)

    def render_tile(self, spp, seed, x0, x1, y0, y1, nthreads=None):
        out = np.zeros(((y1 - y0) * (x1 - x0) * 4,), np.float32)
        _lib().o_render_tile(self.h, spp, seed, x0, x1, y0, y1, nthreads or os.cpu_count(), out)
        return out.reshape(y1 - y0, x1 - x0, 4)


def render_task_count(xres, yres, cores):
    return _lib().o_render_task_count(xres, yres, cores)


def sub_window(num, count, xs, xe, ys, ye):
    out = np.zeros(4, np.int32)
    _lib().o_sub_window(num, count, xs, xe, ys, ye, out.ctypes.data)
    return tuple(int(v) for v in out)


def host_cpus():
    """CPUs this process may run on: its affinity mask, capped by the cgroup CPU quota. On the GPU
    box nproc counts the whole host's CPUs, while a job gets a share of them (16 per GPU); threads
    beyond the share only contend."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            with open(path) as f:
                parts = f.read().split()
            if path.endswith("cpu.max"):
                quota, period = parts[0], parts[1]
            else:
                quota = parts[0]
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                    period = f.read().split()[0]
            if quota not in ("max", "-1"):
                n = min(n, max(1, int(quota) // int(period)))
            break
        except (OSError, ValueError, IndexError):
            continue
    return max(1, n)


def time_cpu_baseline(sc, ctx, spp, seed, seconds, nthreads=None):
    """Time the oracle's pixel loop the way SamplerRenderer::Render runs (samplerrenderer.cpp:
    191-225): nTasks = RoundUpPow2(max(32 * cores, W * H / 256)) sub-windows of the frame, pulled
    from one shared counter by a pool of one worker per host core, in a fixed random order until
    `seconds` pass (a bounded sample of the same frame). The octree is built from the product's
    Preprocess outputs (surface points + irradiance); Preprocess is not timed."""
    import mpss
    cores = host_cpus()
    nthreads = nthreads or cores
    osc = OracleScene(sc, tables_from_ctx(ctx, len(sc.materials)), ctx.cfg, mpss)
    osc.set_octree(ctx.surface_points(), ctx.irradiance())
    ntasks = render_task_count(sc.xres, sc.yres, cores)
    order = np.random.default_rng(1234).permutation(ntasks).astype(np.int32)
    tasks, el = C.c_long(), C.c_double()
    px = _lib().o_cpu_baseline(osc.h, spp, seed, cores, nthreads, float(seconds), order.ctypes.data, ntasks,
                               C.byref(tasks), C.byref(el))
    osc.close()
    dt = el.value
    return {"value": round(px * spp / dt / 1e6, 4), "unit": "Msamples/s", "cores": nthreads, "kind": "port",
            "nproc": os.cpu_count(), "cpu_share": cores,
            "sample": "%d of %d render tasks (pbrt's split RoundUpPow2(max(32 x %d cores, W*H/256)), %d px x %d spp, "
                      "%.1f %% of the frame) in fixed random order, one pool of %d threads, %.1f s; oracle/render.c "
                      "(scalar C restatement, pthreads)" % (tasks.value, ntasks, cores, px, spp,
                                                           100.0 * px / (sc.xres * sc.yres), nthreads, dt),
            "frame_fraction": round(px / float(sc.xres * sc.yres), 4)}
