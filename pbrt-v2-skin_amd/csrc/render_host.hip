// render_host.cpp -- host driver of the per-pixel path: scene upload, Preprocess
// (tessellation -> irradiance kernel -> octree) and tiled rendering (render.hip kernels).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <unordered_map>

#include "context.h"
#include "envmap.h"
#include "render.h"
#include "spectral.h"
#include "texture_build.h"

namespace mpss {

namespace {
int round_up_pow2(int v) {
    int r = 1;
    while (r < v) r <<= 1;
    return r;
}
float det3(const float *m) {
    return m[0] * (m[5] * m[10] - m[6] * m[9]) - m[1] * (m[4] * m[10] - m[6] * m[8]) +
           m[2] * (m[4] * m[9] - m[5] * m[8]);
}
int bvh_depth(const std::vector<BvhNode> &n, int i) {
    if (n[i].nprims > 0) return 1;
    return 1 + std::max(bvh_depth(n, i + 1), bvh_depth(n, n[i].offset));
}
}  // namespace

void Context::add_mesh(uint32_t nv, const float *P, const float *N, const float *S, const float *uv, uint32_t nt,
                       const int32_t *idx, const float *o2w, const float *w2o, bool reverse, uint32_t material) {
    std::lock_guard<std::mutex> g(mu_);
    if (material >= materials_.size()) throw Error(MPSS_ERR_INVALID, "add_mesh: unknown material id");
    if (materials_[material]->dipole)
        throw Error(MPSS_ERR_INVALID, "add_mesh: a dipole material is an Rd functor for mpss_mo_batch, not a surface");
    Mesh m;
    m.P.assign(P, P + 3 * (size_t)nv);
    if (N) m.N.assign(N, N + 3 * (size_t)nv);
    if (S) m.S.assign(S, S + 3 * (size_t)nv);
    if (uv) m.uv.assign(uv, uv + 2 * (size_t)nv);
    m.idx.assign(idx, idx + 3 * (size_t)nt);
    for (uint32_t i = 0; i < 3 * nt; ++i)
        if (m.idx[i] < 0 || (uint32_t)m.idx[i] >= nv) throw Error(MPSS_ERR_INVALID, "add_mesh: vertex index out of range");
    memcpy(m.o2w, o2w, sizeof(m.o2w));
    memcpy(m.w2o, w2o, sizeof(m.w2o));
    m.material = material;
    m.reverse_orientation = reverse;
    m.swaps_handedness = det3(o2w) < 0.f;  // Transform::SwapsHandedness
    scene_.meshes.push_back(std::move(m));
    scene_dirty_ = true;
}

void Context::add_sphere_light(const float *c, float r, const float *Lemit, int nsamples) {
    std::lock_guard<std::mutex> g(mu_);
    if (!(r > 0.f)) throw Error(MPSS_ERR_INVALID, "add_sphere_light: radius must be positive");
    if (nsamples < 1) throw Error(MPSS_ERR_INVALID, "add_sphere_light: nsamples must be >= 1");
    if (scene_.lights.size() >= 254) throw Error(MPSS_ERR_INVALID, "add_sphere_light: at most 254 lights");
    SceneLight l;
    memcpy(l.center, c, sizeof(l.center));
    l.radius = r;
    memcpy(l.Lemit, Lemit, sizeof(l.Lemit));
    l.nsamples = cfg_.quick_render ? std::max(1, nsamples / 4) : nsamples;  // CreateDiffuseAreaLight
    scene_.lights.push_back(l);
    scene_dirty_ = true;
}

// CreateInfiniteLight + the InfiniteAreaLight ctor without a map (lights/infinite.cpp:66-90,
// 180-188): texels[0] = L.ToRGBSpectrum(); Le and Sample_L convert map lookups back with
// Spectrum(rgb, SPECTRUM_ILLUMINANT) on the device (render.hip).
void Context::add_infinite_light(const float *L, int nsamples, const float *l2w, const float *w2l, int W, int H,
                                 const float *texels) {
    std::lock_guard<std::mutex> g(mu_);
    if (nsamples < 1) throw Error(MPSS_ERR_INVALID, "add_infinite_light: nsamples must be >= 1");
    if (scene_.lights.size() >= 254) throw Error(MPSS_ERR_INVALID, "add_infinite_light: at most 254 lights");
    if (texels && (W < 1 || H < 1 || (int64_t)W * H > (int64_t)1 << 28))
        throw Error(MPSS_ERR_INVALID, "add_infinite_light: bad map resolution");
    SceneLight l;
    l.kind = 1;
    l.center[0] = l.center[1] = l.center[2] = 0.f;
    l.radius = 0.f;
    memcpy(l.Lemit, L, sizeof(l.Lemit));
    float rgb[3];
    spectrum_to_rgb(L, rgb);  // L.ToRGBSpectrum()
    if (texels) {             // texels[i] *= L.ToRGBSpectrum()
        l.map_w = W;
        l.map_h = H;
        l.map.resize((size_t)W * H * 3);
        for (size_t i = 0; i < (size_t)W * H; ++i)
            for (int k = 0; k < 3; ++k) l.map[3 * i + k] = texels[3 * i + k] * rgb[k];
    } else {
        l.map_w = l.map_h = 1;
        l.map.assign(rgb, rgb + 3);
    }
    for (int r = 0; r < 3; ++r)
        for (int k = 0; k < 3; ++k) {
            l.l2w[3 * r + k] = l2w[4 * r + k];
            l.w2l[3 * r + k] = w2l[4 * r + k];
        }
    l.nsamples = cfg_.quick_render ? std::max(1, nsamples / 4) : nsamples;  // CreateInfiniteLight
    scene_.lights.push_back(std::move(l));
    scene_dirty_ = true;
}

void Context::set_camera(const float *r2c, const float *c2w, int xres, int yres) {
    std::lock_guard<std::mutex> g(mu_);
    if (xres <= 0 || yres <= 0) throw Error(MPSS_ERR_INVALID, "set_camera: bad resolution");
    memcpy(scene_.camera.raster_to_camera, r2c, sizeof(float) * 16);
    memcpy(scene_.camera.camera_to_world, c2w, sizeof(float) * 16);
    scene_.camera.xres = xres;
    scene_.camera.yres = yres;
    scene_dirty_ = true;
}

void Context::upload_scene() {
    activate();
    quiesce_locked();  // the scene buffers in-flight renders read are about to be replaced
    if (scene_.meshes.empty()) throw Error(MPSS_ERR_INVALID, "scene has no meshes");
    build_bvh(scene_);
    const int depth = bvh_depth(scene_.bvh, 0);
    if (depth > 47) throw Error(MPSS_ERR_INTERNAL, "BVH deeper than the 48-entry traversal stack");
    d_bvh_.upload(scene_.bvh.data(), scene_.bvh.size());
    {
        // the threaded copy for stackless any-hit walks: the nodes are in pre-order (a node's subtree
        // is [i, end_i)), so an interior node's offset becomes end_i -- where a walk continues after
        // missing it; a leaf's end is i + 1
        std::vector<BvhNode> th = scene_.bvh;
        std::vector<int32_t> end(th.size());
        for (size_t i = th.size(); i-- > 0;)
            end[i] = th[i].nprims > 0 ? (int32_t)i + 1 : end[th[i].offset];
        for (size_t i = 0; i < th.size(); ++i)
            if (th[i].nprims == 0) th[i].offset = end[i];
        d_bvh_thread_.upload(th.data(), th.size());
    }
    d_tris_.upload(scene_.tris.data(), scene_.tris.size());
    if (cfg_.sampler == MPSS_SAMPLER_REFERENCE && scene_.camera.xres > 0) {
        CameraBins b;
        build_camera_bins(scene_, b);
        d_bin_off_.upload(b.off.data(), b.off.size());
        d_bin_tri_.upload(b.tri.data(), b.tri.size());
        d_bin_all_.upload(b.all.data(), b.all.size());
        bin_w_ = b.w;
        bin_nall_ = (int)b.all.size();
    }
    d_tri_mesh_.upload(scene_.tri_mesh.data(), scene_.tri_mesh.size());
    d_tri_local_.upload(scene_.tri_local.data(), scene_.tri_local.size());
    d_mesh_bufs_.clear();
    std::vector<RenderMesh> rm;
    for (const Mesh &m : scene_.meshes) {
        auto add = [&](const std::vector<float> &v) -> const float * {
            if (v.empty()) return nullptr;
            d_mesh_bufs_.emplace_back(new DevBuf<float>());
            d_mesh_bufs_.back()->upload(v.data(), v.size());
            return d_mesh_bufs_.back()->ptr;
        };
        RenderMesh r{};
        r.view.P = add(m.P);
        r.view.N = add(m.N);
        r.view.S = add(m.S);
        r.view.uv = add(m.uv);
        std::vector<float> idxf(m.idx.size());
        memcpy(idxf.data(), m.idx.data(), sizeof(int32_t) * m.idx.size());
        r.view.idx = reinterpret_cast<const int32_t *>(add(idxf));
        memcpy(r.view.o2w_store, m.o2w, sizeof(m.o2w));
        memcpy(r.view.w2o_store, m.w2o, sizeof(m.w2o));
        r.view.flip = (int)(m.reverse_orientation ^ m.swaps_handedness);
        r.material = m.material;
        rm.push_back(r);
    }
    // matrices live inside the device-side RenderMesh records; fix up their pointers there
    d_meshes_.alloc(rm.size());
    for (size_t i = 0; i < rm.size(); ++i) {
        rm[i].view.o2w = reinterpret_cast<float *>(reinterpret_cast<char *>(d_meshes_.ptr + i) +
                                                   offsetof(RenderMesh, view) + offsetof(MeshView, o2w_store));
        rm[i].view.w2o = reinterpret_cast<float *>(reinterpret_cast<char *>(d_meshes_.ptr + i) +
                                                   offsetof(RenderMesh, view) + offsetof(MeshView, w2o_store));
    }
    d_meshes_.upload(rm.data(), rm.size());
    std::vector<RenderLight> rl;
    int replay_off = kReplayImage;
    d_envmaps_.clear();
    // every light's map pointers address valid memory (a 1x1 zero map for area lights), so no
    // load the compiler hoists out of a kind test can fault
    if (!d_zero_map_.ptr) {
        const float z[16] = {};
        d_zero_map_.upload(z, 16);
    }
    for (const SceneLight &l : scene_.lights) {
        RenderLight r{};
        r.s.c = V3{l.center[0], l.center[1], l.center[2]};
        r.s.r = l.radius;
        r.s.phi_max = (kPiF / 180.f) * 360.f;   // Radians(Clamp(360, 0, 360))
        r.s.theta_min = m_acos(-1.f);           // acosf(Clamp(zmin/radius))
        r.s.theta_max = m_acos(1.f);
        r.s.area = r.s.phi_max * l.radius * (l.radius - -l.radius);  // Sphere::Area
        memcpy(r.Lemit, l.Lemit, sizeof(r.Lemit));
        r.kind = l.kind;
        r.tw = r.th = r.nu = r.nv = 1;
        r.tex = r.func = r.cdf = r.rint = r.mcdf = d_zero_map_.ptr;
        if (l.kind == 1) {  // radiance MIPMap level 0 + Distribution2D, one device block per light
            memcpy(r.l2w, l.l2w, sizeof(r.l2w));
            memcpy(r.w2l, l.w2l, sizeof(r.w2l));
            const EnvMap em = build_envmap(l.map_w, l.map_h, l.map.data());
            std::vector<float> blk;
            const size_t o_tex = blk.size();
            blk.insert(blk.end(), em.tex.begin(), em.tex.end());
            const size_t o_func = blk.size();
            blk.insert(blk.end(), em.func.begin(), em.func.end());
            const size_t o_cdf = blk.size();
            blk.insert(blk.end(), em.cdf.begin(), em.cdf.end());
            const size_t o_rint = blk.size();
            blk.insert(blk.end(), em.row_int.begin(), em.row_int.end());
            const size_t o_mcdf = blk.size();
            blk.insert(blk.end(), em.mcdf.begin(), em.mcdf.end());
            d_envmaps_.emplace_back(new DevBuf<float>());
            DevBuf<float> &db = *d_envmaps_.back();
            db.upload(blk.data(), blk.size());
            r.tw = em.w0;
            r.th = em.h0;
            r.nu = em.nu;
            r.nv = em.nv;
            r.tex = db.ptr + o_tex;
            r.func = db.ptr + o_func;
            r.cdf = db.ptr + o_cdf;
            r.rint = db.ptr + o_rint;
            r.mcdf = db.ptr + o_mcdf;
            r.mint = em.mint;
            r.s.r = 0.f;
        }
        r.nsamples_pow2 = round_up_pow2(l.nsamples);
        r.nsamples_round = round_up_pow2(l.nsamples);
        r.replay_off = replay_off;
        replay_off += kReplayPerLightSample * r.nsamples_round;
        rl.push_back(r);
    }
    d_lights_.upload(rl.data(), rl.size());
    replay_k_ = replay_off;
    ++scene_gen_;  // the workspaces' replay cursors belong to the old scene
    std::vector<RenderMaterial> rmat;
    if (!d_lut_.ptr) d_lut_.upload(ewa_weight_lut(), kEwaLut);
    for (auto &t : textures_)
        if (!t->dev.ptr) t->dev.upload(t->py.data.data(), t->py.data.size());
    for (const auto &mp : materials_) {
        const Material &m = *mp;
        RenderMaterial r{};
        memcpy(r.R, m.Kr, sizeof(r.R));
        bool black = true;
        for (int c = 0; c < NB; ++c) black = black && m.Kr[c] == 0.f;
        r.has_refl = !black;
        r.r_lo = INFINITY;
        r.r_hi = 0.f;
        r.r_nonneg = 1;
        for (int c = 0; c < NB; ++c) {
            if (!(m.Kr[c] >= 0.f)) r.r_nonneg = 0;
            if (m.Kr[c] > 0.f) r.r_lo = std::min(r.r_lo, m.Kr[c]);
            r.r_hi = std::max(r.r_hi, m.Kr[c]);
        }
        if (black) r.r_lo = 0.f;
        memcpy(r.T, m.Kt, sizeof(r.T));
        bool tblack = true;
        for (int c = 0; c < NB; ++c) tblack = tblack && m.Kt[c] == 0.f;
        r.has_trans = !tblack;
        for (int c = 0; c < NB; ++c) {
            r.alb_mix[c] = m_pow(m.albedo[c], cfg_.mix);
            r.alb_1mmix[c] = m_pow(m.albedo[c], 1.f - cfg_.mix);
        }
        const float rough = m.roughness < 1e-3f ? 1e-3f : m.roughness;
        r.mf.rms2 = rough * rough;
        r.mf.rcp_rms2 = 1 / r.mf.rms2;
        r.mf.eta = m.ior;
        r.mf.fixed_fresnel = m.double_ref_sslf ? 1 : 0;
        r.rho = m.dev_rho.ptr;
        r.n_rho = (int)m.rho.hd.size();
        r.has_bssrdf = m.no_bssrdf ? 0 : 1;
        r.is_mc = m.is_monte_carlo ? 1 : 0;
        r.mix = cfg_.mix;
        for (int c = 0; c < NB; ++c) r.band_pos[c] = m.dev_profile.groups.pos[c];
        if (m.albedo_tex >= 0) {
            r.has_alb_tex = 1;
            r.alb_tex = textures_[m.albedo_tex]->device_view(d_lut_.ptr);
        }
        if (m.bump_tex >= 0) {
            r.has_bump = 1;
            r.bump_tex = textures_[m.bump_tex]->device_view(d_lut_.ptr);
        }
        rmat.push_back(r);
    }
    d_materials_.upload(rmat.data(), rmat.size());
    scene_dirty_ = false;
}

RenderScene Context::render_scene() const {
    RenderScene sc{};
    sc.bvh = d_bvh_.ptr;
    sc.bvh_thread = d_bvh_thread_.ptr;
    sc.nbvh = (int)scene_.bvh.size();
    sc.tris = d_tris_.ptr;
    sc.tri_mesh = d_tri_mesh_.ptr;
    sc.tri_local = d_tri_local_.ptr;
    sc.meshes = d_meshes_.ptr;
    sc.lights = d_lights_.ptr;
    sc.materials = d_materials_.ptr;
    sc.nlights = (int)scene_.lights.size();
    for (const SceneLight &l : scene_.lights) sc.n_infinite += l.kind == 1;
    sc.nmaterials = (int)materials_.size();
    sc.xres = scene_.camera.xres;
    sc.yres = scene_.camera.yres;
    memcpy(sc.raster_to_camera, scene_.camera.raster_to_camera, sizeof(sc.raster_to_camera));
    memcpy(sc.camera_to_world, scene_.camera.camera_to_world, sizeof(sc.camera_to_world));
    // dxCamera = RasterToCamera(Point(1,0,0)) - RasterToCamera(Point(0,0,0)) (perspective.cpp:47-48)
    const V3 c0 = xform_point(sc.raster_to_camera, V3{0.f, 0.f, 0.f});
    const V3 dx = xform_point(sc.raster_to_camera, V3{1.f, 0.f, 0.f}) - c0;
    const V3 dy = xform_point(sc.raster_to_camera, V3{0.f, 1.f, 0.f}) - c0;
    sc.dx_camera[0] = dx.x;
    sc.dx_camera[1] = dx.y;
    sc.dx_camera[2] = dx.z;
    sc.dy_camera[0] = dy.x;
    sc.dy_camera[1] = dy.y;
    sc.dy_camera[2] = dy.z;
    for (const auto &m : materials_) sc.any_tex |= (m->albedo_tex >= 0 || m->bump_tex >= 0);
    return sc;
}

void Context::set_surface_points(uint32_t n, const SurfacePoint *pts) {
    std::lock_guard<std::mutex> g(mu_);
    points_.assign(pts, pts + n);
    have_points_ = n > 0;
}

// TessellateSurfacePointsRenderer's point set on the GPU (tess_kernel): per mesh a counting pass,
// a prefix sum of the per-triangle counts on the host (one int64 per triangle), then the emitting
// pass; the points come back to points_ (mpss_get_surface_points / the pointsfile read them there).
void Context::tessellate_on_gpu() {
    const RenderScene sc = render_scene();
    std::vector<int64_t> base(scene_.meshes.size() + 1, 0);
    for (size_t m = 0; m < scene_.meshes.size(); ++m)
        base[m + 1] = base[m] + (int64_t)(scene_.meshes[m].idx.size() / 3);
    const int64_t ntri = base.back();
    points_.clear();
    if (ntri == 0) return;
    DevBuf<int64_t> cnt, off;
    cnt.alloc((size_t)ntri);
    off.alloc((size_t)ntri);
    for (size_t m = 0; m < scene_.meshes.size(); ++m) {
        const int nt = (int)(base[m + 1] - base[m]);
        if (nt > 0)
            hipLaunchKernelGGL((tess_kernel<false, false>), dim3((unsigned)((nt + 63) / 64)), dim3(64), 0, 0, sc,
                               (int)m, nt, base[m], min_dist_, cnt.ptr, (const int64_t *)nullptr,
                               (SurfacePoint *)nullptr);
    }
    MPSS_HIP(hipGetLastError());
    std::vector<int64_t> h((size_t)ntri);
    MPSS_HIP(hipMemcpy(h.data(), cnt.ptr, sizeof(int64_t) * (size_t)ntri, hipMemcpyDeviceToHost));
    int64_t total = 0;
    for (int64_t i = 0; i < ntri; ++i) {
        const int64_t c = h[(size_t)i];
        h[(size_t)i] = total;
        total += c;
    }
    if (total > ((int64_t)1 << 30)) throw Error(MPSS_ERR_INVALID, "tessellation: more than 2^30 surface points");
    if (total == 0) return;
    MPSS_HIP(hipMemcpy(off.ptr, h.data(), sizeof(int64_t) * (size_t)ntri, hipMemcpyHostToDevice));
    DevBuf<SurfacePoint> pts;
    pts.alloc((size_t)total);
    for (size_t m = 0; m < scene_.meshes.size(); ++m) {
        const int nt = (int)(base[m + 1] - base[m]);
        if (nt > 0) {
            void (*emit)(RenderScene, int, int, int64_t, float, int64_t *, const int64_t *, SurfacePoint *) =
                cfg_.incenter ? tess_kernel<true, true> : tess_kernel<true, false>;
            hipLaunchKernelGGL(emit, dim3((unsigned)((nt + 63) / 64)), dim3(64), 0, 0, sc, (int)m, nt, base[m],
                               min_dist_, cnt.ptr, (const int64_t *)off.ptr, pts.ptr);
        }
    }
    MPSS_HIP(hipGetLastError());
    points_.resize((size_t)total);
    MPSS_HIP(hipMemcpy(points_.data(), pts.ptr, sizeof(SurfacePoint) * (size_t)total, hipMemcpyDeviceToHost));
}

// MultipoleSubsurfaceIntegrator::Preprocess (multipolesubsurface.cpp:170-238)
void Context::preprocess(uint32_t seed) {
    activate();
    std::lock_guard<std::mutex> g(mu_);
    quiesce_locked();  // no render of the previous octree may still be in flight or running
    if (scene_dirty_) upload_scene();
    if (scene_.lights.empty()) {  // "if (scene->lights.size() == 0) return;" -> no octree, no SSS
        have_octree_ = false;
        irradiance_.clear();
        return;
    }
    if (!have_points_) {
        if (cfg_.use_poisson_point_finder)
            find_poisson_points(seed);
        else if (cfg_.tessellate_on_host)
            tessellate_surface_points(scene_, min_dist_, cfg_.incenter != 0, points_, 0, host_bump_views().data());
        else
            tessellate_on_gpu();
    }
    const int n = (int)points_.size();
    if (n == 0) {
        // the reference goes on with an empty point set: its octree holds nothing, so Mo() is 0
        // and the frame has direct lighting only (surfacepoints.cpp:277-281, Preprocess :192-236)
        fprintf(stderr, "mpss: Warning: no surface points with BSSRDFs were found; rendering without "
                        "subsurface scattering\n");
        have_octree_ = false;
        irradiance_.clear();
        return;
    }
    std::vector<float> p(3 * (size_t)n), nr(3 * (size_t)n), eps(n);
    std::vector<uint32_t> mat(n);
    std::vector<float> uv(2 * (size_t)n);
    for (int i = 0; i < n; ++i) {
        uv[2 * (size_t)i] = points_[i].u;
        uv[2 * (size_t)i + 1] = points_[i].v;
        for (int k = 0; k < 3; ++k) {
            p[3 * (size_t)i + k] = points_[i].p[k];
            nr[3 * (size_t)i + k] = points_[i].n[k];
        }
        eps[i] = points_[i].ray_eps;
        mat[i] = points_[i].material;
    }
    DevBuf<float> dp, dn, de, dE, duv;
    DevBuf<uint32_t> dm;
    duv.upload(uv.data(), uv.size());
    dp.upload(p.data(), p.size());
    dn.upload(nr.data(), nr.size());
    de.upload(eps.data(), eps.size());
    dm.upload(mat.data(), mat.size());
    dE.alloc((size_t)n * NB);
    const RenderScene sc = render_scene();
    if (cfg_.show_irradiance_points) {  // IrradianceTask: red points instead of irradiance
        const float red[3] = {1.f, 0.f, 0.f};
        float s[NB];
        spectrum_from_rgb(red, false, s);
        irradiance_.resize((size_t)n * NB);
        for (int i = 0; i < n; ++i) memcpy(&irradiance_[(size_t)i * NB], s, sizeof(s));
    } else {
        RenderScene sci = sc;
        DevBuf<uint32_t> scr, mt;
        if (cfg_.sampler == MPSS_SAMPLER_REFERENCE && !scene_.lights.empty()) {  // IrradianceTask streams
            const int T = replay_irradiance_tasks(n, std::max(1, cfg_.replay_cores));
            scr.alloc((size_t)n * scene_.lights.size() * 2);
            mt.alloc((size_t)624 * T);
            hipLaunchKernelGGL(replay_irradiance_kernel, dim3((T + 63) / 64), dim3(64), 0, 0, n,
                               (int)scene_.lights.size(), T, mt.ptr, scr.ptr);
            MPSS_HIP(hipGetLastError());
            sci.irr_scr = scr.ptr;
        }
        hipEvent_t ev{};
        time_begin(cfg_.kernel_timing != 0, 0, ev);
        hipLaunchKernelGGL(irradiance_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, sci, dp.ptr, dn.ptr, de.ptr,
                           dm.ptr, duv.ptr, n, seed, dE.ptr);
        MPSS_HIP(hipGetLastError());
        time_end(cfg_.kernel_timing != 0, 0, ev, 0, timed_);
        irradiance_.resize((size_t)n * NB);
        MPSS_HIP(hipMemcpy(irradiance_.data(), dE.ptr, sizeof(float) * irradiance_.size(), hipMemcpyDeviceToHost));
    }
    std::vector<float> area(n);
    for (int i = 0; i < n; ++i) area[i] = points_[i].area;
    const bool e_on_device = !cfg_.show_irradiance_points;  // dE holds the irradiance kernel's output
    build_octree_locked(n, p.data(), nr.data(), irradiance_.data(), area.data(), dp.ptr, dn.ptr,
                        e_on_device ? dE.ptr : nullptr);
}

// FindPoissonPointDistribution -> SurfacePointsRenderer::Render (renderers/surfacepoints.cpp:115-150)
// with ONE SurfacePointTask (:175-284; the reference runs one per core and its result depends on
// their interleaving): batches of 20000 paths from pCamera are traced on the GPU, 16 batches per
// launch; on the host each batch's candidates are taken in path order and accepted unless an
// accepted point lies within minDist (PoissonCheck: DistanceSquared < minDist^2; the reference's
// octree lookup finds exactly those), until maxFails candidates in a row fail.
void Context::find_poisson_points(uint32_t seed) {
    if (scene_dirty_) upload_scene();
    activate();
    // scene->WorldBound(): every triangle and every area-light sphere
    float lo[3], hi[3];
    for (int k = 0; k < 3; ++k) {
        lo[k] = scene_.bvh[0].bmin[k];
        hi[k] = scene_.bvh[0].bmax[k];
    }
    for (const SceneLight &l : scene_.lights) {
        if (l.kind != 0) continue;
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], l.center[k] + -l.radius);
            hi[k] = std::max(hi[k], l.center[k] + l.radius);
        }
    }
    PoissonWalk w{};
    const V3 c = V3{.5f * lo[0] + .5f * hi[0], .5f * lo[1] + .5f * hi[1], .5f * lo[2] + .5f * hi[2]};
    const bool inside = c.x >= lo[0] && c.x <= hi[0] && c.y >= lo[1] && c.y <= hi[1] && c.z >= lo[2] && c.z <= hi[2];
    const float rad = inside ? length(c - V3{hi[0], hi[1], hi[2]}) : 0.f;  // BBox::BoundingSphere
    w.bound.c = c;
    w.bound.r = rad;
    w.bound.phi_max = (kPiF / 180.f) * 360.f;
    w.bound.theta_min = m_acos(-1.f);
    w.bound.theta_max = m_acos(1.f);
    w.bound.area = w.bound.phi_max * rad * (rad - -rad);
    w.origin = xform_point(scene_.camera.camera_to_world, V3{0.f, 0.f, 0.f});
    w.seed = mix32(seed * 37u + 0x5eed1u);  // RNG rng(37 * taskNum), replay mode
    const int max_fails = cfg_.quick_render ? std::max(10, 2000 / 10) : 2000;
    const float md = min_dist_, md2 = md * md;
    const float area = kPiF * (md / 2.f) * (md / 2.f);
    constexpr int kBatch = 20000, kBatchesPerLaunch = 16;
    DevBuf<SurfacePoint> dcand;
    DevBuf<int> dcount;
    dcand.alloc((size_t)kBatch * kBatchesPerLaunch * kPoissonCand);
    dcount.alloc((size_t)kBatch * kBatchesPerLaunch);
    std::vector<SurfacePoint> cand((size_t)kBatch * kBatchesPerLaunch * kPoissonCand);
    std::vector<int> cnt((size_t)kBatch * kBatchesPerLaunch);
    // accepted points, bucketed by minDist cells
    std::unordered_map<uint64_t, std::vector<uint32_t>> grid;
    auto cell = [&](float x) { return (int64_t)std::floor((double)x / (double)md); };
    auto key = [](int64_t x, int64_t y, int64_t z) {
        return ((uint64_t)(x & 0x1fffff) << 42) | ((uint64_t)(y & 0x1fffff) << 21) | (uint64_t)(z & 0x1fffff);
    };
    points_.clear();
    const RenderScene sc = render_scene();
    int repeated_fails = 0;
    int64_t total_paths = 0;
    bool done = false;
    for (uint32_t launch = 0; !done; ++launch) {
        w.path0 = launch * (uint32_t)(kBatch * kBatchesPerLaunch);
        w.npaths = kBatch * kBatchesPerLaunch;
        hipLaunchKernelGGL(poisson_walk_kernel, dim3((unsigned)((w.npaths + 255) / 256)), dim3(256), 0, 0, sc, w,
                           dcand.ptr, dcount.ptr);
        MPSS_HIP(hipGetLastError());
        MPSS_HIP(hipMemcpy(cnt.data(), dcount.ptr, sizeof(int) * cnt.size(), hipMemcpyDeviceToHost));
        MPSS_HIP(hipMemcpy(cand.data(), dcand.ptr, sizeof(SurfacePoint) * cand.size(), hipMemcpyDeviceToHost));
        for (int b = 0; b < kBatchesPerLaunch && !done; ++b) {
            total_paths += kBatch;
            for (int i = b * kBatch; i < (b + 1) * kBatch && !done; ++i)
                for (int j = 0; j < cnt[i] && !done; ++j) {
                    SurfacePoint sp = cand[(size_t)i * kPoissonCand + j];
                    const int64_t cx = cell(sp.p[0]), cy = cell(sp.p[1]), cz = cell(sp.p[2]);
                    bool fail = false;
                    for (int dz = -1; dz <= 1 && !fail; ++dz)
                        for (int dy = -1; dy <= 1 && !fail; ++dy)
                            for (int dx = -1; dx <= 1 && !fail; ++dx) {
                                auto it = grid.find(key(cx + dx, cy + dy, cz + dz));
                                if (it == grid.end()) continue;
                                for (uint32_t q : it->second) {
                                    const SurfacePoint &o = points_[q];
                                    const float ex = o.p[0] - sp.p[0], ey = o.p[1] - sp.p[1], ez = o.p[2] - sp.p[2];
                                    if (ex * ex + ey * ey + ez * ez < md2) {
                                        fail = true;
                                        break;
                                    }
                                }
                            }
                    if (fail) {
                        if (++repeated_fails >= max_fails) done = true;
                    } else {
                        repeated_fails = 0;
                        sp.area = area;
                        grid[key(cx, cy, cz)].push_back((uint32_t)points_.size());
                        points_.push_back(sp);
                    }
                }
            if (!done && total_paths > 50000 && points_.empty()) {
                // Warning + return, as FindPoissonPointDistribution (surfacepoints.cpp:277-281)
                fprintf(stderr, "mpss: Warning: There don't seem to be any objects with BSSRDFs in this scene. "
                                "Giving up.\n");
                return;
            }
        }
    }
}

// SamplerRenderer::Render restricted to pixel rectangles. Each rectangle is cut into row
// pieces (a piece = the rows plus a one-pixel border of samples that the box filter carries
// in); pieces are packed into batches of <= max_batch_samples camera samples. Per batch:
// camera/direct kernel per piece (all pieces append their surface hits to one compacted
// list) -> ONE sharded Mo() gather per BSSRDF material over the batch's hits -> film kernel per
// piece. Calls on different streams may overlap: each takes its own workspace (RenderWorkspace),
// and the scene, materials and octree are only read after the context lock is released.
// The reference sampler's values over [x0, x1) x [y0, y1) of the sample extent at `spp`
// (replay_gen.hip) into ws->rp_table, continuing the workspace's task streams.
void Context::replay_window(RenderWorkspace *ws, const RenderScene &sc, int spp, int x0, int x1, int y0, int y1,
                            hipStream_t stream, bool all_values) {
    const int W = sc.xres, H = sc.yres;
    const int T = replay_render_tasks(W, H, std::max(1, cfg_.replay_cores));
    const uint64_t key[3] = {scene_gen_, (uint64_t)spp, (uint64_t)T};
    if (ws->pending) MPSS_HIP(hipStreamWaitEvent(stream, ws->done, 0));  // the workspace's previous user
    if (ws->rp_key[0] != key[0] || ws->rp_key[1] != key[1] || ws->rp_key[2] != key[2]) {
        if ((int64_t)ws->rp_pix.n < T) {
            if (ws->pending) MPSS_HIP(hipEventSynchronize(ws->done));
            ws->rp_mt.alloc((size_t)624 * T);
            ws->rp_pix.alloc((size_t)T);
            ws->rp_mti.alloc((size_t)T);
        }
        MPSS_HIP(hipMemsetAsync(ws->rp_pix.ptr, 0xff, sizeof(int) * (size_t)T, stream));  // -1: not seeded
        for (int k = 0; k < 3; ++k) ws->rp_key[k] = key[k];
    }
    const size_t need = (size_t)(x1 - x0) * (y1 - y0) * spp * replay_k_;
    if (ws->rp_table.n < need) {
        if (ws->pending) MPSS_HIP(hipEventSynchronize(ws->done));
        ws->rp_table.alloc(need);
    }
    ReplayWindow w{};
    replay_window_tasks(W, H, T, x0, x1, y0, y1, w);
    w.spp = spp;
    w.K = replay_k_;
    w.li_draws = (cfg_.max_depth > 0 && !cfg_.show_irradiance_points) ? kReplayLiDraws : 0;
    w.nmax = 1;
    w.nlights = (int)scene_.lights.size();
    w.arr_draws = 0;
    for (const SceneLight &l : scene_.lights) {
        const int n = round_up_pow2(l.nsamples);
        w.nmax = std::max(w.nmax, n);
        w.arr_draws += 3 * (spp * n + spp) + 5;
    }
    w.cur = ReplayCursors{ws->rp_mt.ptr, ws->rp_pix.ptr, ws->rp_mti.ptr};
    w.out = ws->rp_table.ptr;
    if (!d_bin_off_.ptr || bin_w_ != W + 1) throw Error(MPSS_ERR_INTERNAL, "replay: no camera-ray bins for this camera");
    w.bin_off = d_bin_off_.ptr;
    w.bin_tri = d_bin_tri_.ptr;
    w.bin_all = d_bin_all_.ptr;
    w.bin_w = bin_w_;
    w.bin_nall = bin_nall_;
    w.all_values = all_values ? 1 : 0;
    launch_replay_window(sc, w, stream);
}

void Context::check_replay_lds(int spp, const char *who) const {
    std::vector<int> ns;
    for (const SceneLight &l : scene_.lights) ns.push_back(l.nsamples);
    replay_check_lds(spp, ns.data(), (int)ns.size(), who);
}

void Context::replay_samples(int spp, float *out, uint64_t *n_floats, int *k) {
    activate();
    std::unique_lock<std::mutex> lk(mu_);
    if (cfg_.sampler != MPSS_SAMPLER_REFERENCE) throw Error(MPSS_ERR_INVALID, "replay_samples: the context uses the hash sampler");
    if (scene_dirty_) upload_scene();
    const int W = scene_.camera.xres, H = scene_.camera.yres;
    if (W <= 0) throw Error(MPSS_ERR_INVALID, "replay_samples: no camera");
    spp = round_up_pow2(spp);
    if (spp > kReplayMaxSpp) throw Error(MPSS_ERR_INVALID, "replay_samples: spp too large for the replay sampler");
    check_replay_lds(spp, "replay_samples");
    const int K = replay_k_;
    *k = K;
    const int64_t npix = (int64_t)(W + 1) * (H + 1);
    *n_floats = (uint64_t)npix * spp * K;
    if (!out) return;
    // the whole sample extent as one window, on a workspace of its own cursors
    RenderWorkspace *ws = acquire_ws();
    ++inflight_;
    RenderScene sc = render_scene();
    lk.unlock();
    InflightGuard guard{this, ws, nullptr};
    replay_window(ws, sc, spp, 0, W + 1, 0, H + 1, nullptr, true);
    std::vector<float> col((size_t)npix * spp * K);
    MPSS_HIP(hipMemcpy(col.data(), ws->rp_table.ptr, sizeof(float) * col.size(), hipMemcpyDeviceToHost));
    ws->rp_key[0] = ~0ull;  // (its cursors now sit at the end of every stream)
    guard.release();
    // column-major window -> the documented layout [((y (W + 1) + x) spp + s) K + k]
    for (int64_t p = 0; p < npix; ++p)
        for (int s2 = 0; s2 < spp; ++s2)
            for (int c = 0; c < K; ++c) out[(p * spp + s2) * K + c] = col[((size_t)c * npix + p) * spp + s2];
}

void Context::render_tiles(int spp, uint32_t seed, int n, const int32_t *rects, float *const *outs,
                           hipStream_t stream) {
    activate();
    std::unique_lock<std::mutex> lk(mu_);
    if (scene_dirty_) upload_scene();
    const int W = scene_.camera.xres, H = scene_.camera.yres;
    if (W <= 0) throw Error(MPSS_ERR_INVALID, "render_tile: no camera");
    if (spp < 1 || spp > 65535) throw Error(MPSS_ERR_INVALID, "render_tile: spp must be in [1, 65535]");
    const bool replay = cfg_.sampler == MPSS_SAMPLER_REFERENCE;
    if (replay) {
        spp = round_up_pow2(spp);  // LDSampler rounds pixelsamples up (lowdiscrepancy.cpp:45-49)
        if (spp > kReplayMaxSpp)
            throw Error(MPSS_ERR_INVALID, "render_tile: spp must be at most 4096 for the replay sampler");
        check_replay_lds(spp, "render_tile");
    }
    for (int i = 0; i < n; ++i) {
        const int32_t *r = rects + 4 * i;
        if (r[0] < 0 || r[2] < 0 || r[1] > W || r[3] > H || r[0] >= r[1] || r[2] >= r[3])
            throw Error(MPSS_ERR_INVALID, "render_tile: bad rectangle");
        if (!outs[i]) throw Error(MPSS_ERR_INVALID, "render_tile: null output");
    }
    // every LayeredSkin material has a MultipoleBSSRDF (GetMultipoleBSSRDF, layeredskin.cpp:180-185):
    // each evaluates Mo() with its own profile (multipolesubsurface.cpp:267-280)
    struct SssMat {
        int id;
        const Material *m;
        const BandLayout *layout;
    };
    std::vector<SssMat> sss;
    if (have_octree_)
        for (size_t i = 0; i < materials_.size(); ++i)
            if (!materials_[i]->dipole && !materials_[i]->no_bssrdf)
                sss.push_back(SssMat{(int)i, materials_[i].get(),
                                     &dev_octree_.ensure_layout(materials_[i]->dev_profile.groups)});
    RenderScene sc = render_scene();
    sc.have_octree = sss.empty() ? 0 : 1;
    if (replay) {  // (the window and its table: per batch, below)
        sc.replay_k = replay_k_;
        sc.replay_spp = spp;
    }
    const bool timing = cfg_.kernel_timing != 0, counting = cfg_.count_traversal != 0;
    if (counting && !d_counts_.ptr) {
        d_counts_.alloc(kStatStride * kGroups);
        MPSS_HIP(hipMemset(d_counts_.ptr, 0, kStatStride * kGroups * sizeof(unsigned long long)));
    }
    unsigned long long *const counts = counting ? d_counts_.ptr : nullptr;
    const int64_t max_batch = std::max<int64_t>(cfg_.max_batch_samples, 1 << 10);
    const int nlights = (int)scene_.lights.size();
    int ns_max = 1;
    for (const SceneLight &l : scene_.lights) ns_max = std::max(ns_max, round_up_pow2(l.nsamples));
    const float max_error = max_error_;
    const GatherOpts gopts = gather_opts();
    RenderWorkspace *ws = acquire_ws();
    ++inflight_;  // until this call's kernels are queued (see quiesce_locked)
    lk.unlock();
    InflightGuard guard{this, ws, stream};  // every way out: workspace back to the pool, inflight_ down

    std::vector<Timed> timed;
    int64_t n_samples = 0, n_sss = 0;
    {
        if (ws->pending) MPSS_HIP(hipStreamWaitEvent(stream, ws->done, 0));
        // a workspace buffer is reallocated only once its previous user's kernels are done
        auto grow = [&](auto &buf, int64_t &have, int64_t want, size_t per) {
            if (have >= want) return;
            if (ws->pending) MPSS_HIP(hipEventSynchronize(ws->done));
            buf.alloc((size_t)want * per);
            have = want;
        };
        // cut rectangles into pieces of <= max_batch samples
        struct Piece {
            TileBatch tb;
            float *out;
        };
        std::vector<Piece> pieces;
        // replay: rectangles in row order, so that consecutive batches continue the task streams
        // (replay_window) and a batch's window stays compact
        std::vector<int> order(n);
        for (int i = 0; i < n; ++i) order[i] = i;
        if (replay)
            std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
                return rects[4 * a + 2] != rects[4 * b + 2] ? rects[4 * a + 2] < rects[4 * b + 2]
                                                            : rects[4 * a] < rects[4 * b];
            });
        for (int i : order) {
            const int x0 = rects[4 * i], x1 = rects[4 * i + 1], y0 = rects[4 * i + 2], y1 = rects[4 * i + 3];
            const int tw = x1 - x0;
            const int ex0 = std::max(x0 - 1, 0);
            const int ew = std::min(x1 + 1, W) - ex0;
            const int rows = (int)std::max<int64_t>(1, max_batch / ((int64_t)ew * spp) - 2);
            for (int yb = y0; yb < y1; yb += rows) {
                const int ye = std::min(y1, yb + rows);
                Piece p;
                p.tb.x0 = x0;
                p.tb.x1 = x1;
                p.tb.y0 = yb;
                p.tb.y1 = ye;
                p.tb.ex0 = ex0;
                p.tb.ey0 = std::max(yb - 1, 0);
                p.tb.ew = ew;
                p.tb.eh = std::min(ye + 1, H) - p.tb.ey0;
                p.tb.spp = spp;
                p.tb.seed = seed;
                p.tb.nsamples = (int64_t)p.tb.ew * p.tb.eh * spp;
                p.out = outs[i] + (size_t)(yb - y0) * tw * 4;
                pieces.push_back(p);
            }
        }
        size_t pi = 0;
        // replay: the current generated window (it may span several batches: one generation over
        // more tasks keeps more waves in flight, replay_gen.hip)
        bool have_win = false;
        int wx0 = 0, wx1 = 0, wy0 = 0, wy1 = 0;
        while (pi < pieces.size()) {
            // pack pieces into one batch
            size_t pe = pi;
            int64_t total = 0;
            // replay: the batch's window (the pieces' bounding box) holds spp x replay_k_ floats per
            // pixel; kept to <= kReplayWindowFloats
            int bx0 = INT32_MAX, bx1 = 0, by0 = INT32_MAX, by1 = 0;
            auto fits = [&](const TileBatch &tb) {
                if (!replay) return true;
                const int64_t w = std::max(bx1, tb.ex0 + tb.ew) - std::min(bx0, tb.ex0);
                const int64_t h = std::max(by1, tb.ey0 + tb.eh) - std::min(by0, tb.ey0);
                return w * h * spp * replay_k_ <= kReplayWindowFloats;
            };
            while (pe < pieces.size() &&
                   (pe == pi || (total + pieces[pe].tb.nsamples <= max_batch && fits(pieces[pe].tb)))) {
                const TileBatch &tb = pieces[pe].tb;
                bx0 = std::min(bx0, tb.ex0);
                bx1 = std::max(bx1, tb.ex0 + tb.ew);
                by0 = std::min(by0, tb.ey0);
                by1 = std::max(by1, tb.ey0 + tb.eh);
                total += pieces[pe++].tb.nsamples;
            }
            // per-sample buffers: the batch's camera samples (primary_kernel may give each a hit slot)
            if (ws->n < total) {
                int64_t have = ws->n;
                grow(ws->flags, have, total, 1);
                have = ws->n;
                grow(ws->slot, have, total, 1);
                ws->n = total;
            }
            if (ws->rec_n < total) {
                for (auto *b : {&ws->ha, &ws->hb}) {
                    int64_t have = ws->rec_n;
                    grow(*b, have, total, 1);
                }
                int64_t have = ws->rec_n;
                grow(ws->hs, have, total, 1);
                ws->rec_n = total;
            }
            if (ws->px < total / spp) {
                int64_t have = ws->px;
                grow(ws->spill, have, total / spp, 1);
                ws->px = total / spp;
            }
            MPSS_HIP(hipMemsetAsync(ws->count.ptr, 0, sizeof(int), stream));
            MPSS_HIP(hipMemsetAsync(ws->spill.ptr, 0, sizeof(uint32_t) * (size_t)(total / spp), stream));
            auto recs = [&](int64_t off) {  // (the per-hit pointers are read after the hit-count resize)
                return SampleRecs{ws->flags.ptr + off, ws->spill.ptr + off / spp, ws->slot.ptr + off, ws->ld.ptr,
                                  ws->ha.ptr, ws->hb.ptr, ws->hs.ptr, ws->q.ptr, ws->count.ptr, ws->mo.ptr,
                                  ws->xyz.ptr, ws->alb.ptr, ws->frame.ptr};
            };
            // the batch's pieces, kMaxPieces per launch; blocks per piece: samples (primary) or
            // tile pixels (film) / 256
            auto launch_pieces = [&](bool film) {
                int64_t off = 0;
                for (size_t k0 = pi; k0 < pe; k0 += kMaxPieces) {
                    PieceList pl{};
                    int blocks = 0;
                    for (size_t k = k0; k < pe && k < k0 + kMaxPieces; ++k) {
                        const TileBatch &tb = pieces[k].tb;
                        const int j = pl.n++;
                        const int tw = tb.x1 - tb.x0;
                        const int64_t items = film ? (int64_t)tw * (tb.y1 - tb.y0) : tb.nsamples;
                        pl.block0[j] = blocks;
                        pl.tb[j] = tb;
                        pl.off[j] = off;
                        pl.out[j] = pieces[k].out;
                        pl.out_stride[j] = tw;
                        blocks += (int)((items + 255) / 256);
                        off += tb.nsamples;
                    }
                    pl.block0[pl.n] = blocks;
                    if (film)
                        hipLaunchKernelGGL(film_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, sc, pl, recs(0));
                    else
                        hipLaunchKernelGGL(primary_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, sc, pl,
                                           recs(0));
                }
            };
            hipEvent_t ev{};
            if (replay && (!have_win || bx0 < wx0 || bx1 > wx1 || by0 < wy0 || by1 > wy1)) {
                // the reference sampler's values over a new window: this batch's pieces and the
                // following ones, as far as the window table allows (kReplayWindowFloats)
                int gx0 = bx0, gx1 = bx1, gy0 = by0, gy1 = by1;
                for (size_t k = pe; k < pieces.size(); ++k) {
                    const TileBatch &tb = pieces[k].tb;
                    const int nx0 = std::min(gx0, tb.ex0), nx1 = std::max(gx1, tb.ex0 + tb.ew);
                    const int ny0 = std::min(gy0, tb.ey0), ny1 = std::max(gy1, tb.ey0 + tb.eh);
                    if ((int64_t)(nx1 - nx0) * (ny1 - ny0) * spp * replay_k_ > kReplayWindowFloats) break;
                    gx0 = nx0;
                    gx1 = nx1;
                    gy0 = ny0;
                    gy1 = ny1;
                }
                time_begin(timing, stream, ev);
                replay_window(ws, sc, spp, gx0, gx1, gy0, gy1, stream);
                time_end(timing, stream, ev, 6, timed);
                have_win = true;
                wx0 = gx0;
                wx1 = gx1;
                wy0 = gy0;
                wy1 = gy1;
                sc.replay = ws->rp_table.ptr;
                sc.replay_x0 = wx0;
                sc.replay_y0 = wy0;
                sc.replay_w = wx1 - wx0;
                sc.replay_npix = (int64_t)(wx1 - wx0) * (wy1 - wy0);
            }
            time_begin(timing, stream, ev);
            launch_pieces(false);
            time_end(timing, stream, ev, 1, timed);
            // the batch's hit count sizes everything after the compaction: one read-back per batch
            // (the stream only waits for primary_kernel; the GPU idles for the round trip alone)
            int nh_dev = 0;
            MPSS_HIP(hipMemcpyAsync(&nh_dev, ws->count.ptr, sizeof(int), hipMemcpyDeviceToHost, stream));
            MPSS_HIP(hipStreamSynchronize(stream));
            const int64_t nh = std::max<int64_t>(1, nh_dev);
            if (ws->hits < nh) {
                for (auto *b : {&ws->q, &ws->xyz}) {
                    int64_t have = ws->hits;
                    grow(*b, have, nh, 1);
                }
                int64_t have = ws->hits;
                grow(ws->mo, have, nh, kGroups);
                have = ws->hits;
                grow(ws->ld, have, nh, ROW);
                ws->hits = nh;
            }
            grow(ws->perm, ws->perm_n, (nh + 1023) / 1024 * 1024, 1);
            if (sc.any_tex && ws->tex_hits < nh) {
                int64_t have = ws->tex_hits;
                grow(ws->alb, have, nh, 1);
                have = ws->tex_hits;
                grow(ws->frame, have, nh, 2);
                ws->tex_hits = nh;
            }
            {
                const SampleRecs rec = recs(0);
                const int64_t lanes = nh * std::max<int64_t>(1, (int64_t)nlights) * ns_max;
                if (lanes > (int64_t)INT32_MAX)
                    throw Error(MPSS_ERR_INVALID, "render_tile: too many light samples per batch; lower "
                                                  "max_batch_samples");
                grow(ws->terms, ws->terms_n, lanes, 64);
                DirectTerms *terms = reinterpret_cast<DirectTerms *>(ws->terms.ptr);
                float4 *inf_st = nullptr;
                if (sc.n_infinite > 0) {
                    grow(ws->st, ws->st_n, lanes, 1);
                    inf_st = ws->st.ptr;
                }
                if (sc.any_tex) {
                    time_begin(timing, stream, ev);
                    hipLaunchKernelGGL(shade_tex_kernel, dim3((unsigned)((nh + 255) / 256)), dim3(256), 0, stream, sc,
                                       rec, spp, seed, (int)nh);
                    time_end(timing, stream, ev, 5, timed);
                }
                time_begin(timing, stream, ev);
                if (nlights > 0) {
                    hipLaunchKernelGGL(shade_direct_kernel, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0,
                                       stream, sc, rec, spp, seed, (int)nh, ns_max, terms, inf_st);
                    if (sc.n_infinite > 0)
                        hipLaunchKernelGGL(direct_combine_kernel<true>, dim3((unsigned)((nh + 255) / 256)), dim3(256),
                                           0, stream, sc, rec, (int)nh, ns_max, (const DirectTerms *)terms,
                                           (const float4 *)inf_st);
                    else
                        hipLaunchKernelGGL(direct_combine_kernel<false>, dim3((unsigned)((nh + 255) / 256)), dim3(256),
                                           0, stream, sc, rec, (int)nh, ns_max, (const DirectTerms *)terms,
                                           (const float4 *)nullptr);
                } else {
                    hipLaunchKernelGGL(shade_nolight_kernel, dim3((unsigned)((nh + 255) / 256)), dim3(256), 0, stream,
                                       sc, rec, (int)nh);
                }
                time_end(timing, stream, ev, 4, timed);
            }
            if (!sss.empty()) {
                time_begin(timing, stream, ev);
                for (const SssMat &s : sss)  // (an rgbprofile material: FromRGB of its R, G, B lookups)
                    launch_mo_band(dev_octree_, *s.layout, s.m->dev_profile, max_error, (int)nh, ws->q.ptr,
                                   ws->count.ptr, ws->mo.ptr, sss.size() > 1 ? ws->hs.ptr : nullptr, s.id, counts,
                                   ws->work.ptr, ws->perm.ptr, gopts, stream);
                time_end(timing, stream, ev, 2, timed);
            }
            time_begin(timing, stream, ev);
            {
                const SampleRecs rec = recs(0);
                hipLaunchKernelGGL(assemble_kernel, dim3((unsigned)((nh + 255) / 256)), dim3(256), 0, stream, sc, rec,
                                   (int)nh);
                if (sc.n_infinite > 0)
                    hipLaunchKernelGGL(sky_kernel, dim3((unsigned)((nh + 255) / 256)), dim3(256), 0, stream, sc, rec,
                                       (int)nh);
            }
            launch_pieces(true);
            time_end(timing, stream, ev, 3, timed);
            MPSS_HIP(hipGetLastError());
            n_samples += total;
            if (counting) n_sss += nh_dev;
            pi = pe;
        }
    }
    guard.release();
    std::lock_guard<std::mutex> g(mu_);  // (released before the guard's end_inflight takes mu_)
    timed_.insert(timed_.end(), timed.begin(), timed.end());
    stats_.samples += n_samples;
    stats_.sss_samples += n_sss;
}

// Tile-cost probe (mpss_tile_costs): classes per pixel centre, summed per rectangle on the host.
void Context::tile_costs(int n, const int32_t *rects, int64_t *sss, int64_t *surf) {
    activate();
    std::lock_guard<std::mutex> g(mu_);
    if (scene_dirty_) upload_scene();
    const int W = scene_.camera.xres, H = scene_.camera.yres;
    if (W <= 0) throw Error(MPSS_ERR_INVALID, "tile_costs: no camera");
    RenderScene sc = render_scene();
    sc.have_octree = have_octree_ ? 1 : 0;
    DevBuf<uint8_t> cls;
    cls.alloc((size_t)W * H);
    hipLaunchKernelGGL(probe_kernel, dim3((unsigned)(((int64_t)W * H + 255) / 256)), dim3(256), 0, 0, sc, 0, W, 0, H,
                       cls.ptr);
    MPSS_HIP(hipGetLastError());
    std::vector<uint8_t> h((size_t)W * H);
    MPSS_HIP(hipMemcpy(h.data(), cls.ptr, h.size(), hipMemcpyDeviceToHost));
    for (int i = 0; i < n; ++i) {
        const int32_t *r = rects + 4 * i;
        if (r[0] < 0 || r[2] < 0 || r[1] > W || r[3] > H || r[0] >= r[1] || r[2] >= r[3])
            throw Error(MPSS_ERR_INVALID, "tile_costs: bad rectangle");
        int64_t a = 0, b = 0;
        for (int y = r[2]; y < r[3]; ++y)
            for (int x = r[0]; x < r[1]; ++x) {
                const uint8_t c = h[(size_t)y * W + x];
                a += c == 2;
                b += c >= 1;
            }
        sss[i] = a;
        surf[i] = b;
    }
}

void Context::time_begin(bool on, hipStream_t s, hipEvent_t &a) {
    if (!on) return;
    MPSS_HIP(hipEventCreate(&a));
    MPSS_HIP(hipEventRecord(a, s));
}

void Context::time_end(bool on, hipStream_t s, hipEvent_t a, int kind, std::vector<Timed> &out) {
    if (!on) return;
    hipEvent_t b;
    MPSS_HIP(hipEventCreate(&b));
    MPSS_HIP(hipEventRecord(b, s));
    out.push_back(Timed{a, b, kind});
}

mpss_render_stats Context::render_stats() {
    activate();
    std::lock_guard<std::mutex> g(mu_);
    MPSS_HIP(hipDeviceSynchronize());
    for (const Timed &t : timed_) {
        float ms = 0.f;
        MPSS_HIP(hipEventElapsedTime(&ms, t.a, t.b));
        (void)hipEventDestroy(t.a);
        (void)hipEventDestroy(t.b);
        double *dst[7] = {&stats_.ms_irradiance, &stats_.ms_camera, &stats_.ms_shade, &stats_.ms_film,
                          &stats_.ms_direct, &stats_.ms_tex, &stats_.ms_replay};
        int64_t *cnt[7] = {&stats_.n_irradiance, &stats_.n_camera, &stats_.n_shade, &stats_.n_film, &stats_.n_direct,
                           &stats_.n_tex, &stats_.n_replay};
        *dst[t.kind] += ms;
        *cnt[t.kind] += 1;
    }
    timed_.clear();
    mpss_render_stats out = stats_;
    const int sm = first_bssrdf_material();
    for (int g2 = 0; g2 < kGroups; ++g2)
        for (int s = 0; s < 4; ++s)
            out.group_bands[g2][s] = sm >= 0 ? materials_[sm]->dev_profile.groups.band[g2][s] : -1;
    if (d_counts_.ptr) {
        unsigned long long c[kStatStride * kGroups];
        MPSS_HIP(hipMemcpy(c, d_counts_.ptr, sizeof(c), hipMemcpyDeviceToHost));
        for (int g2 = 0; g2 < kGroups; ++g2) {
            out.mo_nodes += (int64_t)c[kStatStride * g2];
            out.mo_points += (int64_t)c[kStatStride * g2 + 1];
            out.group_nodes[g2] = (int64_t)c[kStatStride * g2];
            out.group_points[g2] = (int64_t)c[kStatStride * g2 + 1];
            out.mo_wave_node_iters += (int64_t)c[kStatStride * g2 + 2];
            out.mo_wave_point_iters += (int64_t)c[kStatStride * g2 + 3];
            out.mo_lookups += (int64_t)c[kStatStride * g2 + 4];
            for (int k = 0; k < 3; ++k) out.mo_lookups_near[k] += (int64_t)c[kStatStride * g2 + 5 + k];
            out.mo_row_lane_records += (int64_t)c[kStatStride * g2 + 8];
            out.mo_lds_lane_records += (int64_t)c[kStatStride * g2 + 9];
            out.mo_table_lane_records += (int64_t)c[kStatStride * g2 + 10];
            for (int k = 0; k < 3; ++k) out.group_path_records[g2][k] = (int64_t)c[kStatStride * g2 + 8 + k];
            for (int k = 0; k < 2; ++k) {
                out.group_path_sectors[g2][k] = (int64_t)c[kStatStride * g2 + 11 + k];
                out.group_path_lines[g2][k] = (int64_t)c[kStatStride * g2 + 13 + k];
                out.group_path_fetches[g2][k] = (int64_t)c[kStatStride * g2 + 15 + k];
            }
        }
    }
    return out;
}

void Context::reset_render_stats() {
    (void)render_stats();  // drain pending events
    std::lock_guard<std::mutex> g(mu_);
    stats_ = mpss_render_stats{};
    if (d_counts_.ptr) MPSS_HIP(hipMemset(d_counts_.ptr, 0, kStatStride * kGroups * sizeof(unsigned long long)));
}

int Context::first_bssrdf_material() const {
    for (size_t i = 0; i < materials_.size(); ++i)
        if (!materials_[i]->dipole && !materials_[i]->no_bssrdf) return (int)i;
    return -1;
}

}  // namespace mpss
