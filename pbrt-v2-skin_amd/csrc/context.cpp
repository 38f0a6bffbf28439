// context.cpp -- Context implementation (material preparation, octree upload).
#include "context.h"
#include "spectral.h"

#include <cstring>

namespace mpss {

Context::Context(const mpss_config &cfg) : cfg_(cfg) {
    int ndev = 0;
    MPSS_HIP(hipGetDeviceCount(&ndev));
    if (cfg.device < 0 || cfg.device >= ndev)
        throw Error(MPSS_ERR_INVALID, "mpss_create: device ordinal " + std::to_string(cfg.device) +
                                          " out of range (" + std::to_string(ndev) + " HIP devices)");
    if (cfg.mo_near_field != 10236 && cfg.mo_near_field != 5088)
        throw Error(MPSS_ERR_INVALID, "mpss_create: mo_near_field must be 10236 or 5088");
    if (cfg.mo_common_grid != 0 && cfg.mo_common_grid != 1)
        throw Error(MPSS_ERR_INVALID, "mpss_create: mo_common_grid must be 0 or 1");
    if (cfg.mo_band_dealing != 0 && cfg.mo_band_dealing != 1)
        throw Error(MPSS_ERR_INVALID, "mpss_create: mo_band_dealing must be 0 or 1");
    max_error_ = cfg.max_error;
    min_dist_ = cfg.min_sample_distance;
    if (cfg.quick_render) {  // multipolesubsurface.cpp:401 [file line]
        max_error_ *= 4.f;
        min_dist_ *= 4.f;
    }
    activate();
}

Context::~Context() {
    (void)hipSetDevice(cfg_.device);
    (void)hipDeviceSynchronize();
    for (const Timed &t : timed_) {
        (void)hipEventDestroy(t.a);
        (void)hipEventDestroy(t.b);
    }
}

RenderWorkspace::~RenderWorkspace() {
    if (done) {
        (void)hipSetDevice(device);
        (void)hipEventSynchronize(done);
        (void)hipEventDestroy(done);
    }
}

// A free workspace from the pool -- preferably one whose last user's kernels are done, so this call
// need not queue behind another stream -- or a new one (mu_ held).
RenderWorkspace *Context::acquire_ws() {
    if (!ws_free_.empty()) {
        size_t pick = ws_free_.size() - 1;
        for (size_t i = ws_free_.size(); i-- > 0;)
            if (!ws_free_[i]->pending || hipEventQuery(ws_free_[i]->done) == hipSuccess) {
                pick = i;
                break;
            }
        RenderWorkspace *w = ws_free_[pick].release();
        ws_free_.erase(ws_free_.begin() + (std::ptrdiff_t)pick);
        return w;
    }
    auto w = std::make_unique<RenderWorkspace>();
    w->device = cfg_.device;
    MPSS_HIP(hipEventCreateWithFlags(&w->done, hipEventDisableTiming));
    w->work.alloc(kGroups);
    w->count.alloc(1);
    return w.release();
}

// Back to the pool after its last kernel on `stream` (the next user waits on `done`). The pool keeps
// at most kMaxIdleWorkspaces: a burst of concurrent callers does not pin its peak memory (a full C2
// batch workspace is several GB) for the context's lifetime; the oldest idle one is freed first.
constexpr size_t kMaxIdleWorkspaces = 4;
hipError_t Context::release_ws_nothrow(RenderWorkspace *ws, hipStream_t stream) noexcept {
    const hipError_t e = hipEventRecord(ws->done, stream);
    ws->pending = e == hipSuccess;
    std::unique_ptr<RenderWorkspace> drop;
    try {
        std::lock_guard<std::mutex> g(mu_);
        ws_free_.emplace_back(ws);
        if (ws_free_.size() > kMaxIdleWorkspaces) {
            drop = std::move(ws_free_.front());
            ws_free_.erase(ws_free_.begin());
        }
    } catch (...) {  // the pool could not take it back: free it here
        if (!drop) drop.reset(ws);
    }
    drop.reset();  // waits for its last kernels, outside the lock
    return e;
}

void Context::release_ws(RenderWorkspace *ws, hipStream_t stream) { MPSS_HIP(release_ws_nothrow(ws, stream)); }

// mu_ held (by the caller's lock on it): wait out every in-flight render_tiles / mo_batch, then
// their kernels, before device state they read is replaced.
void Context::quiesce_locked() {
    idle_.wait(mu_, [&] { return inflight_ == 0; });
    MPSS_HIP(hipDeviceSynchronize());
}

// An in-flight call has queued its kernels (mu_ not held).
void Context::end_inflight() {
    std::lock_guard<std::mutex> g(mu_);
    if (--inflight_ == 0) idle_.notify_all();
}

void Context::ensure_layouts() {
    if (!have_octree_) return;
    for (const auto &m : materials_)
        if (!m->dipole) dev_octree_.ensure_layout(m->dev_profile.groups);
}

// SubsurfaceOctreeNode::Mo for a batch of points (mpss_mo_batch). The octree, profile and band
// layout are read-only here; the chunk counters of the sharded gather come from a pooled
// workspace, so concurrent calls on different streams share nothing they write.
void Context::mo_batch(uint32_t mid, int q, const float *p_dev, float *out_dev, int32_t *counters_dev,
                       hipStream_t stream) {
    activate();
    RenderWorkspace *ws = nullptr;
    const BandLayout *layout = nullptr;
    const Material *m = nullptr;
    int mode;
    GatherOpts opts;
    {
        std::lock_guard<std::mutex> g(mu_);
        opts = gather_opts();
        if (!have_octree_) throw Error(MPSS_ERR_INVALID, "no irradiance points: call mpss_set_irradiance_points first");
        if (mid >= materials_.size()) throw Error(MPSS_ERR_INVALID, "unknown material id " + std::to_string(mid));
        m = materials_[mid].get();
        if (m->no_bssrdf)
            throw Error(MPSS_ERR_INVALID, "material " + std::to_string(mid) + " has no profile (genprofile false)");
        mode = cfg_.exact_mo;
        if (m->dipole) {
            mode = -1;  // closed-form functor: the reference-order gather (dipole.h)
        } else if (m->rgb && mode != 0) {
            mode = -2;  // FromRGB of three lookups in the reference order (exact_mo 1; also for the packet mode)
        } else if (mode == 0) {
            layout = &dev_octree_.ensure_layout(m->dev_profile.groups);
            ws = acquire_ws();
        }
        ++inflight_;  // until the kernels are queued (an octree rebuild waits for it)
    }
    InflightGuard guard{this, ws, stream};
    if (mode == -1) {
        launch_mo_dipole(dev_octree_, m->dev_dipole.ptr, max_error_, q, p_dev, out_dev, NB, counters_dev, stream);
        return;
    }
    if (mode == -2) {
        launch_mo_rgb(dev_octree_, m->dev_rgb.ptr, m->dev_rgb_rcp.ptr, m->rgb_rcp, m->profile.length, max_error_, q,
                      p_dev, nullptr, nullptr, nullptr, 0, out_dev, NB, counters_dev, stream);
        return;
    }
    int *perm = nullptr;
    if (ws) {
        const int64_t need = ((int64_t)q + 1023) / 1024 * 1024;
        if (ws->perm_n < need) {
            if (ws->pending) MPSS_HIP(hipEventSynchronize(ws->done));
            ws->perm.alloc((size_t)need);
            ws->perm_n = need;
        }
        perm = ws->perm.ptr;
        if (ws->pending) MPSS_HIP(hipStreamWaitEvent(stream, ws->done, 0));
    }
    launch_mo_gather(dev_octree_, layout, m->dev_profile, max_error_, q, p_dev, out_dev, NB, counters_dev,
                     ws ? ws->work.ptr : nullptr, perm, mode, opts, stream);
    guard.release();
}

void Context::activate() const { MPSS_HIP(hipSetDevice(cfg_.device)); }

void Context::gather_info(uint32_t id, int *common_grid, float *rel_err, float *l1_err) const {
    const Material &m = material(id);  // (takes mu_; materials are never replaced)
    const bool band = !m.dipole;  // (rgbprofile: the grid of its R, G, B profiles, rel/l1_err[0..2])
    const int lay = cfg_.mo_near_field == 10236 ? 0 : 1;  // the grid of the configured LDS layout
    const bool on = band && cfg_.exact_mo == 0 && cfg_.mo_common_grid != 0 &&
                    (lay == 0 ? m.dev_profile.cg.on : m.dev_profile.cg_half.on);
    *common_grid = on ? 1 : 0;
    for (int c = 0; c < NB; ++c) {
        if (rel_err) rel_err[c] = band ? m.dev_profile.cg_rel_err[lay][c] : 0.f;
        if (l1_err) l1_err[c] = band ? m.dev_profile.cg_l1_err[lay][c] : 0.f;
    }
}

// Material ids travel in 8 bits of the render path's per-sample records (render.h REC_MAT_SHIFT).
constexpr size_t kMaxMaterials = 256;

uint32_t Context::add_layeredskin(const mpss_layeredskin &m) {
    activate();
    std::lock_guard<std::mutex> g(mu_);
    if (materials_.size() >= kMaxMaterials) throw Error(MPSS_ERR_INVALID, "at most 256 materials per context");
    auto mat = std::make_unique<Material>();
    SkinParams sp;
    sp.roughness = m.roughness;
    sp.nmperunit = m.nmperunit;
    sp.f_mel = m.f_mel;
    sp.f_eu = m.f_eu;
    sp.f_blood = m.f_blood;
    sp.f_ohg = m.f_ohg;
    for (int l = 0; l < 2; ++l) {
        sp.thickness_nm[l] = m.layer_thickness_nm[l];
        sp.ior[l] = m.layer_ior[l];
    }
    sp.desired_length = m.desired_length;
    sp.lerp_on_thin_slab = m.lerp_on_thin_slab != 0;
    sp.double_ref_sslf = m.double_ref_sslf != 0;
    LayerParams lp;
    skin_layer_params(sp, lp);
    if (m.rgb_profile) {
        // ComputeRGBMultipoleProfile (multipole.cpp:408-451, layeredskin.cpp:85-86,97-99): each layer's
        // mua / musp as ToRGBSpectrum, profile channel k from component k. Every band c is built
        // from component c % 3, so rows 0..2 of the table are the R, G, B profiles.
        for (int l = 0; l < 2; ++l) {
            float ra[3], rs[3];
            spectrum_to_rgb(lp.mua[l], ra);
            spectrum_to_rgb(lp.musp[l], rs);
            for (int c = 0; c < NB; ++c) {
                lp.mua[l][c] = ra[c % 3];
                lp.musp[l][c] = rs[c % 3];
            }
        }
        mat->rgb = true;
    }
    const int distinct = m.rgb_profile ? 3 : NB;  // rgbprofile: 3 distinct channels (R, G, B)
    if (!m.gen_profile) {
        // preparedBSSRDFData = NULL: a zero placeholder profile and rho table (never read by a gather)
        mat->no_bssrdf = true;
        mat->rgb = false;
        irradiance_points_profile(1.f, mat->profile, mat->rho);
        std::fill(mat->profile.table.begin(), mat->profile.table.end(), 0.f);
    } else if (m.show_irradiance_points) {
        // ComputeIrradiancePointsProfile(irradiancePointSize) + ComputeRoughRhoData (layeredskin.cpp:
        // 93-95), in place of the multipole profile (rgbprofile / usemontecarlo are not consulted)
        mat->rgb = false;
        irradiance_points_profile(m.irradiance_point_size, mat->profile, mat->rho);
    } else if (m.use_monte_carlo && !m.rgb_profile)
        build_profile_mc(lp, m.photons, 89, mat->profile);
    else if (cfg_.profile_on_host || sp.desired_length > 1024)
        build_profile(lp, sp.desired_length, sp.lerp_on_thin_slab, mat->profile, 0, distinct);
    else
        build_profile_gpu(lp, sp.desired_length, sp.lerp_on_thin_slab, mat->profile, 0, distinct);
    if (!m.gen_profile || m.show_irradiance_points)
        ;  // (rho set above)
    else if (cfg_.profile_on_host)
        build_rho_table(sp.roughness, sp.ior[0], sp.double_ref_sslf, 1025, 256, mat->rho);
    else
        build_rho_table_gpu(sp.roughness, sp.ior[0], sp.double_ref_sslf, 1025, 256, mat->rho);
    memcpy(mat->albedo, m.albedo, sizeof(mat->albedo));
    memcpy(mat->Kr, m.Kr, sizeof(mat->Kr));
    memcpy(mat->Kt, m.Kt, sizeof(mat->Kt));
    mat->roughness = m.roughness;
    mat->ior = m.layer_ior[0];
    mat->double_ref_sslf = m.double_ref_sslf != 0;
    // Ft = 1 in Li (multipolesubsurface.cpp:285); MultipoleBSSRDFData(..., useMonteCarloProfile) keeps the
    // flag whichever profile was prepared (layeredskin.cpp:116)
    mat->is_monte_carlo = m.use_monte_carlo != 0;
    mat->dev_profile.upload(mat->profile.table.data(), mat->profile.length, mat->profile.rcp, cfg_.mo_band_dealing == 1);
    if (mat->rgb) {
        mat->dev_rgb.upload(mat->profile.table.data(), 3 * (size_t)mat->profile.length);
        for (int k = 0; k < 3; ++k) mat->rgb_rcp[k] = mat->profile.rcp[k];
        mat->dev_rgb_rcp.upload(mat->rgb_rcp, 3);
        mat->dev_profile.set_rgb(mat->profile.table.data());  // the sharded gather's three lookups + FromRGB
    }
    mat->dev_rho.upload(mat->rho.hd.data(), mat->rho.hd.size());
    materials_.push_back(std::move(mat));
    scene_dirty_ = true;
    ensure_layouts();
    return (uint32_t)materials_.size() - 1;
}

uint32_t Context::set_material_tables(const float *rd, uint32_t len, const float *rcp, const float *rho,
                                      uint32_t n_rho, const float *albedo, bool is_mc) {
    activate();
    std::lock_guard<std::mutex> g(mu_);
    if (materials_.size() >= kMaxMaterials) throw Error(MPSS_ERR_INVALID, "at most 256 materials per context");
    auto mat = std::make_unique<Material>();
    mat->profile.length = (int)len;
    mat->profile.table.assign(rd, rd + (size_t)NB * len);
    for (int c = 0; c < NB; ++c) {
        mat->profile.rcp[c] = rcp[c];
        mat->profile.spacing[c] = 1.f / rcp[c];
        mat->profile.total_reflectance[c] = 0.f;
    }
    mat->rho.hd.assign(rho, rho + n_rho);
    for (int c = 0; c < NB; ++c) {
        mat->albedo[c] = albedo ? albedo[c] : 1.f;
        mat->Kr[c] = 1.f;
        mat->Kt[c] = 0.f;
    }
    mat->is_monte_carlo = is_mc;
    mat->dev_profile.upload(mat->profile.table.data(), mat->profile.length, mat->profile.rcp, cfg_.mo_band_dealing == 1);
    mat->dev_rho.upload(mat->rho.hd.data(), mat->rho.hd.size());
    materials_.push_back(std::move(mat));
    scene_dirty_ = true;
    ensure_layouts();
    return (uint32_t)materials_.size() - 1;
}

uint32_t Context::add_dipole_material(const float *sigma_a, const float *sigmap_s, float eta) {
    activate();
    std::lock_guard<std::mutex> g(mu_);
    if (materials_.size() >= kMaxMaterials) throw Error(MPSS_ERR_INVALID, "at most 256 materials per context");
    auto mat = std::make_unique<Material>();
    mat->dipole = true;
    dipole_init(sigma_a, sigmap_s, eta, mat->dip);
    float packed[4 * NB];
    for (int c = 0; c < NB; ++c) {
        packed[c] = mat->dip.zpos[c];
        packed[NB + c] = mat->dip.zneg[c];
        packed[2 * NB + c] = mat->dip.sigma_tr[c];
        packed[3 * NB + c] = mat->dip.k[c];
        mat->albedo[c] = 1.f;
        mat->Kr[c] = 1.f;
        mat->Kt[c] = 0.f;
    }
    mat->ior = eta;
    mat->dev_dipole.upload(packed, 4 * NB);
    mat->rho.hd.assign(2, 0.f);
    mat->dev_rho.upload(mat->rho.hd.data(), mat->rho.hd.size());
    materials_.push_back(std::move(mat));
    scene_dirty_ = true;
    return (uint32_t)materials_.size() - 1;
}

std::unique_ptr<ImageTexture> build_imagemap(const mpss_imagemap &m) {
    auto t = std::make_unique<ImageTexture>();
    const int nch = m.is_float ? 1 : 3;
    if (m.width <= 0 || m.height <= 0 || !m.texels) {
        // the image could not be read: a one-valued MIPMap(1, 1, oneVal) with the MIPMap defaults
        // (no trilinear, maxAniso 8, TEXTURE_REPEAT), oneVal = powf(scale * (1 + shift), gamma)
        const float one = m_pow(m.scale * (1 + m.shift), m.gamma);
        const float v[3] = {one, one, one};
        t->py = build_pyramid(1, 1, nch, v, TEX_REPEAT);
        t->trilinear = 0;
        t->max_aniso = 8.f;
    } else {
        if ((int64_t)m.width * m.height > (int64_t)1 << 28) throw Error(MPSS_ERR_INVALID, "imagemap: image too large");
        const size_t n = (size_t)m.width * m.height;
        std::vector<float> conv(n * nch);
        for (size_t i = 0; i < n; ++i) {
            const float *x = m.texels + 3 * i;
            if (nch == 3) {  // convertIn(RGBSpectrum): scale * (Pow(from, gamma) + shift)
                for (int k = 0; k < 3; ++k) conv[3 * i + k] = m.scale * (m_pow(x[k], m.gamma) + m.shift);
            } else {         // convertIn(float): scale * (powf(from.y(), gamma) + shift)
                const float y = (0.212671f * x[0] + 0.715160f * x[1]) + 0.072169f * x[2];
                conv[i] = m.scale * (m_pow(y, m.gamma) + m.shift);
            }
        }
        if (m.wrap < TEX_REPEAT || m.wrap > TEX_CLAMP) throw Error(MPSS_ERR_INVALID, "imagemap: bad wrap mode");
        t->py = build_pyramid(m.width, m.height, nch, conv.data(), m.wrap);
        t->trilinear = m.trilinear != 0;
        t->max_aniso = m.max_anisotropy;
    }
    t->su = m.uscale;
    t->sv = m.vscale;
    t->du = m.udelta;
    t->dv = m.vdelta;
    t->host = t->py.view(t->trilinear, t->max_aniso);
    t->host.su = t->su;
    t->host.sv = t->sv;
    t->host.du = t->du;
    t->host.dv = t->dv;
    return t;
}

uint32_t Context::add_imagemap(const mpss_imagemap &m) {
    std::lock_guard<std::mutex> g(mu_);
    textures_.push_back(build_imagemap(m));
    scene_dirty_ = true;
    return (uint32_t)textures_.size() - 1;
}

void Context::set_material_textures(uint32_t material, int albedo, int bump) {
    std::lock_guard<std::mutex> g(mu_);
    if (material >= materials_.size()) throw Error(MPSS_ERR_INVALID, "set_material_textures: unknown material id");
    auto check = [&](int id, bool want_float, const char *what) {
        if (id < 0) return;
        if (id >= (int)textures_.size())
            throw Error(MPSS_ERR_INVALID, std::string("set_material_textures: unknown texture id for ") + what);
        if ((textures_[id]->py.nch == 1) != want_float)
            throw Error(MPSS_ERR_INVALID, std::string("set_material_textures: ") + what +
                                              (want_float ? " needs a float texture" : " needs a spectrum texture"));
    };
    check(albedo, false, "albedo");
    check(bump, true, "bumpmap");
    materials_[material]->albedo_tex = albedo;
    materials_[material]->bump_tex = bump;
    scene_dirty_ = true;
}

std::vector<const TexView *> Context::host_bump_views() const {
    std::vector<const TexView *> v(materials_.size(), nullptr);
    for (size_t i = 0; i < materials_.size(); ++i)
        if (materials_[i]->bump_tex >= 0) v[i] = &textures_[materials_[i]->bump_tex]->host;
    return v;
}

const Material &Context::material(uint32_t id) const {
    std::lock_guard<std::mutex> g(mu_);
    if (id >= materials_.size()) throw Error(MPSS_ERR_INVALID, "unknown material id " + std::to_string(id));
    return *materials_[id];
}

void Context::set_irradiance_points(int n, const float *p, const float *nrm, const float *E, const float *area) {
    activate();
    std::lock_guard<std::mutex> g(mu_);
    quiesce_locked();  // no gather of the old octree may still be in flight or running
    build_octree_locked(n, p, nrm, E, area);
}

// SubsurfaceOctreeNode::Insert / InitHierarchy over the points, the device copy and every
// material's band layout (mu_ held).
void Context::build_octree_locked(int n, const float *p, const float *nrm, const float *E, const float *area,
                                  const float *dp, const float *dn, const float *dE) {
    have_octree_ = false;
    if (cfg_.octree_on_host) {
        FlatOctree host;
        build_octree(n, p, nrm, E, area, host);
        dev_octree_.upload(host);
    } else {
        if (n <= 0) throw Error(-1, "build_octree: no irradiance points");
        float bmin[3] = {INFINITY, INFINITY, INFINITY}, bmax[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int i = 0; i < n; ++i)  // Union(BBox, Point), core/geometry.cpp:38-47
            for (int k = 0; k < 3; ++k) {
                const float v = p[3 * (size_t)i + k];
                bmin[k] = (v < bmin[k]) ? v : bmin[k];
                bmax[k] = (bmax[k] < v) ? v : bmax[k];
            }
        DevBuf<float> up, un, uE, uA;
        if (!dp) up.upload(p, 3 * (size_t)n);
        if (!dn) un.upload(nrm, 3 * (size_t)n);
        if (!dE) uE.upload(E, (size_t)n * NB);
        uA.upload(area, n);
        build_octree_device(n, dp ? dp : up.ptr, dn ? dn : un.ptr, dE ? dE : uE.ptr, uA.ptr, bmin, bmax, dev_octree_);
    }
    have_octree_ = true;
    dev_octree_.ensure_leaf_r2(max_error_);
    ensure_layouts();
}

void Context::export_octree(void *nodes, float *node_et, float *pt_hdr, float *pt_e, int32_t *pt_index) {
    activate();
    std::lock_guard<std::mutex> g(mu_);
    if (!have_octree_) throw Error(MPSS_ERR_INVALID, "no irradiance points: call mpss_set_irradiance_points first");
    const DeviceOctree &t = dev_octree_;
    MPSS_HIP(hipDeviceSynchronize());
    if (nodes) MPSS_HIP(hipMemcpy(nodes, t.nodes.ptr, sizeof(NodeHdr) * t.n_nodes, hipMemcpyDeviceToHost));
    if (node_et) MPSS_HIP(hipMemcpy(node_et, t.node_et.ptr, sizeof(float) * ROW * t.n_nodes, hipMemcpyDeviceToHost));
    if (pt_hdr) MPSS_HIP(hipMemcpy(pt_hdr, t.pt_hdr.ptr, sizeof(float4) * t.n_points, hipMemcpyDeviceToHost));
    if (pt_e) MPSS_HIP(hipMemcpy(pt_e, t.pt_e.ptr, sizeof(float) * ROW * t.n_points, hipMemcpyDeviceToHost));
    if (pt_index) MPSS_HIP(hipMemcpy(pt_index, t.pt_index.ptr, sizeof(int) * t.n_points, hipMemcpyDeviceToHost));
}

const DeviceOctree &Context::octree() const {
    if (!have_octree_) throw Error(MPSS_ERR_INVALID, "no irradiance points: call mpss_set_irradiance_points first");
    return dev_octree_;
}

}  // namespace mpss
