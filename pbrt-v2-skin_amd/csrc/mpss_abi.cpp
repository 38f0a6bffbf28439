// mpss_abi.cpp -- the extern "C" boundary of libmpss (include/mpss.h).
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/mpss.h"
#include "context.h"
#include "material.h"
#include "mc_profile.h"
#include "mo_kernel.h"
#include "spectral.h"

using namespace mpss;

namespace {
thread_local std::string g_last_error;

template <class F>
int guarded(F &&fn) {
    try {
        fn();
        return MPSS_OK;
    } catch (const Error &e) {
        g_last_error = e.what();
        return e.code;
    } catch (const std::bad_alloc &) {
        g_last_error = "out of memory";
        return MPSS_ERR_NOMEM;
    } catch (const std::exception &e) {
        g_last_error = e.what();
        return MPSS_ERR_INTERNAL;
    } catch (...) {
        g_last_error = "unknown error";
        return MPSS_ERR_INTERNAL;
    }
}

void require(bool ok, const char *msg) {
    if (!ok) throw Error(MPSS_ERR_INVALID, msg);
}
}  // namespace

extern "C" {

int mpss_abi_version(void) { return 13; }  // 2: poisson point finder, infinite lights; 3: imagemap textures;
                                          // 4: tile costs, wave-iteration stats, thread-safe calls;
                                          // 5: reference-sampler replay, dipole materials;
                                          // 6: GPU octree build (octree_on_host), mpss_octree_export;
                                          // 7: gather choices in mpss_config (mo_band_dealing,
                                          //    mo_work_stealing, mo_near_field), count_traversal 2;
                                          // 8: light spheres seen directly shaded (default matte),
                                          //    rebuilds wait for in-flight render / mo_batch calls;
                                          // 9: GPU tessellation (tessellate_on_host), size bounds
                                          // 10: mo_common_grid, mpss_get_gather_info, common-grid
                                          //     lane-record counts in mpss_render_stats
                                          // 11: rgbprofile through the sharded gather (its own common
                                          //     grid), mpss_host_common_grid u1start / rgb mode
                                          // 12: LayeredSkin genprofile / showirradiancepoints /
                                          //     irradiancepointsize; mpss_host_common_grid near_field
                                          // 13: per-group, per-path L2 footprint in mpss_render_stats;
                                          //     common-grid rows H steps apart past ua, bad cells
                                          //     flagged (mpss_host_common_grid ua / hinv)
const char *mpss_last_error(void) { return g_last_error.c_str(); }

void mpss_config_defaults(mpss_config *c) {
    if (!c) return;
    c->device = 0;
    c->max_depth = 5;
    c->max_error = .05f;
    c->min_sample_distance = .25f;
    c->mix = .5f;
    c->show_irradiance_points = 0;
    c->incenter = 0;
    c->quick_render = 0;
    c->exact_mo = 0;
    c->kernel_timing = 0;
    c->count_traversal = 0;
    c->profile_on_host = 0;
    c->max_batch_samples = (int64_t)1 << 26;
    c->use_poisson_point_finder = 0;
    c->sampler = MPSS_SAMPLER_HASH;
    c->replay_cores = 8;
    c->octree_on_host = 0;
    c->mo_band_dealing = 0;
    c->mo_work_stealing = 1;
    c->mo_near_field = 5088;
    c->tessellate_on_host = 0;
    c->mo_common_grid = 1;
}

int mpss_create(const mpss_config *cfg, mpss_ctx **out) {
    return guarded([&] {
        require(cfg && out, "mpss_create: null argument");
        *out = nullptr;
        auto ctx = std::make_unique<Context>(*cfg);
        *out = reinterpret_cast<mpss_ctx *>(ctx.release());
    });
}

void mpss_destroy(mpss_ctx *ctx) { delete reinterpret_cast<Context *>(ctx); }

void mpss_layeredskin_defaults(mpss_layeredskin *m) {
    if (!m) return;
    m->roughness = 0.4f;
    m->nmperunit = 100e6f;
    m->f_mel = 0.15f;
    m->f_eu = 1.f;
    m->f_blood = 0.002f;
    m->f_ohg = 0.3f;
    m->ga_epi = 0.9f;
    m->ga_derm = 0.8f;
    m->b_derm = 0.4f;
    m->layer_thickness_nm[0] = 0.25e6f;
    m->layer_thickness_nm[1] = 20e6f;
    m->layer_ior[0] = m->layer_ior[1] = 1.4f;
    for (int i = 0; i < MPSS_NBANDS; ++i) m->albedo[i] = m->Kr[i] = m->Kt[i] = 1.f;
    m->desired_length = 512;
    m->lerp_on_thin_slab = 1;
    m->double_ref_sslf = 0;
    m->use_monte_carlo = 0;
    m->photons = 10000000ull;
    m->rgb_profile = 0;
    m->gen_profile = 1;
    m->show_irradiance_points = 0;
    m->irradiance_point_size = 0.002f;
}

int mpss_add_layeredskin(mpss_ctx *c, const mpss_layeredskin *m, uint32_t *id) {
    return guarded([&] {
        require(c && m && id, "mpss_add_layeredskin: null argument");
        require(m->desired_length >= 2 && m->desired_length <= 4096, "desiredlength out of range [2, 4096]");
        require(m->nmperunit > 0.f, "nmperunit must be positive");
        require(!m->show_irradiance_points || m->irradiance_point_size > 0.f,
                "irradiancepointsize must be positive with showirradiancepoints");
        *id = reinterpret_cast<Context *>(c)->add_layeredskin(*m);
    });
}

void mpss_imagemap_defaults(mpss_imagemap *t) {
    if (!t) return;
    memset(t, 0, sizeof(*t));
    t->scale = 1.f;
    t->gamma = 1.f;
    t->max_anisotropy = 8.f;
    t->uscale = t->vscale = 1.f;
}

int mpss_add_imagemap(mpss_ctx *c, const mpss_imagemap *t, uint32_t *id) {
    return guarded([&] {
        require(c && t && id, "mpss_add_imagemap: null argument");
        *id = reinterpret_cast<Context *>(c)->add_imagemap(*t);
    });
}

int mpss_set_material_textures(mpss_ctx *c, uint32_t mid, int32_t albedo, int32_t bump) {
    return guarded([&] {
        require(c != nullptr, "mpss_set_material_textures: null context");
        reinterpret_cast<Context *>(c)->set_material_textures(mid, albedo, bump);
    });
}

int mpss_set_material_tables(mpss_ctx *c, const float *rd, uint32_t len, const float *rcp, const float *rho,
                             uint32_t n_rho, const float *albedo, int is_mc, uint32_t *id) {
    return guarded([&] {
        require(c && rd && rcp && rho && id, "mpss_set_material_tables: null argument");
        require(len >= 2 && n_rho >= 2, "tables need at least 2 entries");
        *id = reinterpret_cast<Context *>(c)->set_material_tables(rd, len, rcp, rho, n_rho, albedo, is_mc != 0);
    });
}

int mpss_add_dipole_material(mpss_ctx *c, const float *sigma_a, const float *sigmap_s, float eta, uint32_t *id) {
    return guarded([&] {
        require(c && sigma_a && sigmap_s && id, "mpss_add_dipole_material: null argument");
        require(eta > 0.f, "mpss_add_dipole_material: eta must be positive");
        *id = reinterpret_cast<Context *>(c)->add_dipole_material(sigma_a, sigmap_s, eta);
    });
}

int mpss_get_material_tables(mpss_ctx *c, uint32_t id, float *rd, uint32_t *len, float *rcp, float *rho,
                             uint32_t *n_rho, float *total) {
    return guarded([&] {
        require(c && len && n_rho, "mpss_get_material_tables: null argument");
        const Material &m = reinterpret_cast<Context *>(c)->material(id);
        *len = (uint32_t)m.profile.length;
        *n_rho = (uint32_t)m.rho.hd.size();
        if (rd) memcpy(rd, m.profile.table.data(), sizeof(float) * m.profile.table.size());
        if (rcp) memcpy(rcp, m.profile.rcp, sizeof(float) * NB);
        if (rho) memcpy(rho, m.rho.hd.data(), sizeof(float) * m.rho.hd.size());
        if (total) memcpy(total, m.profile.total_reflectance, sizeof(float) * NB);
    });
}

int mpss_host_common_grid(const float *table, uint32_t L, const float *rcp, int snake, int near_field, float *rows,
                          uint32_t *n_rows, int32_t *bands, float *rg, float *u0lim, float *u1lim, float *u1start,
                          uint32_t *row0, uint32_t *ubase, float *rel_err, float *l1_err, float *ua, float *hinv,
                          int *ok) {
    return guarded([&] {
        require(table && rcp && ok, "mpss_host_common_grid: null argument");
        require(L >= 2 && L < (1u << 24), "mpss_host_common_grid: L out of range");
        require(snake >= 0 && snake <= 2, "mpss_host_common_grid: snake must be 0, 1 or 2");
        require(near_field == 10236 || near_field == 5088, "mpss_host_common_grid: near_field must be 10236 or 5088");
        BandGroups g = make_band_groups(rcp, snake == 1);
        if (snake == 2)  // rgbprofile: rows 0..2 (R, G, B) in every group (DeviceProfile::set_rgb)
            for (int k = 0; k < kGroups; ++k)
                for (int j = 0; j < 4; ++j) g.band[k][j] = j < 3 ? j : -1;
        CommonGrid cg;
        std::vector<float4> h;
        float rel[NB], l1[NB];
        *ok = build_common_grid(table, (int)L, rcp, g, cg, h, rel, l1, near_field, snake == 2 ? 28 : 0, snake == 2) ? 1 : 0;
        if (n_rows) {
            if (rows) require(*n_rows >= h.size() / 2, "mpss_host_common_grid: rows too small");
            *n_rows = (uint32_t)(h.size() / 2);
        }
        if (rows) memcpy(rows, h.data(), sizeof(float4) * h.size());
        for (int k = 0; k < kGroups; ++k) {
            for (int j = 0; j < 4; ++j)
                if (bands) bands[4 * k + j] = g.band[k][j];
            if (rg) rg[k] = cg.rg[k];
            if (u0lim) u0lim[k] = cg.u0lim[k];
            if (u1lim) u1lim[k] = cg.u1lim[k];
            if (u1start) u1start[k] = cg.u1start[k];
            if (row0) row0[k] = cg.row0[k];
            if (ubase) ubase[k] = cg.ubase[k];
            if (ua) ua[k] = cg.ua[k];
            if (hinv) hinv[k] = cg.hinv[k];
        }
        for (int c = 0; c < NB; ++c) {
            if (rel_err) rel_err[c] = rel[c];
            if (l1_err) l1_err[c] = l1[c];
        }
    });
}

int mpss_get_gather_info(mpss_ctx *c, uint32_t id, int *common_grid, float *rel_err, float *l1_err) {
    return guarded([&] {
        require(c && common_grid, "mpss_get_gather_info: null argument");
        reinterpret_cast<Context *>(c)->gather_info(id, common_grid, rel_err, l1_err);
    });
}

int mpss_set_irradiance_points(mpss_ctx *c, uint32_t n, const float *p, const float *nrm, const float *E,
                               const float *area) {
    return guarded([&] {
        require(c && p && nrm && E && area, "mpss_set_irradiance_points: null argument");
        require(n > 0, "mpss_set_irradiance_points: empty point set");
        require(n <= (1u << 30), "mpss_set_irradiance_points: at most 2^30 points");
        reinterpret_cast<Context *>(c)->set_irradiance_points((int)n, p, nrm, E, area);
    });
}

int mpss_octree_info(mpss_ctx *c, uint32_t *nn, uint32_t *md, uint32_t *np) {
    return guarded([&] {
        require(c, "mpss_octree_info: null ctx");
        const DeviceOctree &t = reinterpret_cast<Context *>(c)->octree();
        if (nn) *nn = (uint32_t)t.n_nodes;
        if (md) *md = (uint32_t)t.max_depth;
        if (np) *np = (uint32_t)t.n_points;
    });
}

int mpss_octree_export(mpss_ctx *c, void *nodes, float *node_et, float *pt_hdr, float *pt_e, int32_t *pt_index) {
    return guarded([&] {
        require(c, "mpss_octree_export: null ctx");
        reinterpret_cast<Context *>(c)->export_octree(nodes, node_et, pt_hdr, pt_e, pt_index);
    });
}

int mpss_mo_batch(mpss_ctx *c, uint32_t id, uint32_t q, const float *p_dev, float *mo_dev, int32_t *counters_dev,
                  void *stream) {
    return guarded([&] {
        require(c && (q == 0 || (p_dev && mo_dev)), "mpss_mo_batch: null argument");
        require(q <= (1u << 30), "mpss_mo_batch: at most 2^30 queries per call");
        reinterpret_cast<Context *>(c)->mo_batch(id, (int)q, p_dev, mo_dev, counters_dev, (hipStream_t)stream);
    });
}

int mpss_add_mesh(mpss_ctx *c, uint32_t nv, const float *P, const float *N, const float *S, const float *uv,
                  uint32_t nt, const int32_t *idx, const float *o2w, const float *w2o, int rev, uint32_t mat) {
    return guarded([&] {
        require(c && P && idx && o2w && w2o && nv > 0 && nt > 0, "mpss_add_mesh: bad argument");
        reinterpret_cast<Context *>(c)->add_mesh(nv, P, N, S, uv, nt, idx, o2w, w2o, rev != 0, mat);
    });
}

int mpss_add_sphere_light(mpss_ctx *c, const float *center, float r, const float *L, int ns) {
    return guarded([&] {
        require(c && center && L, "mpss_add_sphere_light: null argument");
        reinterpret_cast<Context *>(c)->add_sphere_light(center, r, L, ns);
    });
}

int mpss_add_infinite_light(mpss_ctx *c, const float *L, int ns, const float *l2w, const float *w2l) {
    return guarded([&] {
        require(c && L && l2w && w2l, "mpss_add_infinite_light: null argument");
        reinterpret_cast<Context *>(c)->add_infinite_light(L, ns, l2w, w2l);
    });
}

int mpss_add_infinite_light_map(mpss_ctx *c, const float *L, int ns, const float *l2w, const float *w2l, int w, int h,
                                const float *texels) {
    return guarded([&] {
        require(c && L && l2w && w2l && texels, "mpss_add_infinite_light_map: null argument");
        reinterpret_cast<Context *>(c)->add_infinite_light(L, ns, l2w, w2l, w, h, texels);
    });
}

int mpss_set_camera(mpss_ctx *c, const float *r2c, const float *c2w, int xres, int yres) {
    return guarded([&] {
        require(c && r2c && c2w, "mpss_set_camera: null argument");
        reinterpret_cast<Context *>(c)->set_camera(r2c, c2w, xres, yres);
    });
}

int mpss_set_surface_points(mpss_ctx *c, uint32_t n, const void *rec) {
    return guarded([&] {
        require(c && (n == 0 || rec), "mpss_set_surface_points: null argument");
        reinterpret_cast<Context *>(c)->set_surface_points(n, reinterpret_cast<const SurfacePoint *>(rec));
    });
}

int mpss_get_surface_points(mpss_ctx *c, void *rec, uint32_t *n) {
    return guarded([&] {
        require(c && n, "mpss_get_surface_points: null argument");
        const auto &v = reinterpret_cast<Context *>(c)->surface_points();
        *n = (uint32_t)v.size();
        if (rec) memcpy(rec, v.data(), sizeof(SurfacePoint) * v.size());
    });
}

int mpss_load_pointsfile(mpss_ctx *c, const char *path) {
    return guarded([&] {
        require(c && path, "mpss_load_pointsfile: null argument");
        FILE *f = fopen(path, "rb");
        if (!f) throw Error(MPSS_ERR_INVALID, std::string("mpss_load_pointsfile: cannot open ") + path);
        fseek(f, 0, SEEK_END);
        const long size = ftell(f);
        fseek(f, 0, SEEK_SET);
        std::vector<SurfacePoint> pts((size_t)(size > 0 ? size : 0) / sizeof(SurfacePoint));
        const size_t got = pts.empty() ? 0 : fread(pts.data(), sizeof(SurfacePoint), pts.size(), f);
        fclose(f);
        if (got != pts.size()) throw Error(MPSS_ERR_INVALID, "mpss_load_pointsfile: short read");
        reinterpret_cast<Context *>(c)->set_surface_points((uint32_t)pts.size(), pts.data());
    });
}

int mpss_save_pointsfile(mpss_ctx *c, const char *path) {
    return guarded([&] {
        require(c && path, "mpss_save_pointsfile: null argument");
        const auto &v = reinterpret_cast<Context *>(c)->surface_points();
        FILE *f = fopen(path, "wb");
        if (!f) throw Error(MPSS_ERR_INVALID, std::string("mpss_save_pointsfile: cannot open ") + path);
        const size_t put = v.empty() ? 0 : fwrite(v.data(), sizeof(SurfacePoint), v.size(), f);
        fclose(f);
        if (put != v.size()) throw Error(MPSS_ERR_INVALID, "mpss_save_pointsfile: short write");
    });
}

int mpss_replay_samples(mpss_ctx *c, int spp, float *out, uint64_t *n_floats, int *k) {
    return guarded([&] {
        require(c && n_floats && k, "mpss_replay_samples: null argument");
        require(spp >= 1 && spp <= 32768, "mpss_replay_samples: spp out of range");
        reinterpret_cast<Context *>(c)->replay_samples(spp, out, n_floats, k);
    });
}

int mpss_get_irradiance(mpss_ctx *c, float *E, uint32_t *n) {
    return guarded([&] {
        require(c && n, "mpss_get_irradiance: null argument");
        const auto &v = reinterpret_cast<Context *>(c)->irradiance();
        *n = (uint32_t)(v.size() / NB);
        if (E) memcpy(E, v.data(), sizeof(float) * v.size());
    });
}

int mpss_get_render_stats(mpss_ctx *c, mpss_render_stats *out) {
    return guarded([&] {
        require(c && out, "mpss_get_render_stats: null argument");
        *out = reinterpret_cast<Context *>(c)->render_stats();
    });
}

int mpss_set_instrumentation(mpss_ctx *c, int timing, int counting) {
    return guarded([&] {
        require(c, "mpss_set_instrumentation: null ctx");
        reinterpret_cast<Context *>(c)->set_instrumentation(timing != 0, counting);
    });
}

int mpss_reset_render_stats(mpss_ctx *c) {
    return guarded([&] {
        require(c, "mpss_reset_render_stats: null ctx");
        reinterpret_cast<Context *>(c)->reset_render_stats();
    });
}

int mpss_preprocess(mpss_ctx *c, uint32_t seed) {
    return guarded([&] {
        require(c, "mpss_preprocess: null ctx");
        reinterpret_cast<Context *>(c)->preprocess(seed);
    });
}

int mpss_render_tile(mpss_ctx *c, int spp, uint32_t seed, int x0, int x1, int y0, int y1, float *out, void *stream) {
    return guarded([&] {
        require(c && out, "mpss_render_tile: null argument");
        const int32_t r[4] = {x0, x1, y0, y1};
        float *o[1] = {out};
        reinterpret_cast<Context *>(c)->render_tiles(spp, seed, 1, r, o, (hipStream_t)stream);
    });
}

int mpss_tile_costs(mpss_ctx *c, int n, const int32_t *rects, int64_t *sss_hits, int64_t *surf_hits) {
    return guarded([&] {
        require(c && n >= 0 && (n == 0 || (rects && sss_hits && surf_hits)), "mpss_tile_costs: null argument");
        reinterpret_cast<Context *>(c)->tile_costs(n, rects, sss_hits, surf_hits);
    });
}

int mpss_render_tiles(mpss_ctx *c, int spp, uint32_t seed, int n, const int32_t *rects, float *const *outs,
                      void *stream) {
    return guarded([&] {
        require(c && n >= 0 && (n == 0 || (rects && outs)), "mpss_render_tiles: null argument");
        reinterpret_cast<Context *>(c)->render_tiles(spp, seed, n, rects, outs, (hipStream_t)stream);
    });
}

}  // extern "C"

// ---------------------------------------------------------------- host-side utilities
extern "C" {

int mpss_mc_profile(mpss_ctx *c, const mpss_layer *layers, int n, float mfp_range, int nseg, uint64_t nphotons,
                    uint64_t seed, double *refl, double *trans, double *tr, double *tt, uint64_t *events,
                    void *stream) {
    return guarded([&] {
        require(c && layers && refl && trans && tr && tt, "mpss_mc_profile: null argument");
        Context &ctx = *reinterpret_cast<Context *>(c);
        MPSS_HIP(hipSetDevice(ctx.config().device));
        static_assert(sizeof(mpss_layer) == sizeof(McLayer), "layer layout");
        const McScene sc = make_mc_scene(reinterpret_cast<const McLayer *>(layers), n, (double)mfp_range, nseg);
        run_mc_profile(sc, nphotons, seed, refl, trans, tr, tt, events, (hipStream_t)stream);
    });
}

int mpss_mc_reference(const mpss_layer *layers, int n, float mfp_range, int nseg, int lerp, double *refl,
                      double *trans, double *tr, double *tt) {
    return guarded([&] {
        require(layers && refl && trans && tr && tt, "mpss_mc_reference: null argument");
        require(n >= 1 && n <= 8 && nseg >= 1 && nseg <= (1 << 16), "mpss_mc_reference: bad layer or ring count");
        std::vector<MpcLayer> ml(n);
        double mfp_total = 0.;
        for (int i = 0; i < n; ++i) {
            require(layers[i].musp > 0.f && layers[i].mua >= 0.f && layers[i].thickness > 0.f,
                    "mpss_mc_reference: layers need musp > 0, mua >= 0, thickness > 0");
            ml[i] = MpcLayer{layers[i].mua, layers[i].musp, layers[i].ior, layers[i].thickness};
            mfp_total += 1. / (double)(layers[i].mua + layers[i].musp);  // Render, mcprofile.cpp:457-463
        }
        const double extent = mfp_range * (mfp_total / (double)n);
        mc_reference_profile(ml.data(), n, extent, nseg, lerp != 0, refl, trans, tr, tt);
    });
}

int mpss_host_tessellate(uint32_t nv, const float *P, const float *N, const float *S, const float *uv, uint32_t nt,
                         const int32_t *idx, const float *o2w, const float *w2o, int flip, uint32_t mat,
                         float min_dist, int incenter, void *rec, uint32_t *n) {
    return mpss_host_tessellate_bumped(nv, P, N, S, uv, nt, idx, o2w, w2o, flip, mat, min_dist, incenter, nullptr, rec,
                                       n);
}

int mpss_host_imagemap_lookup(const mpss_imagemap *t, uint32_t n, const float *uvd, float *out) {
    return guarded([&] {
        require(t && (n == 0 || (uvd && out)), "mpss_host_imagemap_lookup: null argument");
        const std::unique_ptr<ImageTexture> tex = build_imagemap(*t);
        for (uint32_t i = 0; i < n; ++i) {
            const float *a = uvd + 6 * (size_t)i;
            const UVDiff g{a[0], a[1], a[2], a[3], a[4], a[5]};
            tex_eval(tex->host, g, out + 3 * (size_t)i);
        }
    });
}

int mpss_host_tessellate_bumped(uint32_t nv, const float *P, const float *N, const float *S, const float *uv,
                                uint32_t nt, const int32_t *idx, const float *o2w, const float *w2o, int flip,
                                uint32_t mat, float min_dist, int incenter, const mpss_imagemap *bump, void *rec,
                                uint32_t *n) {
    return guarded([&] {
        require(P && idx && o2w && w2o && n && nv > 0 && min_dist > 0.f, "mpss_host_tessellate: bad argument");
        SceneData sd;
        Mesh m;
        m.P.assign(P, P + 3 * (size_t)nv);
        if (N) m.N.assign(N, N + 3 * (size_t)nv);
        if (S) m.S.assign(S, S + 3 * (size_t)nv);
        if (uv) m.uv.assign(uv, uv + 2 * (size_t)nv);
        m.idx.assign(idx, idx + 3 * (size_t)nt);
        for (int32_t v : m.idx) require(v >= 0 && (uint32_t)v < nv, "mpss_host_tessellate: index out of range");
        memcpy(m.o2w, o2w, sizeof(m.o2w));
        memcpy(m.w2o, w2o, sizeof(m.w2o));
        m.reverse_orientation = flip != 0;
        m.swaps_handedness = false;
        m.material = mat;
        sd.meshes.push_back(std::move(m));
        std::vector<SurfacePoint> pts;
        std::unique_ptr<ImageTexture> bt;
        std::vector<const TexView *> bv;
        if (bump) {
            require(bump->is_float != 0, "mpss_host_tessellate_bumped: the bumpmap is a float texture");
            bt = build_imagemap(*bump);
            bv.assign((size_t)mat + 1, nullptr);
            bv[mat] = &bt->host;
        }
        tessellate_surface_points(sd, min_dist, incenter != 0, pts, 0, bump ? bv.data() : nullptr);
        if (rec) {
            require(*n >= pts.size(), "mpss_host_tessellate: records buffer too small");
            memcpy(rec, pts.data(), pts.size() * sizeof(SurfacePoint));
        }
        *n = (uint32_t)pts.size();
    });
}

int mpss_host_from_rgb(const float *rgb, int illuminant, float *out) {
    return guarded([&] {
        require(rgb && out, "mpss_host_from_rgb: null argument");
        spectrum_from_rgb(rgb, illuminant != 0, out);
    });
}

int mpss_host_skin_layers(const mpss_layeredskin *m, float *mua, float *musp, float *thickness, float *eta) {
    return guarded([&] {
        require(m && mua && musp && thickness && eta, "mpss_host_skin_layers: null argument");
        SkinParams sp;
        sp.roughness = m->roughness;
        sp.nmperunit = m->nmperunit;
        sp.f_mel = m->f_mel;
        sp.f_eu = m->f_eu;
        sp.f_blood = m->f_blood;
        sp.f_ohg = m->f_ohg;
        for (int l = 0; l < 2; ++l) {
            sp.thickness_nm[l] = m->layer_thickness_nm[l];
            sp.ior[l] = m->layer_ior[l];
        }
        LayerParams lp;
        skin_layer_params(sp, lp);
        memcpy(mua, lp.mua, sizeof(lp.mua));
        memcpy(musp, lp.musp, sizeof(lp.musp));
        memcpy(thickness, lp.thickness, sizeof(lp.thickness));
        memcpy(eta, lp.eta, sizeof(lp.eta));
    });
}

int mpss_host_build_profile(const float *mua, const float *musp, const float *thickness, const float *eta,
                            int desired_length, int lerp, float *rd, uint32_t *length, float *rcp, float *total) {
    return guarded([&] {
        require(mua && musp && thickness && eta && length, "mpss_host_build_profile: null argument");
        require(desired_length >= 2 && desired_length <= 4096, "desired_length out of range");
        LayerParams lp;
        memcpy(lp.mua, mua, sizeof(lp.mua));
        memcpy(lp.musp, musp, sizeof(lp.musp));
        memcpy(lp.thickness, thickness, sizeof(lp.thickness));
        memcpy(lp.eta, eta, sizeof(lp.eta));
        ProfileTables pt;
        build_profile(lp, desired_length, lerp != 0, pt);
        *length = (uint32_t)pt.length;
        if (rd) memcpy(rd, pt.table.data(), sizeof(float) * pt.table.size());
        if (rcp) memcpy(rcp, pt.rcp, sizeof(pt.rcp));
        if (total) memcpy(total, pt.total_reflectance, sizeof(pt.total_reflectance));
    });
}

int mpss_host_dipole_rd(const float *sigma_a, const float *sigmap_s, float eta, uint32_t n, const float *d2, float *rd,
                        float *total) {
    return guarded([&] {
        require(sigma_a && sigmap_s && (n == 0 || (d2 && rd)), "mpss_host_dipole_rd: null argument");
        DipoleRd d;
        dipole_init(sigma_a, sigmap_s, eta, d);
        for (uint32_t i = 0; i < n; ++i) dipole_eval(d, d2[i], rd + (size_t)i * NB);
        if (total) dipole_total(d, total);
    });
}

int mpss_host_rho_table(float roughness, float eta, int fixed, int n, int sq, float *hd, float *hh) {
    return guarded([&] {
        require(hd && n >= 2 && sq >= 1, "mpss_host_rho_table: bad argument");
        RhoTable rt;
        build_rho_table(roughness, eta, fixed != 0, n, sq, rt);
        memcpy(hd, rt.hd.data(), sizeof(float) * n);
        if (hh) *hh = rt.hh;
    });
}

int mpss_host_octree_export(uint32_t n, const float *p, const float *nrm, const float *E, const float *area,
                            uint32_t *n_nodes, float *node_p, float *node_area, float *node_et, int32_t *depth,
                            int32_t *skip, int32_t *leaf_first, int32_t *leaf_count, int32_t *order) {
    return guarded([&] {
        require(p && nrm && E && area && n_nodes && n > 0, "mpss_host_octree_export: bad argument");
        FlatOctree t;
        build_octree((int)n, p, nrm, E, area, t);
        *n_nodes = (uint32_t)t.hdr.size();
        for (size_t i = 0; i < t.hdr.size(); ++i) {
            const NodeHdr &h = t.hdr[i];
            if (node_p) { node_p[3 * i] = h.px; node_p[3 * i + 1] = h.py; node_p[3 * i + 2] = h.pz; }
            if (node_area) node_area[i] = h.sum_area;
            if (node_et) memcpy(node_et + i * NB, &t.node_et[i * ROW], sizeof(float) * NB);
            if (depth) depth[i] = h.depth;
            if (skip) skip[i] = h.skip;
            if (leaf_first) leaf_first[i] = h.leaf_first;
            if (leaf_count) leaf_count[i] = h.leaf_count;
        }
        if (order) memcpy(order, t.pt_index.data(), sizeof(int32_t) * t.pt_index.size());
    });
}

}  // extern "C"
