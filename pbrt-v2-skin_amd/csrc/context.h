// context.h -- per-integrator state behind the C ABI (one mpss_ctx per
// MultipoleSubsurfaceIntegrator instance; reference integrators/multipolesubsurface.h:36-80).
#pragma once
#include <condition_variable>
#include <memory>
#include <mutex>
#include <vector>

#include "../../include/mpss.h"
#include "common.h"
#include "dipole.h"
#include "material.h"
#include "mo_kernel.h"
#include "octree.h"
#include "replay.h"
#include "scene.h"
#include "texture_build.h"

namespace mpss {

struct RenderScene;

struct Material {
    ProfileTables profile;
    RhoTable rho;
    float albedo[NB];
    float Kr[NB];              // Microfacet reflectance (layeredskin "Kr")
    float Kt[NB];              // MicrofacetTransmission transmittance (layeredskin "Kt")
    float roughness = 0.4f, ior = 1.4f;
    bool double_ref_sslf = false;
    bool is_monte_carlo = false;
    // "genprofile" false (layeredskin.cpp:70,120-122): no MultipoleBSSRDF data -- no Mo() term on its
    // surfaces, its irradiance points lit as points without a BSSRDF; the tables are a zero placeholder
    bool no_bssrdf = false;
    DeviceProfile dev_profile;
    DevBuf<float> dev_rho;  // [n_rho]
    int albedo_tex = -1, bump_tex = -1;  // ImageTexture ids ("texture albedo" / "texture bumpmap")
    // rgbprofile (ComputeRGBMultipoleProfile): Rd = FromRGB of three tables, Mo() in the
    // reference-order gather; dev_rgb [3][L] (rows 0..2 of profile.table), rgb_rcp their rcp
    bool rgb = false;
    DevBuf<float> dev_rgb, dev_rgb_rcp;
    float rgb_rcp[3] = {0.f, 0.f, 0.f};
    // a DiffusionReflectance functor instead of a profile (mpss_add_dipole_material): Mo only
    bool dipole = false;
    DipoleRd dip{};
    DevBuf<float> dev_dipole;  // [4][NB] zpos, zneg, sigma_tr, k
};

// ImageTexture<RGBSpectrum, Spectrum> / ImageTexture<float, float> (textures/imagemap.{h,cpp})
// with its UVMapping2D: the converted texels' MIPMap, on the host and (after upload) the device.
struct ImageTexture {
    HostPyramid py;
    int trilinear = 0;
    float max_aniso = 8.f, su = 1.f, sv = 1.f, du = 0.f, dv = 0.f;
    TexView host;  // over py.data
    DevBuf<float> dev;
    TexView device_view(const float *lut) const {
        TexView v = host;
        v.data = dev.ptr;
        v.lut = lut;
        return v;
    }
};
// ImageTexture::GetTexture's conversion + MIPMap (imagemap.cpp:55-84): texels through convertIn,
// or the one-valued map when the image could not be read (width == 0)
std::unique_ptr<ImageTexture> build_imagemap(const mpss_imagemap &m);

// Device workspace of one render_tiles (or mo_batch) call. Calls on different streams may run
// at once (pbrt calls Li from every worker thread), so each call takes a workspace of its own
// from the context's pool; `done` (recorded on the call's stream) orders a later user of the
// same workspace after the kernels of the previous one.
// Per-sample buffers (flags, slot, and the hit records primary_kernel writes: ha, hb, hs) are sized
// for the batch's camera samples; everything after the hit compaction (Mo() queries and results,
// direct-light terms, XYZ) for the batch's actual hit count, which render_tiles reads back once per
// batch.
struct RenderWorkspace {
    DevBuf<uint32_t> flags, hs, spill;
    DevBuf<int32_t> slot;
    DevBuf<int> count, work, perm;  // perm: the sharded gather's sorted query ids
    int64_t perm_n = 0;
    DevBuf<float4> q, mo, ha, hb, xyz, alb, frame, st;
    DevBuf<unsigned char> terms;
    DevBuf<float> ld;
    // reference-sampler replay: the batch's window table and the render tasks' stream cursors
    // (render.h ReplayCursors; valid for rp_key = {scene generation, spp, tasks})
    DevBuf<float> rp_table;
    DevBuf<uint32_t> rp_mt;
    DevBuf<int> rp_pix, rp_mti;
    uint64_t rp_key[3] = {~0ull, 0, 0};
    int64_t n = 0, rec_n = 0, hits = 0, tex_hits = 0, terms_n = 0, st_n = 0, px = 0;
    hipEvent_t done = nullptr;
    int device = 0;
    bool pending = false;
    ~RenderWorkspace();
};

class Context {
public:
    explicit Context(const mpss_config &cfg);
    ~Context();
    uint32_t add_layeredskin(const mpss_layeredskin &m);
    uint32_t set_material_tables(const float *rd, uint32_t len, const float *rcp, const float *rho, uint32_t n_rho,
                                 const float *albedo, bool is_mc);
    // the single-dipole Rd of the dipolesubsurface integrator (dipole.h); usable with mo_batch
    uint32_t add_dipole_material(const float *sigma_a, const float *sigmap_s, float eta);
    const Material &material(uint32_t id) const;
    void gather_info(uint32_t id, int *common_grid, float *rel_err, float *l1_err) const;
    void set_irradiance_points(int n, const float *p, const float *nrm, const float *E, const float *area);
    const DeviceOctree &octree() const;
    void export_octree(void *nodes, float *node_et, float *pt_hdr, float *pt_e, int32_t *pt_index);
    uint32_t add_imagemap(const mpss_imagemap &m);
    void set_material_textures(uint32_t material, int albedo, int bump);
    std::vector<const TexView *> host_bump_views() const;
    float max_error() const { return max_error_; }
    GatherOpts gather_opts() const {
        GatherOpts o;
        o.near_field = cfg_.mo_near_field;
        o.steal = cfg_.mo_work_stealing != 0;
        o.count_noprune = cfg_.count_traversal == 2;
        o.common_grid = cfg_.mo_common_grid != 0;
        return o;
    }
    const mpss_config &config() const { return cfg_; }

    // scene + per-pixel path (render_host.cpp)
    void add_mesh(uint32_t nv, const float *P, const float *N, const float *S, const float *uv, uint32_t nt,
                  const int32_t *idx, const float *o2w, const float *w2o, bool reverse, uint32_t material);
    void add_sphere_light(const float *c, float r, const float *Lemit, int nsamples);
    // texels: W x H RGB (nullable: no "mapname", the 1x1 map L.ToRGBSpectrum())
    void add_infinite_light(const float *L, int nsamples, const float *l2w, const float *w2l, int W = 0, int H = 0,
                            const float *texels = nullptr);
    void set_camera(const float *r2c, const float *c2w, int xres, int yres);
    void set_surface_points(uint32_t n, const SurfacePoint *pts);
    void preprocess(uint32_t seed);
    void tessellate_on_gpu();  // Preprocess point set, GPU build (render_host.hip)
    // FindPoissonPointDistribution (usepoissonpointfinder): fills points_ (render_host.hip)
    void find_poisson_points(uint32_t seed);
    void render_tiles(int spp, uint32_t seed, int n, const int32_t *rects, float *const *outs, hipStream_t stream);
    // the replay sampler's table (mpss_replay_samples); out may be null to query sizes
    void replay_samples(int spp, float *out, uint64_t *n_floats, int *k);
    void check_replay_lds(int spp, const char *who) const;  // replay_check_lds over the scene's lights
    // SubsurfaceOctreeNode::Mo over q device-resident points with material `mid`'s profile
    // (mpss_mo_batch); stream-ordered, safe for concurrent callers on their own streams
    void mo_batch(uint32_t mid, int q, const float *p_dev, float *out_dev, int32_t *counters_dev, hipStream_t stream);
    // Cost probe for tile dealing: one camera ray through every pixel centre; per rect, the rays
    // that hit a BSSRDF surface (sss) and any mesh surface (surf). Synchronous.
    void tile_costs(int n, const int32_t *rects, int64_t *sss, int64_t *surf);
    const std::vector<SurfacePoint> &surface_points() const { return points_; }
    const std::vector<float> &irradiance() const { return irradiance_; }
    bool has_octree() const { return have_octree_; }
    mpss_render_stats render_stats();
    void reset_render_stats();
    void set_instrumentation(bool timing, int counting) {
        std::lock_guard<std::mutex> g(mu_);
        cfg_.kernel_timing = timing;
        cfg_.count_traversal = counting;
    }

private:
    void activate() const;
    void upload_scene();
    RenderScene render_scene() const;
    int first_bssrdf_material() const;
    // reference-sampler replay (mpss_config.sampler): floats per camera sample in the window tables,
    // and the scene generation the workspaces' task cursors belong to (upload_scene bumps it)
    int replay_k_ = kReplayImage;
    uint64_t scene_gen_ = 0;
    // the window [x0, x1) x [y0, y1) of the sample extent at spp into ws->rp_table (the cursors in ws
    // reset when the scene, spp or task count changed); on `stream`
    // all_values: every sample's light-sample values (the whole table, replay_samples), not only those
    // of samples whose camera ray hits (all a render reads)
    void replay_window(RenderWorkspace *ws, const RenderScene &sc, int spp, int x0, int x1, int y0, int y1,
                       hipStream_t stream, bool all_values = false);
    SceneData scene_;
    bool scene_dirty_ = true, have_points_ = false;
    std::vector<SurfacePoint> points_;
    std::vector<float> irradiance_;
    DevBuf<BvhNode> d_bvh_;
    DevBuf<BvhNode> d_bvh_thread_;  // threaded copy (interior offset = end of subtree), any-hit walks
    DevBuf<TriRec> d_tris_;
    // reference sampler: the camera rays' candidate triangles per pixel (scene.h CameraBins)
    DevBuf<uint32_t> d_bin_off_;
    DevBuf<int32_t> d_bin_tri_, d_bin_all_;
    int bin_w_ = 0, bin_nall_ = 0;
    DevBuf<int32_t> d_tri_mesh_, d_tri_local_;
    std::vector<std::unique_ptr<DevBuf<float>>> d_mesh_bufs_;
    DevBuf<struct RenderMesh> d_meshes_;
    DevBuf<struct RenderLight> d_lights_;
    std::vector<std::unique_ptr<DevBuf<float>>> d_envmaps_;  // per infinite light (envmap.h layout)
    DevBuf<float> d_zero_map_;                                // stand-in map of area lights
    DevBuf<struct RenderMaterial> d_materials_;
    std::vector<std::unique_ptr<ImageTexture>> textures_;
    DevBuf<float> d_lut_;  // EWA weight table
    // workspace pool (render_tiles / mo_batch); guarded by mu_
    std::vector<std::unique_ptr<RenderWorkspace>> ws_free_;
    RenderWorkspace *acquire_ws();
    void release_ws(RenderWorkspace *ws, hipStream_t stream);
    hipError_t release_ws_nothrow(RenderWorkspace *ws, hipStream_t stream) noexcept;  // for unwinding paths
    // One in-flight call (inflight_ already counted under mu_): on every way out of the call, exceptions
    // included, its workspace returns to the pool and the count drops (so quiesce_locked never waits
    // for a call that has failed). mu_ must not be held when the guard dies.
    struct InflightGuard {
        Context *c;
        RenderWorkspace *ws;
        hipStream_t stream;
        void release() {  // the normal path: hands the workspace back, throwing on a HIP error
            RenderWorkspace *w = ws;
            ws = nullptr;
            if (w) c->release_ws(w, stream);
        }
        ~InflightGuard() {
            if (ws) (void)c->release_ws_nothrow(ws, stream);
            c->end_inflight();
        }
    };
    // every BSSRDF material's band layout exists on the device octree (mu_ held)
    void ensure_layouts();
    // p, nrm, E, area: host arrays; dp / dn / dE (nullable): the same on the device, when the caller
    // has them there already (Preprocess)
    void build_octree_locked(int n, const float *p, const float *nrm, const float *E, const float *area,
                             const float *dp = nullptr, const float *dn = nullptr, const float *dE = nullptr);
    // serializes everything that changes the context (scene, materials, octree, stats) and the
    // workspace pool; launches happen outside it
    mutable std::mutex mu_;
    // render_tiles / mo_batch calls between taking their device pointers (under mu_) and queueing
    // their last kernel; a call that replaces what they read (octree and band layouts, scene
    // buffers, replay table) first waits for none to be in flight, then for the queued kernels
    // (quiesce_locked). Guarded by mu_.
    int inflight_ = 0;
    std::condition_variable_any idle_;
    void quiesce_locked();
    void end_inflight();
    // kernel timing (cfg_.kernel_timing) and traversal counting (cfg_.count_traversal)
    struct Timed {
        hipEvent_t a, b;
        int kind;
    };
    std::vector<Timed> timed_;  // guarded by mu_
    void time_begin(bool on, hipStream_t s, hipEvent_t &a);
    void time_end(bool on, hipStream_t s, hipEvent_t a, int kind, std::vector<Timed> &out);
    mpss_render_stats stats_{};
    DevBuf<unsigned long long> d_counts_;  // [kStatStride * kGroups] traversal counts (mo_kernel.h)
    mpss_config cfg_;
    float max_error_, min_dist_;
    std::vector<std::unique_ptr<Material>> materials_;

    DeviceOctree dev_octree_;
    bool have_octree_ = false;
};

}  // namespace mpss
