// context.h -- per-integrator state behind the C ABI (one mpss_ctx per
// MultipoleSubsurfaceIntegrator instance; reference integrators/multipolesubsurface.h:36-80).
#pragma once
#include <memory>
#include <vector>

#include "../../include/mpss.h"
#include "common.h"
#include "material.h"
#include "mo_kernel.h"
#include "octree.h"
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
    DeviceProfile dev_profile;
    DevBuf<float> dev_rho;  // [n_rho]
    int albedo_tex = -1, bump_tex = -1;  // ImageTexture ids ("texture albedo" / "texture bumpmap")
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

class Context {
public:
    explicit Context(const mpss_config &cfg);
    ~Context();
    uint32_t add_layeredskin(const mpss_layeredskin &m);
    uint32_t set_material_tables(const float *rd, uint32_t len, const float *rcp, const float *rho, uint32_t n_rho,
                                 const float *albedo, bool is_mc);
    const Material &material(uint32_t id) const;
    void set_irradiance_points(int n, const float *p, const float *nrm, const float *E, const float *area);
    const DeviceOctree &octree() const;
    uint32_t add_imagemap(const mpss_imagemap &m);
    void set_material_textures(uint32_t material, int albedo, int bump);
    std::vector<const TexView *> host_bump_views() const;
    float max_error() const { return max_error_; }
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
    // FindPoissonPointDistribution (usepoissonpointfinder): fills points_ (render_host.hip)
    void find_poisson_points(uint32_t seed);
    void render_tiles(int spp, uint32_t seed, int n, const int32_t *rects, float *const *outs, hipStream_t stream);
    const std::vector<SurfacePoint> &surface_points() const { return points_; }
    const std::vector<float> &irradiance() const { return irradiance_; }
    bool has_octree() const { return have_octree_; }
    mpss_render_stats render_stats();
    void reset_render_stats();
    void set_instrumentation(bool timing, bool counting) {
        cfg_.kernel_timing = timing;
        cfg_.count_traversal = counting;
    }

private:
    void activate() const;
    void upload_scene();
    RenderScene render_scene() const;
    int first_bssrdf_material() const;
    SceneData scene_;
    bool scene_dirty_ = true, have_points_ = false;
    std::vector<SurfacePoint> points_;
    std::vector<float> irradiance_;
    DevBuf<BvhNode> d_bvh_;
    DevBuf<TriRec> d_tris_;
    DevBuf<int32_t> d_tri_mesh_, d_tri_local_;
    std::vector<std::unique_ptr<DevBuf<float>>> d_mesh_bufs_;
    DevBuf<struct RenderMesh> d_meshes_;
    DevBuf<struct RenderLight> d_lights_;
    std::vector<std::unique_ptr<DevBuf<float>>> d_envmaps_;  // per infinite light (envmap.h layout)
    DevBuf<float> d_zero_map_;                                // stand-in map of area lights
    DevBuf<struct RenderMaterial> d_materials_;
    std::vector<std::unique_ptr<ImageTexture>> textures_;
    DevBuf<float> d_lut_;  // EWA weight table
    DevBuf<float4> ws_alb_, ws_frame_;  // per hit: albedo lookup, bumped frame (textured scenes)
    int64_t ws_tex_hits_ = 0;
    // render workspace: per camera sample (flags, slot) and per surface hit (ld, Mo query, Mo)
    DevBuf<uint32_t> ws_flags_;
    DevBuf<int32_t> ws_slot_;
    DevBuf<int> ws_count_;
    DevBuf<float4> ws_q_, ws_mo_, ws_ha_, ws_hb_, ws_xyz_;
    DevBuf<uint32_t> ws_hs_, ws_spill_;
    DevBuf<unsigned char> ws_terms_;
    int64_t ws_terms_n_ = 0;
    DevBuf<float4> ws_st_;  // infinite lights: radiance-map coordinates per direct-light lane
    int64_t ws_st_n_ = 0;
    int64_t ws_px_ = 0;
    DevBuf<float> ws_ld_;
    int64_t ws_n_ = 0, ws_hits_ = 0;
    // kernel timing (cfg_.kernel_timing) and traversal counting (cfg_.count_traversal)
    struct Timed {
        hipEvent_t a, b;
        int kind;
    };
    std::vector<Timed> timed_;
    void time_begin(hipStream_t s, hipEvent_t &a);
    void time_end(hipStream_t s, hipEvent_t a, int kind);
    mpss_render_stats stats_{};
    DevBuf<unsigned long long> d_counts_;  // [2 * kGroups]: nodes, points per band group
    mpss_config cfg_;
    float max_error_, min_dist_;
    std::vector<std::unique_ptr<Material>> materials_;
    FlatOctree host_octree_;
    DeviceOctree dev_octree_;
    bool have_octree_ = false;
};

}  // namespace mpss
