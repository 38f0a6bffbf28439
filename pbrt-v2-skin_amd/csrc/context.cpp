// context.cpp -- Context implementation (material preparation, octree upload).
#include "context.h"

#include <cstring>

namespace mpss {

Context::Context(const mpss_config &cfg) : cfg_(cfg) {
    int ndev = 0;
    MPSS_HIP(hipGetDeviceCount(&ndev));
    if (cfg.device < 0 || cfg.device >= ndev)
        throw Error(MPSS_ERR_INVALID, "mpss_create: device ordinal " + std::to_string(cfg.device) +
                                          " out of range (" + std::to_string(ndev) + " HIP devices)");
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
    for (const Timed &t : timed_) {
        (void)hipEventDestroy(t.a);
        (void)hipEventDestroy(t.b);
    }
}

void Context::activate() const { MPSS_HIP(hipSetDevice(cfg_.device)); }

uint32_t Context::add_layeredskin(const mpss_layeredskin &m) {
    activate();
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
    if (cfg_.profile_on_host || sp.desired_length > 1024)
        build_profile(lp, sp.desired_length, sp.lerp_on_thin_slab, mat->profile);
    else
        build_profile_gpu(lp, sp.desired_length, sp.lerp_on_thin_slab, mat->profile);
    build_rho_table(sp.roughness, sp.ior[0], sp.double_ref_sslf, 1025, 256, mat->rho);
    memcpy(mat->albedo, m.albedo, sizeof(mat->albedo));
    memcpy(mat->Kr, m.Kr, sizeof(mat->Kr));
    memcpy(mat->Kt, m.Kt, sizeof(mat->Kt));
    mat->roughness = m.roughness;
    mat->ior = m.layer_ior[0];
    mat->double_ref_sslf = m.double_ref_sslf != 0;
    mat->dev_profile.upload(mat->profile.table.data(), mat->profile.length, mat->profile.rcp);
    mat->dev_rho.upload(mat->rho.hd.data(), mat->rho.hd.size());
    materials_.push_back(std::move(mat));
    return (uint32_t)materials_.size() - 1;
}

uint32_t Context::set_material_tables(const float *rd, uint32_t len, const float *rcp, const float *rho,
                                      uint32_t n_rho, const float *albedo, bool is_mc) {
    activate();
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
    mat->dev_profile.upload(mat->profile.table.data(), mat->profile.length, mat->profile.rcp);
    mat->dev_rho.upload(mat->rho.hd.data(), mat->rho.hd.size());
    materials_.push_back(std::move(mat));
    return (uint32_t)materials_.size() - 1;
}

const Material &Context::material(uint32_t id) const {
    if (id >= materials_.size()) throw Error(MPSS_ERR_INVALID, "unknown material id " + std::to_string(id));
    return *materials_[id];
}

void Context::set_irradiance_points(int n, const float *p, const float *nrm, const float *E, const float *area) {
    activate();
    build_octree(n, p, nrm, E, area, host_octree_);
    dev_octree_.upload(host_octree_);
    have_octree_ = true;
}

const DeviceOctree &Context::octree() const {
    if (!have_octree_) throw Error(MPSS_ERR_INVALID, "no irradiance points: call mpss_set_irradiance_points first");
    return dev_octree_;
}

}  // namespace mpss
