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

namespace mpss {

struct Material {
    ProfileTables profile;
    RhoTable rho;
    float albedo[NB];
    bool is_monte_carlo = false;
    DeviceProfile dev_profile;
    DevBuf<float> dev_rho;  // [n_rho]
};

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
    float max_error() const { return max_error_; }
    const mpss_config &config() const { return cfg_; }

private:
    void activate() const;
    mpss_config cfg_;
    float max_error_, min_dist_;
    std::vector<std::unique_ptr<Material>> materials_;
    FlatOctree host_octree_;
    DeviceOctree dev_octree_;
    bool have_octree_ = false;
};

}  // namespace mpss
