// material.h -- LayeredSkin material preparation (host side).
//
// Follows the reference's parse-time precompute for `Material "layeredskin"`:
//   CreateLayeredSkinMaterial / LayeredSkin::LayeredSkin  (src/materials/layeredskin.cpp:39-123, 222-262)
//   SkinCoefficients                                       (src/materials/skincoeffs.h:38-158)
//   ComputeMultipoleProfile -> MultipoleProfileTask::Run   (src/core/multipole.cpp:241-295, 371-406)
//   MPC_ComputeDiffusionProfile + resample                 (MultipoleProfileCalculator.cpp:151-426)
//   ComputeRhoDataFromBxDF                                 (src/core/multipole.cpp:466-549)
// The product's Rd table is channel-major: table[c * length + k].
#pragma once
#include <vector>
#include "common.h"

namespace mpss {

struct SkinParams {
    float roughness = 0.4f, nmperunit = 100e6f;
    float f_mel = 0.15f, f_eu = 1.f, f_blood = 0.002f, f_ohg = 0.3f;
    float thickness_nm[2] = {0.25e6f, 20e6f};
    float ior[2] = {1.4f, 1.4f};
    int desired_length = 512;
    bool lerp_on_thin_slab = true;
    bool double_ref_sslf = false;
};

struct LayerParams {
    float mua[2][NB], musp[2][NB], thickness[2], eta[2];
};

struct ProfileTables {
    int length = 0;                   // entries per channel (resampled)
    std::vector<float> table;         // [NB][length]
    float rcp[NB], spacing[NB], total_reflectance[NB];
};

struct RhoTable {
    std::vector<float> hd;  // [n] scalar rho_hd(cos theta) (all channels equal for this BxDF)
    float hh = 0.f;
};

void skin_layer_params(const SkinParams &p, LayerParams &out);
// distinct: channels 0..distinct-1 are built and channel c >= distinct copies channel c % distinct
// (rgbprofile: lp's band c already holds component c % 3, so 3 builds give all 30 rows)
void build_profile(const LayerParams &lp, int desired_length, bool lerp_on_thin_slab, ProfileTables &out,
                   int nthreads = 0, int distinct = NB);
// The same profile built on the current HIP device (profile_gpu.hip); out is filled on the host.
void build_profile_gpu(const LayerParams &lp, int desired_length, bool lerp_on_thin_slab, ProfileTables &out,
                       hipStream_t stream = 0, int distinct = NB);
// The same rho_hd table on the current HIP device (rho_gpu.hip): bit-identical to build_rho_table
// (one MT19937 stream per entry, terms Kahan-summed in sample order); rho_hh on the host.
void build_rho_table_gpu(float roughness, float eta, bool fixed_fresnel, int n_entries, int sqrt_samples,
                         RhoTable &out, hipStream_t stream = 0);
// ComputeRhoHHFromBxDF (multipole.cpp:466-480)
float rho_hh(float roughness, float eta, bool fixed_fresnel, int sqrt_samples);
// LayeredSkin "showirradiancepoints": ComputeIrradiancePointsProfile(radius) (multipole.cpp:551-567) --
// every band the two-entry table {1 / area, 1 / area}, area = (float)(M_PI * r * r), dsqSpacing = r * r,
// so Rd(d^2) = 1 / area for d < r and 0 beyond -- and ComputeRoughRhoData (:569-572): rho_hd = {0, 0}.
void irradiance_points_profile(float radius, ProfileTables &p, RhoTable &rho);
void build_rho_table(float roughness, float eta, bool fixed_fresnel, int n_entries, int sqrt_samples,
                     RhoTable &out, int nthreads = 0);

// MPC_LayerSpec (MultipoleProfileCalculator.h; g_HG unused by the multipole code)
struct MpcLayer {
    float mua, musp, ior, thickness;
};
struct MpcOutput {  // MPC_Output before resampling: the unique-d^2 samples
    std::vector<float> dsq, refl, trans;
    float total_reflectance = 0.f, total_transmittance = 0.f;
};
void mpc_compute(const MpcLayer *layers, int n, float step, int desired_length, bool lerp_on_thin_slab,
                 MpcOutput &out);
void mpc_resample_distribution(const MpcOutput &in, int n, const float *points, float *refl, float *trans);
// MultipoleReferenceTask (mcprofile.cpp:381-425): ring-centre profile of the layers' multipole model
void mc_reference_profile(const MpcLayer *layers, int n, double extent, int nsegments, bool lerp_on_thin_slab,
                          double *refl, double *trans, double *total_r, double *total_t);

// ComputeMonteCarloProfile's ring -> table conversion (multipole.cpp:328-355) for one band
void profile_from_rings(const double *refl, int nseg, double extent, int target, std::vector<float> &table,
                        float &rcp, float &spacing);
// usemontecarlo (multipole.cpp:298-368): per band, a GPU random walk of `photons` photons over
// 4096 rings within 12 mean free paths, resampled to 65536 entries uniform in d^2 (mc_profile.hip)
void build_profile_mc(const LayerParams &lp, uint64_t photons, uint64_t seed, ProfileTables &out);

}  // namespace mpss
