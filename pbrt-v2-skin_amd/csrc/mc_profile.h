// mc_profile.h -- Monte-Carlo layered random-walk profile (MonteCarloProfileRenderer,
// reference src/renderers/mcprofile.cpp:120-341, 443-533): photons enter a stack of plane-
// parallel layers at the origin, random-walk in double precision with Fresnel interfaces and
// Russian roulette, and are tallied by exit radius into reflectance / transmittance rings.
#pragma once
#include <cstdint>

#include "common.h"
#include "pbrt_math.h"

namespace mpss {

constexpr int kMcMaxLayers = 8;

struct McLayer {  // core/layer.h:35-46 (float fields, as FindLayer stores them)
    float mua, musp, ior, thickness;
};

struct McScene {  // MiniScene (mcprofile.cpp:142-193)
    int nlayers;
    McLayer layer[kMcMaxLayers];
    double depth[kMcMaxLayers + 1];  // interface depths: 0, d0, d0 + d1, ...
    double extent;                   // mfpRange * mean mfp
    int nsegments;
    // per-layer constants of the walk, divided once on the host (the same IEEE double quotients)
    double mfp[kMcMaxLayers];     // 1 / musp
    double eta_dn[kMcMaxLayers];  // ior / ior of the layer below (1 past the last), the ray going down
    double eta_up[kMcMaxLayers];  // ior / ior of the layer above (1 above the first), the ray going up
};

// Per-photon random stream ("replay mode"): splitmix64 seeded from (seed, photon),
// 53-bit doubles in [0, 1). Host (oracle) and device draw identical sequences.
MPSS_HD uint64_t mc_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
struct McRng {
    uint64_t s;
    MPSS_HD void init(uint64_t seed, uint64_t photon) { s = mc_mix64(seed * 0x9e3779b97f4a7c15ull ^ mc_mix64(photon)); }
    MPSS_HD double next() {
        s += 0x9e3779b97f4a7c15ull;
        return (double)(mc_mix64(s) >> 11) * 0x1p-53;
    }
};

// mfp_range * mean mfp over layers = the tally extent (Render, mcprofile.cpp:460-467).
McScene make_mc_scene(const McLayer *layers, int n, double mfp_range, int nsegments);
// Trace nphotons; refl / trans receive the ring-normalised profiles [nsegments], totals the
// tallied fractions (photons exiting within the extent), events the free-flight count.
void run_mc_profile(const McScene &sc, uint64_t nphotons, uint64_t seed, double *refl, double *trans,
                    double *total_r, double *total_t, uint64_t *events, hipStream_t stream);

}  // namespace mpss
