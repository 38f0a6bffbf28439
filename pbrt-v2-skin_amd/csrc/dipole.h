// dipole.h -- the classic single-dipole diffusion reflectance, pbrt-v2's DiffusionReflectance
// (reference src/integrators/diffusionutil.h:38-83, Jensen et al. 2001), host and device.
//
// It is the Rd functor the reference's dipolesubsurface integrator hands to the same
// SubsurfaceOctreeNode::Mo (src/integrators/dipolesubsurface.cpp:171-172). Here it backs
// "dipole" materials of mpss_mo_batch (mo_kernel.hip evaluates it per band inside the exact
// reference-order gather) and gives a closed-form Rd to pin the tabulated gathers against.
//
// Every product, quotient and sum is the reference's float operation in the reference's order
// (compile with -ffp-contract=off); exp is evaluated in double and rounded once, the render
// path's convention (pbrt_math.h), which the CPU oracle (oracle/octree.c) follows too.
#pragma once
#include "pbrt_math.h"

namespace mpss {

constexpr int kDipoleBands = 30;

// Fdr (src/core/reflection.h:64-71)
MPSS_HD float fdr(float eta) {
    if (eta >= 1) return -1.4399f / (eta * eta) + 0.7099f / eta + 0.6681f + 0.0636f * eta;
    return -0.4399f + .7099f / eta - .3319f / (eta * eta) + .0636f / (eta * eta * eta);
}

// DiffusionReflectance's data members, per band; `k` is the band's alphap / (4 M_PI), the first
// factor of operator() (a float quotient with pbrt's float M_PI, pbrt.h:196).
struct DipoleRd {
    float zpos[kDipoleBands], zneg[kDipoleBands], sigma_tr[kDipoleBands], k[kDipoleBands];
    float sigmap_t[kDipoleBands], A;
};

// DiffusionReflectance::DiffusionReflectance (diffusionutil.h:40-48)
inline void dipole_init(const float *sigma_a, const float *sigmap_s, float eta, DipoleRd &d) {
    d.A = (1.f + fdr(eta)) / (1.f - fdr(eta));
    const float zs = 1.f + (4.f / 3.f) * d.A;
    for (int c = 0; c < kDipoleBands; ++c) {
        const float st = sigma_a[c] + sigmap_s[c];
        d.sigmap_t[c] = st;
        d.sigma_tr[c] = sqrtf(sigma_a[c] * 3.f * st);
        const float alphap = sigmap_s[c] / st;
        d.zpos[c] = 1.f / st;
        d.zneg[c] = -d.zpos[c] * zs;
        d.k[c] = alphap / (4.f * kPiF);
    }
}

// DiffusionReflectance::operator() for one band (diffusionutil.h:49-58), Clamp(0, inf) included
MPSS_HD float dipole_band(float zpos, float zneg, float sigma_tr, float k, float d2) {
    const float dpos = sqrtf(d2 + zpos * zpos);
    const float dneg = sqrtf(d2 + zneg * zneg);
    const float pos = zpos * (dpos * sigma_tr + 1.f) * m_exp(-sigma_tr * dpos) / (dpos * dpos * dpos);
    const float neg = zneg * (dneg * sigma_tr + 1.f) * m_exp(-sigma_tr * dneg) / (dneg * dneg * dneg);
    const float rd = k * (pos - neg);
    return rd < 0.f ? 0.f : (rd > INFINITY ? INFINITY : rd);
}

inline void dipole_eval(const DipoleRd &d, float d2, float *out) {
    for (int c = 0; c < kDipoleBands; ++c) out[c] = dipole_band(d.zpos[c], d.zneg[c], d.sigma_tr[c], d.k[c], d2);
}

// DiffusionReflectance::TotalReflectance (diffusionutil.h:69-77): 1024-step Riemann sum in d^2
// over (4 mfp)^2
inline void dipole_total(const DipoleRd &d, float *out) {
    for (int c = 0; c < kDipoleBands; ++c) {
        const float mfp = 1.f / d.sigmap_t[c];
        const float step = (4.f * mfp) * (4.f * mfp) / 1024.f;
        float integral = 0.f;
        for (int i = 0; i < 1024; ++i)
            integral += dipole_band(d.zpos[c], d.zneg[c], d.sigma_tr[c], d.k[c], step * (float)i);
        out[c] = integral * step * kPiF;
    }
}

}  // namespace mpss
