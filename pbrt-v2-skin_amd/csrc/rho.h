// rho.h -- the LayeredSkin rho_hd table's per-sample term, host and device.
//
// ComputeRhoDataFromBxDF / RhoTask (reference src/core/multipole.cpp:488-549) estimate, for
// 1025 values of cos(theta_o), BxDF::rho(wo) (core/reflection.cpp:623-652) of
// Microfacet(R = 1, (Fixed)FresnelDielectric(1, eta), Beckmann(roughness))
// (materials/layeredskin.cpp:104-109) from 256^2 stratified samples (StratifiedSample2D,
// montecarlo.cpp:158-168) jittered by MT19937 seeded 6428263 * entry (core/rng.cpp), summed
// in sample order with Kahan compensation. The estimator's term for one sample is
//   Sample_f(wo, u1, u2) * |cos(theta_i)| / pdf   when pdf > 0 (skipped otherwise),
// with Microfacet::Sample_f (reflection.cpp:391-397) = Beckmann::Sample_f (:548-570) + the
// same-hemisphere test + Microfacet::f (:228-240). The functions are geom.h's render-path
// ones, so the table and the render's BSDF are one implementation.
#pragma once
#include "geom.h"

namespace mpss {

constexpr uint32_t kRhoSeed = 6428263u;  // RhoTask::Run's RNG(6428263 * id)

// cos(theta_o) of table entry id (ComputeRhoDataFromBxDF: id / 1024, 0 -> 0.01 / 1024)
MPSS_HD float rho_costheta(int id, int n_entries) {
    float ct = (float)id / (float)(n_entries - 1);
    if (ct == 0.f) ct = 0.01f / (float)(n_entries - 1);
    return ct;
}

// wo = SphericalDirection(sqrtf(1 - ct^2), ct, 0) (geometry.h)
MPSS_HD V3 rho_wo(float ct) {
    const float st = sqrtf(1 - ct * ct);
    return V3{st * m_cos(0.f), st * m_sin(0.f), ct};
}

// One stratified sample (x, y) of an n x n grid with MT jitters jx, jy (StratifiedSample2D)
MPSS_HD void rho_stratum(int x, int y, int n, float jx, float jy, float &u1, float &u2) {
    const float d = 1.f / (float)n;
    const float a = ((float)x + jx) * d, b = ((float)y + jy) * d;
    u1 = a < kOneMinusEps ? a : kOneMinusEps;
    u2 = b < kOneMinusEps ? b : kOneMinusEps;
}

// The estimator term of one sample; false when pdf <= 0 (the sample adds nothing)
MPSS_HD bool rho_term(const Microfacet &m, V3 wo, float u1, float u2, float &term) {
    V3 wi;
    float pdf = 0.f;
    beckmann_sample(m, wo, u1, u2, wi, pdf);
    float f = 0.f;
    if (wo.z * wi.z > 0.f) {
        const MfTerms t = microfacet_terms(m, wo, wi);
        if (!t.zero) f = 1.f * t.D * t.G * t.F / t.den;
    }
    if (!(pdf > 0.f)) return false;
    term = f * fabsf(wi.z) / pdf;
    return true;
}

// KahanSum (the fork's core/kahansum.h): y = v - c; t = sum + y; c = (t - sum) - y; sum = t
struct KahanF {
    float sum = 0.f, c = 0.f;
    MPSS_HD void add(float v) {
        const float y = v - c, t = sum + y;
        c = (t - sum) - y;
        sum = t;
    }
};

MPSS_HD Microfacet rho_bxdf(float roughness, float eta, bool fixed) {
    Microfacet m;
    const float rms = roughness < 1e-3f ? 1e-3f : roughness;
    m.rms2 = rms * rms;
    m.rcp_rms2 = 1 / m.rms2;
    m.eta = eta;
    m.fixed_fresnel = fixed ? 1 : 0;
    return m;
}

}  // namespace mpss
