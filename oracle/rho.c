/* oracle/rho.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 * Restates the LayeredSkin rho_hd table: ComputeRhoDataFromBxDF / RhoTask
 * (src/core/multipole.cpp:466-549) over Microfacet(R=1, FresnelDielectric(1,eta),
 * Beckmann(roughness)) (materials/layeredskin.cpp:104-109), i.e. BxDF::rho
 * (core/reflection.cpp:623-652) with Microfacet::Sample_f/f (reflection.cpp:228-240,
 * 391-397), Beckmann::D/Sample_f (reflection.h:507-529, reflection.cpp:548-570),
 * FresnelDielectric::Evaluate + FrDiel (reflection.cpp:62-84,132-153) -- or, with LayeredSkin's
 * "doublerefsslf", FixedFresnelDielectric (reflection.h:315-324; layeredskin.cpp:105) --, KahanSum
 * (core/kahansum.h), StratifiedSample2D (montecarlo.cpp:158-168) and MT19937
 * (core/rng.cpp).  All channels of this BxDF are equal (R=1, spectrally flat
 * Fresnel), so the table is computed as scalars and replicated. */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

#define O_PIF 3.14159265358979323846f   /* pbrt.h:196 (float literal) */
#define O_INV_TWOPI 0.15915494309189533577f
static const float ONE_M_EPS = 0x1.fffffep-1f; /* montecarlo.h:48-50 */

/* ---- MT19937, rng.cpp ---- */
typedef o_mt mt_rng;
void o_mt_seed(mt_rng *r, uint32_t s) {
    r->mt[0] = s;
    for (r->mti = 1; r->mti < 624; r->mti++)
        r->mt[r->mti] = (1812433253u * (r->mt[r->mti - 1] ^ (r->mt[r->mti - 1] >> 30)) + (uint32_t)r->mti);
}
uint32_t o_mt_u32(mt_rng *r) {
    static const uint32_t mag01[2] = {0x0u, 0x9908b0dfu};
    uint32_t y;
    if (r->mti >= 624) {
        int kk;
        for (kk = 0; kk < 624 - 397; kk++) {
            y = (r->mt[kk] & 0x80000000u) | (r->mt[kk + 1] & 0x7fffffffu);
            r->mt[kk] = r->mt[kk + 397] ^ (y >> 1) ^ mag01[y & 1u];
        }
        for (; kk < 623; kk++) {
            y = (r->mt[kk] & 0x80000000u) | (r->mt[kk + 1] & 0x7fffffffu);
            r->mt[kk] = r->mt[kk + (397 - 624)] ^ (y >> 1) ^ mag01[y & 1u];
        }
        y = (r->mt[623] & 0x80000000u) | (r->mt[0] & 0x7fffffffu);
        r->mt[623] = r->mt[396] ^ (y >> 1) ^ mag01[y & 1u];
        r->mti = 0;
    }
    y = r->mt[r->mti++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}
static float mt_float(mt_rng *r) { return (float)(o_mt_u32(r) & 0xffffff) / (float)(1 << 24); }

uint32_t o_mt_first(uint32_t seed, int n, uint32_t *out) {
    mt_rng r;
    o_mt_seed(&r, seed);
    for (int i = 0; i < n; ++i) out[i] = o_mt_u32(&r);
    return n > 0 ? out[0] : 0;
}

static void stratified2d(float *s, int nx, int ny, mt_rng *r) {
    float dx = 1.f / nx, dy = 1.f / ny;
    for (int y = 0; y < ny; ++y)
        for (int x = 0; x < nx; ++x) {
            float jx = mt_float(r), jy = mt_float(r);
            float a = (x + jx) * dx, b = (y + jy) * dy;
            *s++ = a < ONE_M_EPS ? a : ONE_M_EPS;
            *s++ = b < ONE_M_EPS ? b : ONE_M_EPS;
        }
}

/* Transcendentals: evaluated in double and rounded once to float, the convention the product
 * shares with this oracle on host and device (pbrt_math.h); the reference calls float libm. */
static float fe(float x) { return (float)exp((double)x); }
static float fl(float x) { return (float)log((double)x); }
static float fat(float x) { return (float)atan((double)x); }
static float fc(float x) { return (float)cos((double)x); }
static float fs(float x) { return (float)sin((double)x); }

typedef struct { float x, y, z; } v3;
static float dot3(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

typedef struct { float rms2, rcp_rms2, eta; int fixed; } mf;

static float beck_d(const mf *m, v3 wh) { /* reflection.h:514-521 */
    float ct = fabsf(wh.z);
    float c2 = ct * ct;
    float d = c2 * c2 * O_PIF;
    if (d == 0.f) return 0.f;
    float e = (c2 - 1) * m->rcp_rms2 / c2;
    return m->rcp_rms2 * fe(e) / d;
}

static float fresnel_diel(float cosi, float eta_i, float eta_t) { /* reflection.cpp:132-153 */
    cosi = cosi < -1.f ? -1.f : cosi > 1.f ? 1.f : cosi;
    int entering = cosi > 0.;
    float ei = eta_i, et = eta_t;
    if (!entering) { float t = ei; ei = et; et = t; }
    float x = 1.f - cosi * cosi;
    float sint = ei / et * sqrtf(x > 0.f ? x : 0.f);
    if (sint >= 1.) return 1.f;
    float y = 1.f - sint * sint;
    float cost = sqrtf(y > 0.f ? y : 0.f);
    float ci = fabsf(cosi);
    float rparl = ((et * ci) - (ei * cost)) / ((et * ci) + (ei * cost));
    float rperp = ((ei * ci) - (et * cost)) / ((ei * ci) + (et * cost));
    return (rparl * rparl + rperp * rperp) / 2.f;
}

static float mf_G(v3 wo, v3 wi, v3 wh) { /* reflection.h:430-437 */
    float nwh = fabsf(wh.z), nwo = fabsf(wo.z), nwi = fabsf(wi.z);
    float wowh = fabsf(dot3(wo, wh));
    float a = 2.f * nwh * nwo / wowh, b = 2.f * nwh * nwi / wowh;
    float m = a < b ? a : b;
    return 1.f < m ? 1.f : m;
}

static float mf_f(const mf *m, v3 wo, v3 wi) { /* reflection.cpp:228-240 with R = 1 */
    float cto = fabsf(wo.z), cti = fabsf(wi.z);
    if (cti == 0.f || cto == 0.f) return 0.f;
    v3 wh = {wi.x + wo.x, wi.y + wo.y, wi.z + wo.z};
    if (wh.x == 0. && wh.y == 0. && wh.z == 0.) return 0.f;
    float inv = 1.f / sqrtf(wh.x * wh.x + wh.y * wh.y + wh.z * wh.z);
    wh.x *= inv; wh.y *= inv; wh.z *= inv;
    float cth = dot3(wi, wh);
    float F = fresnel_diel(cth, 1.f, m->eta);
    if (m->fixed) F = F + (F * (1.f - F)) * (1.f - F); /* FixedFresnelDielectric: val + val (1 - val)(1 - val) */
    return 1.f * beck_d(m, wh) * mf_G(wo, wi, wh) * F / (4.f * cti * cto);
}

/* Beckmann::Sample_f (reflection.cpp:548-570) + Microfacet::Sample_f (:391-397) */
static float mf_sample_f(const mf *m, v3 wo, v3 *wi, float u1, float u2, float *pdf) {
    float theta = fat(sqrtf(-m->rms2 * fl(1.f - u1)));
    float ct = fc(theta), st = fs(theta);
    float phi = u2 * 2.f * O_PIF;
    v3 wh = {st * fc(phi), st * fs(phi), ct};
    if (!(wo.z * wh.z > 0.f)) { wh.x = -wh.x; wh.y = -wh.y; wh.z = -wh.z; }
    float d = dot3(wo, wh);
    wi->x = -wo.x + 2.f * d * wh.x;
    wi->y = -wo.y + 2.f * d * wh.y;
    wi->z = -wo.z + 2.f * d * wh.z;
    float bp = beck_d(m, wh) * ct / (4.f * dot3(wo, wh));
    if (dot3(wo, wh) <= 0.f || bp < 1e-20f) bp = 0.f;
    *pdf = bp;
    if (!(wo.z * wi->z > 0.f)) return 0.f;
    return mf_f(m, wo, *wi);
}

typedef struct {
    mf m;
    int sqrt_samples, n_entries, next;
    float *hd;
    pthread_mutex_t mu;
} rho_job;

static float rho_entry(const rho_job *j, int id) { /* RhoTask::Run, multipole.cpp:506-518 */
    mt_rng r;
    o_mt_seed(&r, (uint32_t)(6428263u * (uint32_t)id));
    int n = j->sqrt_samples * j->sqrt_samples;
    float *s = (float *)malloc(sizeof(float) * 2 * n);
    stratified2d(s, j->sqrt_samples, j->sqrt_samples, &r);
    float ct = (float)id / (float)(j->n_entries - 1);
    if (ct == 0.f) ct = 0.01f / (float)(j->n_entries - 1);
    v3 wo = {sqrtf(1 - ct * ct) * fc(0.f), sqrtf(1 - ct * ct) * fs(0.f), ct};
    float sum = 0.f, c = 0.f; /* KahanSum<Spectrum>, one channel */
    for (int i = 0; i < n; ++i) {
        v3 wi;
        float pdf = 0.f;
        float f = mf_sample_f(&j->m, wo, &wi, s[2 * i], s[2 * i + 1], &pdf);
        if (pdf > 0.) {
            float v = f * fabsf(wi.z) / pdf;
            float y = v - c, t = sum + y;
            c = (t - sum) - y;
            sum = t;
        }
    }
    free(s);
    return sum / (float)n;
}

static void *rho_worker(void *arg) {
    rho_job *j = (rho_job *)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        int id = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (id >= j->n_entries) break;
        j->hd[id] = rho_entry(j, id);
    }
    return NULL;
}

/* ComputeRhoHHFromBxDF (multipole.cpp:466-480) with BxDF::rho(nSamples, s1, s2) (reflection.cpp:637-652) */
static float rho_hh(const mf *m, int sq) {
    mt_rng r;
    o_mt_seed(&r, (uint32_t)(6428263u * 3u * 7u));
    int n = sq * sq;
    float *s1 = (float *)malloc(sizeof(float) * 2 * n), *s2 = (float *)malloc(sizeof(float) * 2 * n);
    stratified2d(s1, sq, sq, &r);
    stratified2d(s2, sq, sq, &r);
    float sum = 0.f, c = 0.f;
    for (int i = 0; i < n; ++i) {
        /* UniformSampleHemisphere, montecarlo.cpp:268-276 */
        float z = s1[2 * i];
        float rr = sqrtf(fmaxf(0.f, 1.f - z * z));
        float phi = 2 * O_PIF * s1[2 * i + 1];
        v3 wo = {rr * fc(phi), rr * fs(phi), z}, wi;
        float pdf_o = O_INV_TWOPI, pdf_i = 0.f;
        float f = mf_sample_f(m, wo, &wi, s2[2 * i], s2[2 * i + 1], &pdf_i);
        if (pdf_i > 0.) {
            float v = f * fabsf(wi.z) * fabsf(wo.z) / (pdf_o * pdf_i);
            float y = v - c, t = sum + y;
            c = (t - sum) - y;
            sum = t;
        }
    }
    free(s1);
    free(s2);
    return sum / (O_PIF * n);
}

void o_rho_table(float roughness, float eta, int n_entries, int sqrt_samples, int nthreads, float *hd, float *hh) {
    o_rho_table_ex(roughness, eta, 0, n_entries, sqrt_samples, nthreads, hd, hh);
}

void o_rho_table_ex(float roughness, float eta, int fixed, int n_entries, int sqrt_samples, int nthreads, float *hd,
                    float *hh) {
    rho_job j;
    memset(&j, 0, sizeof(j));
    float rms = roughness < 1e-3f ? 1e-3f : roughness; /* Beckmann ctor, reflection.h:509-513 */
    j.m.rms2 = rms * rms;
    j.m.rcp_rms2 = 1 / j.m.rms2;
    j.m.eta = eta;
    j.m.fixed = fixed;
    j.sqrt_samples = sqrt_samples;
    j.n_entries = n_entries;
    j.hd = hd;
    pthread_mutex_init(&j.mu, NULL);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    pthread_t th[64];
    for (int i = 0; i < nthreads; ++i) pthread_create(&th[i], NULL, rho_worker, &j);
    for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
    pthread_mutex_destroy(&j.mu);
    if (hh) *hh = rho_hh(&j.m, sqrt_samples);
}
