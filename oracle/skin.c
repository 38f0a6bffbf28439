/* oracle/skin.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 * Restates SkinCoefficients (materials/skincoeffs.h:38-158, tables skincoeffs.cpp:35-73)
 * and the LayeredSkin layer-parameter setup (materials/layeredskin.cpp:39-89). */
#include <math.h>
#include "oracle.h"

#define WLD_N 61 /* core/material.h:96 */
static float wld_lambda(int i) { return 400.f + 5.f * (float)i; } /* material.cpp:117-125 */

static const float hb_oxy[WLD_N] = { /* skincoeffs.cpp:44-52 (oxy-hemoglobin, 400..700 nm step 5) */
    266200, 331450, 466800, 523100, 480400, 351100, 246100, 149050, 102600, 78880, 62820, 51525,
    44480, 38440, 33210, 29480, 26630, 24925, 23680, 22155, 20930, 20185, 20040, 20715, 24200,
    30885, 39960, 48335, 53240, 50985, 43020, 35650, 32610, 35210, 44500, 54425, 50100, 30620,
    14400, 6681.5f, 3200, 1958.5f, 1506, 1166.5f, 942, 740.8f, 610, 495.6f, 442, 397.7f, 368,
    340.3f, 319.6f, 305.6f, 294, 283.8f, 277.6f, 273.6f, 276, 280.6f, 290};
static const float hb_deoxy[WLD_N] = { /* skincoeffs.cpp:64-72 */
    223300, 261950, 304000, 353200, 407600, 471500, 528600, 549600, 413300, 259950, 103300,
    33435, 23390, 18700, 16160, 14920, 14550, 15375, 16680, 18650, 20860, 23285, 25770, 28680,
    31590, 35170, 39040, 42840, 46590, 50490, 53410, 54530, 53790, 49700, 45070, 40905, 37020,
    33590, 28320, 21185, 14680, 12040, 9444, 7553.5f, 6510, 5763.5f, 5149, 4666.5f, 4345,
    4026.5f, 3750, 3481.5f, 3227, 3011, 2795, 2591, 2408, 2224.5f, 2052, 1923.5f, 1794};

/* WLDValue::FromSampled, material.h:118-141 */
static void wld_from_sampled(const float *vals, float out[WLD_N]) {
    int idx = 0;
    float l0 = 0.f, l1 = wld_lambda(0), v0 = vals[0], v1 = vals[0];
    for (int i = 0; i < WLD_N; ++i) {
        float lam = wld_lambda(i);
        while (lam > l1 && idx < WLD_N - 1) {
            ++idx;
            l0 = l1;
            l1 = wld_lambda(idx);
            v0 = v1;
            v1 = vals[idx];
        }
        if (lam <= l1) {
            float t = (lam - l0) / (l1 - l0);
            out[i] = (1.f - t) * v0 + t * v1;
        } else
            out[i] = v1;
    }
}

static void to_bands(const float w[WLD_N], float out[O_NB]) {
    float lam[WLD_N];
    for (int i = 0; i < WLD_N; ++i) lam[i] = wld_lambda(i);
    o_from_sampled(lam, w, WLD_N, out);
}

void o_skin_layers(const o_skin_params *p, float mua[2][O_NB], float musp[2][O_NB],
                   float thickness[2], float eta[2]) {
    float base[WLD_N], eu[WLD_N], pheo[WLD_N], mie[WLD_N], ray[WLD_N];
    for (int i = 0; i < WLD_N; ++i) {
        float wl = wld_lambda(i);
        base[i] = 0.244f + 85.3f * expf(-(wl - 154.f) / 66.2f);
        eu[i] = 6.6e11f * powf(wl, -3.33f);
        pheo[i] = 2.9e15f * powf(wl, -4.75f);
        mie[i] = 147.4f * powf(wl, (float)-0.22);
        ray[i] = 2e12f * powf(wl, -4.f);
    }
    float oxy[WLD_N], deo[WLD_N];
    wld_from_sampled(hb_oxy, oxy);
    wld_from_sampled(hb_deoxy, deo);
    const float scale = p->nmperunit / 1e7f; /* layeredskin.cpp:47,51 */
    float epi_a[WLD_N], epi_s[WLD_N], der_a[WLD_N], der_s[WLD_N];
    const float kblood = 2.303f / 64500.f * 150.f;
    for (int i = 0; i < WLD_N; ++i) {
        float a = eu[i] * p->f_eu + pheo[i] * (1 - p->f_eu);
        epi_a[i] = (a * p->f_mel + base[i] * (1 - p->f_mel)) * scale;
        float sp = ray[i] + mie[i];
        epi_s[i] = sp * scale;
        float blood = (oxy[i] * p->f_ohg + deo[i] * (1.f - p->f_ohg)) * kblood;
        der_a[i] = (blood * p->f_blood + base[i] * (1 - p->f_blood)) * scale;
        der_s[i] = (sp * 0.5f) * scale;
    }
    to_bands(epi_a, mua[0]);
    to_bands(epi_s, musp[0]);
    to_bands(der_a, mua[1]);
    to_bands(der_s, musp[1]);
    thickness[0] = p->layer_thickness_nm[0] / p->nmperunit;
    thickness[1] = p->layer_thickness_nm[1] / p->nmperunit;
    eta[0] = p->layer_ior[0];
    eta[1] = p->layer_ior[1];
}
