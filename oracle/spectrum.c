/* oracle/spectrum.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 * Restates pbrt's 30-band SampledSpectrum helpers used on the hot path. */
#include "oracle.h"
#include "../data/spectral_bands.h"

static float o_lerpf(float t, float a, float b) { return (1.f - t) * a + t * b; }

/* spectrum.cpp:60-94 */
float o_average_spectrum_samples(const float *lambda, const float *vals, int n, float l0, float l1) {
    if (l1 <= lambda[0]) return vals[0];
    if (l0 >= lambda[n - 1]) return vals[n - 1];
    if (n == 1) return vals[0];
    float sum = 0.f;
    if (l0 < lambda[0]) sum += vals[0] * (lambda[0] - l0);
    if (l1 > lambda[n - 1]) sum += vals[n - 1] * (l1 - lambda[n - 1]);
    int i = 0;
    while (l0 > lambda[i + 1]) ++i;
    for (; i + 1 < n && l1 >= lambda[i]; ++i) {
        float s0 = l0 > lambda[i] ? l0 : lambda[i];
        float s1 = l1 < lambda[i + 1] ? l1 : lambda[i + 1];
        float a = o_lerpf((s0 - lambda[i]) / (lambda[i + 1] - lambda[i]), vals[i], vals[i + 1]);
        float b = o_lerpf((s1 - lambda[i]) / (lambda[i + 1] - lambda[i]), vals[i], vals[i + 1]);
        sum += (0.5f * (a + b)) * (s1 - s0);
    }
    return sum / (l1 - l0);
}

/* spectrum.h:302-321 (lambda assumed sorted, as every caller on the path passes) */
void o_from_sampled(const float *lambda, const float *vals, int n, float out[O_NB]) {
    for (int i = 0; i < O_NB; ++i) {
        float l0 = o_lerpf((float)i / (float)O_NB, 400.f, 700.f);
        float l1 = o_lerpf((float)(i + 1) / (float)O_NB, 400.f, 700.f);
        out[i] = o_average_spectrum_samples(lambda, vals, n, l0, l1);
    }
}

static void o_axpy(float a, const float *b, float *acc) {
    for (int i = 0; i < O_NB; ++i) acc[i] += b[i] * a;
}

/* spectrum.cpp:103-187 */
void o_from_rgb(const float rgb[3], int illum, float out[O_NB]) {
    const float *W = illum ? MPSS_BAND_RGBILLUM2SPECTWHITE : MPSS_BAND_RGBREFL2SPECTWHITE;
    const float *C = illum ? MPSS_BAND_RGBILLUM2SPECTCYAN : MPSS_BAND_RGBREFL2SPECTCYAN;
    const float *M = illum ? MPSS_BAND_RGBILLUM2SPECTMAGENTA : MPSS_BAND_RGBREFL2SPECTMAGENTA;
    const float *Y = illum ? MPSS_BAND_RGBILLUM2SPECTYELLOW : MPSS_BAND_RGBREFL2SPECTYELLOW;
    const float *R = illum ? MPSS_BAND_RGBILLUM2SPECTRED : MPSS_BAND_RGBREFL2SPECTRED;
    const float *G = illum ? MPSS_BAND_RGBILLUM2SPECTGREEN : MPSS_BAND_RGBREFL2SPECTGREEN;
    const float *B = illum ? MPSS_BAND_RGBILLUM2SPECTBLUE : MPSS_BAND_RGBREFL2SPECTBLUE;
    float r[O_NB];
    for (int i = 0; i < O_NB; ++i) r[i] = 0.f;
    if (rgb[0] <= rgb[1] && rgb[0] <= rgb[2]) {
        o_axpy(rgb[0], W, r);
        if (rgb[1] <= rgb[2]) { o_axpy(rgb[1] - rgb[0], C, r); o_axpy(rgb[2] - rgb[1], B, r); }
        else { o_axpy(rgb[2] - rgb[0], C, r); o_axpy(rgb[1] - rgb[2], G, r); }
    } else if (rgb[1] <= rgb[0] && rgb[1] <= rgb[2]) {
        o_axpy(rgb[1], W, r);
        if (rgb[0] <= rgb[2]) { o_axpy(rgb[0] - rgb[1], M, r); o_axpy(rgb[2] - rgb[0], B, r); }
        else { o_axpy(rgb[2] - rgb[1], M, r); o_axpy(rgb[0] - rgb[2], R, r); }
    } else {
        o_axpy(rgb[2], W, r);
        if (rgb[0] <= rgb[1]) { o_axpy(rgb[0] - rgb[2], Y, r); o_axpy(rgb[1] - rgb[0], G, r); }
        else { o_axpy(rgb[1] - rgb[2], Y, r); o_axpy(rgb[0] - rgb[1], R, r); }
    }
    float s = illum ? .86445f : (float).94; /* spectrum.cpp:140 (.94 double -> float operator*=) and :185 */
    for (int i = 0; i < O_NB; ++i) {
        float v = r[i] * s;
        out[i] = v < 0.f ? 0.f : v; /* Clamp(0, INFINITY) */
    }
}

/* spectrum.h:387-393 */
float o_y(const float s[O_NB]) {
    float yy = 0.f;
    for (int i = 0; i < O_NB; ++i) yy += MPSS_BAND_CIE_Y[i] * s[i];
    return yy * (float)(700 - 400) / (float)(MPSS_CIE_Y_INTEGRAL * O_NB);
}

/* spectrum.h:374-386 */
void o_to_xyz(const float s[O_NB], float xyz[3]) {
    xyz[0] = xyz[1] = xyz[2] = 0.f;
    for (int i = 0; i < O_NB; ++i) {
        xyz[0] += MPSS_BAND_CIE_X[i] * s[i];
        xyz[1] += MPSS_BAND_CIE_Y[i] * s[i];
        xyz[2] += MPSS_BAND_CIE_Z[i] * s[i];
    }
    float scale = (float)(700 - 400) / (float)(MPSS_CIE_Y_INTEGRAL * O_NB);
    xyz[0] *= scale;
    xyz[1] *= scale;
    xyz[2] *= scale;
}

/* spectrum.h:374-398 (ToXYZ) and :51-55 (XYZToRGB) */
void o_to_rgb(const float s[O_NB], float rgb[3]) {
    static const float X[O_NB] = MPSS_BAND_CIE_X_INIT, Y[O_NB] = MPSS_BAND_CIE_Y_INIT, Z[O_NB] = MPSS_BAND_CIE_Z_INIT;
    float xyz[3];
    xyz[0] = xyz[1] = xyz[2] = 0.f;
    for (int i = 0; i < O_NB; ++i) {
        xyz[0] += X[i] * s[i];
        xyz[1] += Y[i] * s[i];
        xyz[2] += Z[i] * s[i];
    }
    float scale = (float)(700 - 400) / (float)(MPSS_CIE_Y_INTEGRAL * O_NB);
    xyz[0] *= scale;
    xyz[1] *= scale;
    xyz[2] *= scale;
    rgb[0] = 3.240479f * xyz[0] - 1.537150f * xyz[1] - 0.498535f * xyz[2];
    rgb[1] = -0.969256f * xyz[0] + 1.875991f * xyz[1] + 0.041556f * xyz[2];
    rgb[2] = 0.055648f * xyz[0] - 0.204043f * xyz[1] + 1.057311f * xyz[2];
}
