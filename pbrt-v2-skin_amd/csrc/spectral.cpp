// spectral.cpp -- host spectrum helpers (see spectral.h for the reference lines followed).
#include "spectral.h"

namespace mpss {

float average_spectrum_samples(const float *lambda, const float *vals, int n, float l0, float l1) {
    if (l1 <= lambda[0]) return vals[0];
    if (l0 >= lambda[n - 1]) return vals[n - 1];
    if (n == 1) return vals[0];
    float sum = 0.f;
    if (l0 < lambda[0]) sum += vals[0] * (lambda[0] - l0);
    if (l1 > lambda[n - 1]) sum += vals[n - 1] * (l1 - lambda[n - 1]);
    int i = 0;
    while (l0 > lambda[i + 1]) ++i;
    auto interp = [&](float w, int k) {
        return lerpf_((w - lambda[k]) / (lambda[k + 1] - lambda[k]), vals[k], vals[k + 1]);
    };
    for (; i + 1 < n && l1 >= lambda[i]; ++i) {
        const float s0 = l0 > lambda[i] ? l0 : lambda[i];
        const float s1 = l1 < lambda[i + 1] ? l1 : lambda[i + 1];
        sum += (0.5f * (interp(s0, i) + interp(s1, i))) * (s1 - s0);
    }
    return sum / (l1 - l0);
}

void spectrum_from_sampled(const float *lambda, const float *vals, int n, float out[NB]) {
    for (int i = 0; i < NB; ++i) {
        const float l0 = lerpf_((float)i / (float)NB, 400.f, 700.f);
        const float l1 = lerpf_((float)(i + 1) / (float)NB, 400.f, 700.f);
        out[i] = average_spectrum_samples(lambda, vals, n, l0, l1);
    }
}

void spectrum_from_rgb(const float rgb[3], bool illum, float out[NB]) {
    const float *W = illum ? MPSS_BAND_RGBILLUM2SPECTWHITE : MPSS_BAND_RGBREFL2SPECTWHITE;
    const float *Cy = illum ? MPSS_BAND_RGBILLUM2SPECTCYAN : MPSS_BAND_RGBREFL2SPECTCYAN;
    const float *Mg = illum ? MPSS_BAND_RGBILLUM2SPECTMAGENTA : MPSS_BAND_RGBREFL2SPECTMAGENTA;
    const float *Ye = illum ? MPSS_BAND_RGBILLUM2SPECTYELLOW : MPSS_BAND_RGBREFL2SPECTYELLOW;
    const float *Rd = illum ? MPSS_BAND_RGBILLUM2SPECTRED : MPSS_BAND_RGBREFL2SPECTRED;
    const float *Gr = illum ? MPSS_BAND_RGBILLUM2SPECTGREEN : MPSS_BAND_RGBREFL2SPECTGREEN;
    const float *Bl = illum ? MPSS_BAND_RGBILLUM2SPECTBLUE : MPSS_BAND_RGBREFL2SPECTBLUE;
    float r[NB] = {};
    auto add = [&](float a, const float *b) {
        for (int i = 0; i < NB; ++i) r[i] += b[i] * a;
    };
    const float R = rgb[0], G = rgb[1], B = rgb[2];
    if (R <= G && R <= B) {
        add(R, W);
        if (G <= B) { add(G - R, Cy); add(B - G, Bl); }
        else { add(B - R, Cy); add(G - B, Gr); }
    } else if (G <= R && G <= B) {
        add(G, W);
        if (R <= B) { add(R - G, Mg); add(B - R, Bl); }
        else { add(B - G, Mg); add(R - B, Rd); }
    } else {
        add(B, W);
        if (R <= G) { add(R - B, Ye); add(G - R, Gr); }
        else { add(G - B, Ye); add(R - G, Rd); }
    }
    const float s = illum ? .86445f : (float).94;
    for (int i = 0; i < NB; ++i) {
        const float v = r[i] * s;
        out[i] = v < 0.f ? 0.f : v;
    }
}

}  // namespace mpss
