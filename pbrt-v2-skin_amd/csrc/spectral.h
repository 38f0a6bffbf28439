// spectral.h -- 30-band spectrum helpers (host side), following pbrt's SampledSpectrum
// (reference src/core/spectrum.h:291-393 and spectrum.cpp:60-187). Band tables are the
// committed 30-band averages in data/spectral_bands.h (tools/gen_spectral_bands.py).
#pragma once
#include "common.h"
#include "../../data/spectral_bands.h"

namespace mpss {

inline float lerpf_(float t, float a, float b) { return (1.f - t) * a + t * b; }

// AverageSpectrumSamples, spectrum.cpp:60-94
float average_spectrum_samples(const float *lambda, const float *vals, int n, float l0, float l1);
// SampledSpectrum::FromSampled, spectrum.h:302-321
void spectrum_from_sampled(const float *lambda, const float *vals, int n, float out[NB]);
// SampledSpectrum::FromRGB, spectrum.cpp:103-187
void spectrum_from_rgb(const float rgb[3], bool illuminant, float out[NB]);

// SampledSpectrum::y(), spectrum.h:387-393
inline float spectrum_y(const float *s) {
    float yy = 0.f;
    for (int i = 0; i < NB; ++i) yy += MPSS_BAND_CIE_Y[i] * s[i];
    return yy * (float)(700 - 400) / (float)(MPSS_CIE_Y_INTEGRAL * NB);
}

// SampledSpectrum::ToXYZ + XYZToRGB (spectrum.h:51-55, 370-393): ToRGBSpectrum's texel value
inline void spectrum_to_rgb(const float *s, float rgb[3]) {
    float xyz[3] = {0.f, 0.f, 0.f};
    for (int i = 0; i < NB; ++i) {
        xyz[0] += MPSS_BAND_CIE_X[i] * s[i];
        xyz[1] += MPSS_BAND_CIE_Y[i] * s[i];
        xyz[2] += MPSS_BAND_CIE_Z[i] * s[i];
    }
    const float scale = (float)(700 - 400) / (float)(MPSS_CIE_Y_INTEGRAL * NB);
    for (int k = 0; k < 3; ++k) xyz[k] *= scale;
    rgb[0] = (3.240479f * xyz[0] - 1.537150f * xyz[1]) - 0.498535f * xyz[2];
    rgb[1] = (-0.969256f * xyz[0] + 1.875991f * xyz[1]) + 0.041556f * xyz[2];
    rgb[2] = (0.055648f * xyz[0] - 0.204043f * xyz[1]) + 1.057311f * xyz[2];
}

}  // namespace mpss
