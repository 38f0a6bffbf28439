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

}  // namespace mpss
