// envmap.h -- InfiniteAreaLight's radiance map and its sampling distribution, built on the host
// once per light and uploaded flat (render_host.hip). Follows, in float like the reference:
//   MIPMap<RGBSpectrum> ctor            core/mipmap.h:147-220 (Lanczos resampling of a non-power-
//                                       of-two image, TEXTURE_REPEAT, box-filtered pyramid)
//   MIPMap::Lookup(s, t, width)         core/mipmap.h:239-269 (trilinear between two levels)
//   InfiniteAreaLight ctor              lights/infinite.cpp:66-106 (img = Lookup(u/W, v/H,
//                                       1/max(W,H)).y() * sin(theta))
//   Distribution2D / Distribution1D     core/montecarlo.h:54-175, montecarlo.cpp:358-370
// The device side only needs level 0 of the pyramid (Le and Sample_L look up with width 0,
// i.e. triangle(0, s, t)) and the distribution arrays.
#pragma once
#include <vector>

namespace mpss {

struct EnvMap {
    int w0 = 0, h0 = 0;          // level-0 resolution (powers of two)
    std::vector<float> tex;      // level 0, 3 floats per texel, row t at t * w0
    int nu = 0, nv = 0;          // Distribution2D resolution (the image's own)
    std::vector<float> func;     // nv rows of nu: the conditional distributions' func
    std::vector<float> cdf;      // nv rows of nu + 1
    std::vector<float> row_int;  // nv: conditional funcInt = the marginal's func
    std::vector<float> mcdf;     // nv + 1
    float mint = 0.f;            // the marginal's funcInt
};

// texels: W x H RGB triples, row-major, already multiplied by L.ToRGBSpectrum() (infinite.cpp:76-79)
EnvMap build_envmap(int W, int H, const float *texels);

}  // namespace mpss
