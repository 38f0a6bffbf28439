// texture_build.h -- host construction of a MIPMap pyramid (core/mipmap.h:147-220) in the flat
// layout texture.h reads, shared by ImageTexture (texture.cpp) and InfiniteAreaLight (envmap.cpp).
#pragma once
#include <vector>

#include "texture.h"

namespace mpss {

struct HostPyramid {
    int nch = 3, nlevels = 0, wrap = TEX_REPEAT;
    int lw[kTexMaxLevels] = {}, lh[kTexMaxLevels] = {};
    uint32_t off[kTexMaxLevels] = {};
    std::vector<float> data;  // every level, nch floats per texel
    // a view over the host copy (lut: ewa_weight_lut())
    TexView view(int trilinear = 0, float max_aniso = 8.f) const;
};

// MIPMap ctor: Lanczos resampling of a non-power-of-two image (with the wrap mode), then the
// box-filtered levels. img: sres x tres texels of nch floats, row-major.
HostPyramid build_pyramid(int sres, int tres, int nch, const float *img, int wrap);

// The EWA weight table (mipmap.h:210-218): expf(-2 r2) - expf(-2) at r2 = i / 127
const float *ewa_weight_lut();

}  // namespace mpss
