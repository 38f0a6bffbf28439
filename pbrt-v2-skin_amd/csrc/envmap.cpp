// envmap.cpp -- see envmap.h for the reference lines this build follows.
#include "envmap.h"

#include <algorithm>
#include <cmath>
#include <cstdint>

#include "../../include/mpss.h"
#include "common.h"
#include "pbrt_math.h"
#include "texture_build.h"

namespace mpss {
namespace {

// Distribution1D ctor (montecarlo.h:56-76): cdf of n values written at cdf[0..n]; returns funcInt
float distribution1d(const float *f, int n, float *cdf) {
    cdf[0] = 0.f;
    for (int i = 1; i < n + 1; ++i) cdf[i] = cdf[i - 1] + f[i - 1] / (float)n;
    const float fi = cdf[n];
    if (fi == 0.f) {
        for (int i = 1; i < n + 1; ++i) cdf[i] = (float)i / (float)n;
    } else {
        for (int i = 1; i < n + 1; ++i) cdf[i] /= fi;
    }
    return fi;
}

}  // namespace

EnvMap build_envmap(int W, int H, const float *texels) {
    if (W < 1 || H < 1) throw Error(MPSS_ERR_INVALID, "infinite light map: empty image");
    const HostPyramid py = build_pyramid(W, H, 3, texels, TEX_REPEAT);
    const TexView tv = py.view();
    EnvMap m;
    m.w0 = py.lw[0];
    m.h0 = py.lh[0];
    m.tex.assign(py.data.begin(), py.data.begin() + (size_t)m.w0 * m.h0 * 3);
    m.nu = W;
    m.nv = H;
    // img (infinite.cpp:92-101)
    m.func.resize((size_t)W * H);
    const float filter = 1.f / (float)std::max(W, H);
    for (int v = 0; v < H; ++v) {
        const float vp = (float)v / (float)H;
        // sinf(M_PI * float(v+.5f)/float(height)) (infinite.cpp:94): pbrt redefines M_PI as the
        // float literal 3.14159265358979323846f (core/pbrt.h:193-196), so the argument is a float
        // product and quotient -- not a double one
        const float sin_theta = m_sin(kPiF * ((float)v + .5f) / (float)H);
        for (int u = 0; u < W; ++u) {
            const float up = (float)u / (float)W;
            float rgb[3];
            tex_lookup_width(tv, up, vp, filter, rgb);
            const float y = (0.212671f * rgb[0] + 0.715160f * rgb[1]) + 0.072169f * rgb[2];  // RGBSpectrum::y
            m.func[(size_t)v * W + u] = y * sin_theta;
        }
    }
    // Distribution2D (montecarlo.cpp:358-370)
    m.cdf.resize((size_t)H * (W + 1));
    m.row_int.resize(H);
    for (int v = 0; v < H; ++v)
        m.row_int[v] = distribution1d(&m.func[(size_t)v * W], W, &m.cdf[(size_t)v * (W + 1)]);
    m.mcdf.resize(H + 1);
    m.mint = distribution1d(m.row_int.data(), H, m.mcdf.data());
    return m;
}

}  // namespace mpss
