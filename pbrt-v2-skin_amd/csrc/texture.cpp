// texture.cpp -- MIPMap pyramid construction (core/mipmap.h:67-87, 147-220) and the
// ImageTexture texel conversion (textures/imagemap.cpp:55-84, imagemap.h:89-96), on the host.
#include <algorithm>
#include <cmath>
#include <cstring>

#include "../../include/mpss.h"
#include "texture_build.h"

namespace mpss {
namespace {

uint32_t round_up_pow2_u(uint32_t v) {
    v--;
    v |= v >> 1;
    v |= v >> 2;
    v |= v >> 4;
    v |= v >> 8;
    v |= v >> 16;
    return v + 1;
}

float lanczos(float x, float tau = 2.f) {  // core/texture.cpp:266-274
    x = fabsf(x);
    if ((double)x < 1e-5) return 1.f;
    if (x > 1.f) return 0.f;
    x *= kPiF;
    const float s = m_sin(x * tau) / (x * tau);
    const float l = m_sin(x) / x;
    return s * l;
}

struct ResampleWeight {
    int first;
    float w[4];
};

std::vector<ResampleWeight> resample_weights(uint32_t oldres, uint32_t newres) {  // mipmap.h:67-87
    std::vector<ResampleWeight> wt(newres);
    const float filterwidth = 2.f;
    for (uint32_t i = 0; i < newres; ++i) {
        const float center = ((float)i + .5f) * (float)oldres / (float)newres;
        wt[i].first = (int)floorf((center - filterwidth) + 0.5f);
        for (int j = 0; j < 4; ++j) {
            const float pos = (float)(wt[i].first + j) + .5f;
            wt[i].w[j] = lanczos((pos - center) / filterwidth);
        }
        const float inv = 1.f / (((wt[i].w[0] + wt[i].w[1]) + wt[i].w[2]) + wt[i].w[3]);
        for (int j = 0; j < 4; ++j) wt[i].w[j] *= inv;
    }
    return wt;
}

// the resampling's source index under the wrap mode (mipmap.h:163-167, 182-184); -1: skipped
int wrap_index(int i, int n, int wrap) {
    if (wrap == TEX_REPEAT) i = tex_mod(i, n);
    else if (wrap == TEX_CLAMP) i = std::min(std::max(i, 0), n - 1);
    return (i >= 0 && i < n) ? i : -1;
}

}  // namespace

TexView HostPyramid::view(int trilinear, float max_aniso) const {
    TexView v{};
    v.data = data.data();
    v.lut = ewa_weight_lut();
    v.nch = nch;
    v.nlevels = nlevels;
    v.wrap = wrap;
    v.trilinear = trilinear;
    v.max_aniso = max_aniso;
    v.su = v.sv = 1.f;
    v.du = v.dv = 0.f;
    memcpy(v.lw, lw, sizeof(lw));
    memcpy(v.lh, lh, sizeof(lh));
    memcpy(v.off, off, sizeof(off));
    return v;
}

const float *ewa_weight_lut() {
    static const std::vector<float> lut = [] {
        std::vector<float> w(kEwaLut);
        for (int i = 0; i < kEwaLut; ++i) {
            const float alpha = 2;
            const float r2 = float(i) / float(kEwaLut - 1);
            w[i] = m_exp(-alpha * r2) - m_exp(-alpha);
        }
        return w;
    }();
    return lut.data();
}

HostPyramid build_pyramid(int sres_i, int tres_i, int nch, const float *img, int wrap) {
    if (sres_i < 1 || tres_i < 1) throw Error(MPSS_ERR_INVALID, "MIPMap: empty image");
    if (nch != 1 && nch != 3) throw Error(MPSS_ERR_INVALID, "MIPMap: 1 or 3 channels");
    if (wrap < TEX_REPEAT || wrap > TEX_CLAMP) throw Error(MPSS_ERR_INVALID, "MIPMap: bad wrap mode");
    uint32_t sres = (uint32_t)sres_i, tres = (uint32_t)tres_i;
    std::vector<float> resampled;
    if ((sres & (sres - 1)) != 0 || (tres & (tres - 1)) != 0) {
        const uint32_t sp = round_up_pow2_u(sres), tp = round_up_pow2_u(tres);
        const std::vector<ResampleWeight> sw = resample_weights(sres, sp);
        resampled.assign((size_t)sp * tp * nch, 0.f);
        for (uint32_t t = 0; t < tres; ++t)
            for (uint32_t s = 0; s < sp; ++s) {
                float *o = &resampled[nch * ((size_t)t * sp + s)];
                for (int k = 0; k < nch; ++k) o[k] = 0.f;
                for (int j = 0; j < 4; ++j) {
                    const int os = wrap_index(sw[s].first + j, (int)sres, wrap);
                    if (os >= 0) {
                        const float *x = &img[nch * ((size_t)t * sres + os)];
                        for (int k = 0; k < nch; ++k) o[k] += x[k] * sw[s].w[j];
                    }
                }
            }
        const std::vector<ResampleWeight> tw = resample_weights(tres, tp);
        std::vector<float> work((size_t)tp * nch);
        for (uint32_t s = 0; s < sp; ++s) {
            for (uint32_t t = 0; t < tp; ++t) {
                float *o = &work[nch * (size_t)t];
                for (int k = 0; k < nch; ++k) o[k] = 0.f;
                for (int j = 0; j < 4; ++j) {
                    const int ot = wrap_index(tw[t].first + j, (int)tres, wrap);
                    if (ot >= 0) {
                        const float *x = &resampled[nch * ((size_t)ot * sp + s)];
                        for (int k = 0; k < nch; ++k) o[k] += x[k] * tw[t].w[j];
                    }
                }
            }
            for (uint32_t t = 0; t < tp; ++t)
                for (int k = 0; k < nch; ++k) {  // clamp(): Clamp(v, 0, INFINITY)
                    const float v = work[nch * (size_t)t + k];
                    resampled[nch * ((size_t)t * sp + s) + k] = v < 0.f ? 0.f : (v > INFINITY ? INFINITY : v);
                }
        }
        img = resampled.data();
        sres = sp;
        tres = tp;
    }
    HostPyramid py;
    py.nch = nch;
    py.wrap = wrap;
    py.nlevels = 1 + (int)floorf(tex_log2((float)std::max(sres, tres)));  // 1 + Log2Int(float(max))
    if (py.nlevels > kTexMaxLevels) throw Error(MPSS_ERR_INVALID, "MIPMap: image larger than 32768 texels");
    size_t total = 0;
    for (int i = 0; i < py.nlevels; ++i) {
        py.lw[i] = i == 0 ? (int)sres : std::max(1, py.lw[i - 1] / 2);
        py.lh[i] = i == 0 ? (int)tres : std::max(1, py.lh[i - 1] / 2);
        py.off[i] = (uint32_t)total;
        total += (size_t)py.lw[i] * py.lh[i] * nch;
    }
    if (total > 0xffffffffull) throw Error(MPSS_ERR_INVALID, "MIPMap: pyramid too large");
    py.data.resize(total);
    std::copy(img, img + (size_t)sres * tres * nch, py.data.begin());
    TexView v = py.view();
    for (int i = 1; i < py.nlevels; ++i) {
        v.data = py.data.data();
        for (int t = 0; t < py.lh[i]; ++t)
            for (int s = 0; s < py.lw[i]; ++s) {  // .25f * (four texels of level i - 1, summed in order)
                float a[3], b[3], c[3], d[3];
                tex_texel(v, i - 1, 2 * s, 2 * t, a);
                tex_texel(v, i - 1, 2 * s + 1, 2 * t, b);
                tex_texel(v, i - 1, 2 * s, 2 * t + 1, c);
                tex_texel(v, i - 1, 2 * s + 1, 2 * t + 1, d);
                float *o = &py.data[py.off[i] + nch * ((size_t)t * py.lw[i] + s)];
                for (int k = 0; k < nch; ++k) o[k] = .25f * (((a[k] + b[k]) + c[k]) + d[k]);
            }
    }
    return py;
}

}  // namespace mpss
