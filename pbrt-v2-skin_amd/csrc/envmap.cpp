// envmap.cpp -- see envmap.h for the reference lines this build follows.
#include "envmap.h"

#include <algorithm>
#include <cmath>
#include <cstdint>

#include "../../include/mpss.h"
#include "common.h"
#include "pbrt_math.h"

namespace mpss {
namespace {

float log2f_pbrt(float x) {  // Log2 (pbrt.h:300-303): logf(x) * (1 / logf(2))
    static const float inv_log2 = 1.f / m_log(2.f);
    return m_log(x) * inv_log2;
}
int log2int_pbrt(float v) { return (int)floorf(log2f_pbrt(v)); }
int mod_pbrt(int a, int b) {  // Mod (pbrt.h:282-287)
    const int n = a / b;
    a -= n * b;
    if (a < 0) a += b;
    return a;
}
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

struct Level {
    int w, h;
    std::vector<float> rgb;
    const float *texel(int s, int t) const {  // MIPMap::Texel with TEXTURE_REPEAT
        s = mod_pbrt(s, w);
        t = mod_pbrt(t, h);
        return &rgb[3 * ((size_t)t * w + s)];
    }
};

struct Pyramid {
    std::vector<Level> lv;

    // MIPMap::triangle (mipmap.h:258-269)
    void triangle(int level, float s, float t, float out[3]) const {
        level = std::min(std::max(level, 0), (int)lv.size() - 1);
        const Level &L = lv[level];
        s = s * (float)L.w - 0.5f;
        t = t * (float)L.h - 0.5f;
        const int s0 = (int)floorf(s), t0 = (int)floorf(t);
        const float ds = s - (float)s0, dt = t - (float)t0;
        const float w00 = (1.f - ds) * (1.f - dt), w01 = (1.f - ds) * dt, w10 = ds * (1.f - dt), w11 = ds * dt;
        const float *a = L.texel(s0, t0), *b = L.texel(s0, t0 + 1), *c = L.texel(s0 + 1, t0),
                    *d = L.texel(s0 + 1, t0 + 1);
        for (int k = 0; k < 3; ++k) out[k] = ((a[k] * w00 + b[k] * w01) + c[k] * w10) + d[k] * w11;
    }

    // MIPMap::Lookup(s, t, width) (mipmap.h:239-255)
    void lookup(float s, float t, float width, float out[3]) const {
        const int n = (int)lv.size();
        const float level = (float)(uint32_t)(n - 1) + log2f_pbrt(std::max(width, 1e-8f));
        if (level < 0.f) {
            triangle(0, s, t, out);
        } else if (level >= (float)(uint32_t)(n - 1)) {
            const float *x = lv[n - 1].texel(0, 0);
            for (int k = 0; k < 3; ++k) out[k] = x[k];
        } else {
            const int il = (int)floorf(level);
            const float delta = level - (float)il;
            float a[3], b[3];
            triangle(il, s, t, a);
            triangle(il + 1, s, t, b);
            for (int k = 0; k < 3; ++k) out[k] = a[k] * (1.f - delta) + b[k] * delta;
        }
    }
};

Pyramid build_pyramid(uint32_t sres, uint32_t tres, const float *img) {  // mipmap.h:147-205
    std::vector<float> resampled;
    if ((sres & (sres - 1)) != 0 || (tres & (tres - 1)) != 0) {
        const uint32_t sp = round_up_pow2_u(sres), tp = round_up_pow2_u(tres);
        const std::vector<ResampleWeight> sw = resample_weights(sres, sp);
        resampled.assign((size_t)sp * tp * 3, 0.f);
        for (uint32_t t = 0; t < tres; ++t)
            for (uint32_t s = 0; s < sp; ++s) {
                float *o = &resampled[3 * ((size_t)t * sp + s)];
                o[0] = o[1] = o[2] = 0.f;
                for (int j = 0; j < 4; ++j) {
                    const int os = mod_pbrt(sw[s].first + j, (int)sres);
                    if (os >= 0 && os < (int)sres) {
                        const float *x = &img[3 * ((size_t)t * sres + os)];
                        for (int k = 0; k < 3; ++k) o[k] += x[k] * sw[s].w[j];
                    }
                }
            }
        const std::vector<ResampleWeight> tw = resample_weights(tres, tp);
        std::vector<float> work((size_t)tp * 3);
        for (uint32_t s = 0; s < sp; ++s) {
            for (uint32_t t = 0; t < tp; ++t) {
                float *o = &work[3 * (size_t)t];
                o[0] = o[1] = o[2] = 0.f;
                for (int j = 0; j < 4; ++j) {
                    const int ot = mod_pbrt(tw[t].first + j, (int)tres);
                    if (ot >= 0 && ot < (int)tres) {
                        const float *x = &resampled[3 * ((size_t)ot * sp + s)];
                        for (int k = 0; k < 3; ++k) o[k] += x[k] * tw[t].w[j];
                    }
                }
            }
            for (uint32_t t = 0; t < tp; ++t)
                for (int k = 0; k < 3; ++k) {  // RGBSpectrum::Clamp(0, INFINITY)
                    const float v = work[3 * (size_t)t + k];
                    resampled[3 * ((size_t)t * sp + s) + k] = v < 0.f ? 0.f : (v > INFINITY ? INFINITY : v);
                }
        }
        img = resampled.data();
        sres = sp;
        tres = tp;
    }
    Pyramid py;
    const int n = 1 + log2int_pbrt((float)std::max(sres, tres));
    py.lv.resize(n);
    py.lv[0].w = (int)sres;
    py.lv[0].h = (int)tres;
    py.lv[0].rgb.assign(img, img + (size_t)sres * tres * 3);
    for (int i = 1; i < n; ++i) {
        const Level &p = py.lv[i - 1];
        Level &L = py.lv[i];
        L.w = std::max(1, p.w / 2);
        L.h = std::max(1, p.h / 2);
        L.rgb.resize((size_t)L.w * L.h * 3);
        for (int t = 0; t < L.h; ++t)
            for (int s = 0; s < L.w; ++s) {
                const float *a = p.texel(2 * s, 2 * t), *b = p.texel(2 * s + 1, 2 * t), *c = p.texel(2 * s, 2 * t + 1),
                            *d = p.texel(2 * s + 1, 2 * t + 1);
                for (int k = 0; k < 3; ++k) L.rgb[3 * ((size_t)t * L.w + s) + k] = (((a[k] + b[k]) + c[k]) + d[k]) * .25f;
            }
    }
    return py;
}

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
    const Pyramid py = build_pyramid((uint32_t)W, (uint32_t)H, texels);
    EnvMap m;
    m.w0 = py.lv[0].w;
    m.h0 = py.lv[0].h;
    m.tex = py.lv[0].rgb;
    m.nu = W;
    m.nv = H;
    // img (infinite.cpp:92-101)
    m.func.resize((size_t)W * H);
    const float filter = 1.f / (float)std::max(W, H);
    for (int v = 0; v < H; ++v) {
        const float vp = (float)v / (float)H;
        const float sin_theta = m_sin(kPiF * ((float)v + .5f) / (float)H);
        for (int u = 0; u < W; ++u) {
            const float up = (float)u / (float)W;
            float rgb[3];
            py.lookup(up, vp, filter, rgb);
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
