/*
 * envmap.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Scalar restatement of the radiance map and sampling distribution of InfiniteAreaLight:
 *   MIPMap<RGBSpectrum>::MIPMap        core/mipmap.h:147-205 (resampleWeights :67-87, Lanczos
 *                                      core/texture.cpp:266-274, TEXTURE_REPEAT Texel :207-227)
 *   MIPMap::Lookup / triangle           core/mipmap.h:239-269
 *   InfiniteAreaLight ctor              lights/infinite.cpp:66-106
 *   Distribution1D / Distribution2D     core/montecarlo.h:54-175, montecarlo.cpp:358-370
 * Float arithmetic in the reference's order; logf / sinf are double-evaluated and rounded once.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define PI_F 3.14159265358979323846f

static float e_log2(float x) {
    static float inv_log2 = 0.f;
    if (inv_log2 == 0.f) inv_log2 = 1.f / (float)log(2.0);
    return (float)log((double)x) * inv_log2;
}

static int e_mod(int a, int b) {
    int n = a / b;
    a -= n * b;
    if (a < 0) a += b;
    return a;
}

static float e_lanczos(float x) {
    const float tau = 2.f;
    x = fabsf(x);
    if (x < 1e-5) return 1;
    if (x > 1.) return 0;
    x *= PI_F;
    float s = (float)sin((double)(x * tau)) / (x * tau);
    float lz = (float)sin((double)x) / x;
    return s * lz;
}

typedef struct { int first; float w[4]; } e_wt;

static e_wt *e_weights(unsigned oldres, unsigned newres) {
    e_wt *wt = (e_wt *)malloc(newres * sizeof(e_wt));
    for (unsigned i = 0; i < newres; ++i) {
        float center = (i + .5f) * oldres / newres;
        wt[i].first = (int)floorf((center - 2.f) + 0.5f);
        for (int j = 0; j < 4; ++j) {
            float pos = wt[i].first + j + .5f;
            wt[i].w[j] = e_lanczos((pos - center) / 2.f);
        }
        float inv = 1.f / (wt[i].w[0] + wt[i].w[1] + wt[i].w[2] + wt[i].w[3]);
        for (int j = 0; j < 4; ++j) wt[i].w[j] *= inv;
    }
    return wt;
}

typedef struct { int w, h; float *rgb; } e_level;

static const float *e_texel(const e_level *l, int s, int t) {
    s = e_mod(s, l->w);
    t = e_mod(t, l->h);
    return l->rgb + 3 * ((size_t)t * l->w + s);
}

static void e_triangle(const e_level *lv, int nlev, int level, float s, float t, float out[3]) {
    if (level < 0) level = 0;
    if (level > nlev - 1) level = nlev - 1;
    const e_level *l = &lv[level];
    s = s * l->w - 0.5f;
    t = t * l->h - 0.5f;
    int s0 = (int)floorf(s), t0 = (int)floorf(t);
    float ds = s - s0, dt = t - t0;
    const float *a = e_texel(l, s0, t0), *b = e_texel(l, s0, t0 + 1), *c = e_texel(l, s0 + 1, t0),
                *d = e_texel(l, s0 + 1, t0 + 1);
    for (int k = 0; k < 3; ++k)
        out[k] = (1.f - ds) * (1.f - dt) * a[k] + (1.f - ds) * dt * b[k] + ds * (1.f - dt) * c[k] + ds * dt * d[k];
}

static void e_lookup(const e_level *lv, int nlev, float s, float t, float width, float out[3]) {
    float level = (unsigned)(nlev - 1) + e_log2(width > 1e-8f ? width : 1e-8f);
    if (level < 0) {
        e_triangle(lv, nlev, 0, s, t, out);
    } else if (level >= (unsigned)(nlev - 1)) {
        memcpy(out, e_texel(&lv[nlev - 1], 0, 0), 3 * sizeof(float));
    } else {
        unsigned il = (unsigned)(int)floorf(level);
        float delta = level - il, a[3], b[3];
        e_triangle(lv, nlev, (int)il, s, t, a);
        e_triangle(lv, nlev, (int)il + 1, s, t, b);
        for (int k = 0; k < 3; ++k) out[k] = (1.f - delta) * a[k] + delta * b[k];
    }
}

static float e_distribution1d(const float *f, int n, float *cdf) {
    cdf[0] = 0.;
    for (int i = 1; i < n + 1; ++i) cdf[i] = cdf[i - 1] + f[i - 1] / n;
    float fi = cdf[n];
    if (fi == 0.f) {
        for (int i = 1; i < n + 1; ++i) cdf[i] = (float)i / (float)n;
    } else {
        for (int i = 1; i < n + 1; ++i) cdf[i] /= fi;
    }
    return fi;
}

static unsigned e_pow2(unsigned v) {
    unsigned r = 1;
    while (r < v) r <<= 1;
    return r;
}

int o_envmap_build(int W, int H, const float *img, o_envmap *m) {
    if (W < 1 || H < 1) return -1;
    unsigned sres = (unsigned)W, tres = (unsigned)H;
    float *base = NULL;
    const float *src = img;
    if ((sres & (sres - 1)) || (tres & (tres - 1))) {
        unsigned sp = e_pow2(sres), tp = e_pow2(tres);
        e_wt *sw = e_weights(sres, sp);
        base = (float *)calloc((size_t)sp * tp * 3, sizeof(float));
        for (unsigned t = 0; t < tres; ++t)
            for (unsigned s = 0; s < sp; ++s) {
                float *o = base + 3 * ((size_t)t * sp + s);
                o[0] = o[1] = o[2] = 0.f;
                for (int j = 0; j < 4; ++j) {
                    int os = e_mod(sw[s].first + j, (int)sres);
                    if (os >= 0 && os < (int)sres)
                        for (int k = 0; k < 3; ++k) o[k] += sw[s].w[j] * img[3 * ((size_t)t * sres + os) + k];
                }
            }
        free(sw);
        e_wt *tw = e_weights(tres, tp);
        float *work = (float *)malloc((size_t)tp * 3 * sizeof(float));
        for (unsigned s = 0; s < sp; ++s) {
            for (unsigned t = 0; t < tp; ++t) {
                float *o = work + 3 * t;
                o[0] = o[1] = o[2] = 0.f;
                for (int j = 0; j < 4; ++j) {
                    int ot = e_mod(tw[t].first + j, (int)tres);
                    if (ot >= 0 && ot < (int)tres)
                        for (int k = 0; k < 3; ++k) o[k] += tw[t].w[j] * base[3 * ((size_t)ot * sp + s) + k];
                }
            }
            for (unsigned t = 0; t < tp; ++t)
                for (int k = 0; k < 3; ++k) {
                    float v = work[3 * t + k];
                    base[3 * ((size_t)t * sp + s) + k] = v < 0.f ? 0.f : (v > INFINITY ? INFINITY : v);
                }
        }
        free(work);
        free(tw);
        src = base;
        sres = sp;
        tres = tp;
    }
    int nlev = 1 + (int)floorf(e_log2((float)(sres > tres ? sres : tres)));
    e_level *lv = (e_level *)calloc(nlev, sizeof(e_level));
    lv[0].w = (int)sres;
    lv[0].h = (int)tres;
    lv[0].rgb = (float *)malloc((size_t)sres * tres * 3 * sizeof(float));
    memcpy(lv[0].rgb, src, (size_t)sres * tres * 3 * sizeof(float));
    free(base);
    for (int i = 1; i < nlev; ++i) {
        e_level *p = &lv[i - 1], *l = &lv[i];
        l->w = p->w / 2 > 1 ? p->w / 2 : 1;
        l->h = p->h / 2 > 1 ? p->h / 2 : 1;
        l->rgb = (float *)malloc((size_t)l->w * l->h * 3 * sizeof(float));
        for (int t = 0; t < l->h; ++t)
            for (int s = 0; s < l->w; ++s)
                for (int k = 0; k < 3; ++k)
                    l->rgb[3 * ((size_t)t * l->w + s) + k] =
                        .25f * (e_texel(p, 2 * s, 2 * t)[k] + e_texel(p, 2 * s + 1, 2 * t)[k] +
                                e_texel(p, 2 * s, 2 * t + 1)[k] + e_texel(p, 2 * s + 1, 2 * t + 1)[k]);
    }
    /* img for the sampling distribution, at the image's own resolution */
    m->nu = W;
    m->nv = H;
    m->func = (float *)malloc((size_t)W * H * sizeof(float));
    float filter = 1.f / (W > H ? W : H);
    for (int v = 0; v < H; ++v) {
        float vp = (float)v / (float)H;
        /* infinite.cpp:94 with pbrt's float M_PI (core/pbrt.h:193-196): a float argument */
        float sin_theta = (float)sin((double)(PI_F * (float)(v + .5f) / (float)H));
        for (int u = 0; u < W; ++u) {
            float up = (float)u / (float)W, rgb[3];
            e_lookup(lv, nlev, up, vp, filter, rgb);
            float y = 0.212671f * rgb[0] + 0.715160f * rgb[1] + 0.072169f * rgb[2];
            m->func[(size_t)v * W + u] = y;
            m->func[(size_t)v * W + u] *= sin_theta;
        }
    }
    m->cdf = (float *)malloc((size_t)H * (W + 1) * sizeof(float));
    m->rint = (float *)malloc((size_t)H * sizeof(float));
    for (int v = 0; v < H; ++v) m->rint[v] = e_distribution1d(m->func + (size_t)v * W, W, m->cdf + (size_t)v * (W + 1));
    m->mcdf = (float *)malloc((size_t)(H + 1) * sizeof(float));
    m->mint = e_distribution1d(m->rint, H, m->mcdf);
    m->tw = lv[0].w;
    m->th = lv[0].h;
    m->tex = lv[0].rgb;
    for (int i = 1; i < nlev; ++i) free(lv[i].rgb);
    free(lv);
    return 0;
}

void o_envmap_free(o_envmap *m) {
    free(m->tex);
    free(m->func);
    free(m->cdf);
    free(m->rint);
    free(m->mcdf);
    memset(m, 0, sizeof(*m));
}

/* MIPMap::Lookup(s, t) with width 0 = triangle(0, s, t) */
void o_envmap_lookup(const o_envmap *m, float s, float t, float out[3]) {
    e_level l0 = {m->tw, m->th, m->tex};
    e_triangle(&l0, 1, 0, s, t, out);
}

/* Distribution1D::SampleContinuous (montecarlo.h:81-98) */
static float e_sample1d(const float *func, const float *cdf, float fint, int count, float u, float *pdf, int *off) {
    /* std::upper_bound: first cdf[i] > u */
    int i = 0;
    while (i < count + 1 && !(u < cdf[i])) ++i;
    int offset = i - 1 > 0 ? i - 1 : 0;
    if (offset > count - 1) offset = count - 1;
    if (off) *off = offset;
    float du = (u - cdf[offset]) / (cdf[offset + 1] - cdf[offset]);
    if (pdf) *pdf = func[offset] / fint;
    return (offset + du) / count;
}

/* Distribution2D::SampleContinuous (montecarlo.h:154-161) */
void o_envmap_sample(const o_envmap *m, float u0, float u1, float uv[2], float *pdf) {
    float pdfs[2];
    int v;
    uv[1] = e_sample1d(m->rint, m->mcdf, m->mint, m->nv, u1, &pdfs[1], &v);
    uv[0] = e_sample1d(m->func + (size_t)v * m->nu, m->cdf + (size_t)v * (m->nu + 1), m->rint[v], m->nu, u0, &pdfs[0],
                       NULL);
    *pdf = pdfs[0] * pdfs[1];
}

/* Distribution2D::Pdf (montecarlo.h:162-170) */
float o_envmap_pdf(const o_envmap *m, float u, float v) {
    int iu = (int)(u * m->nu), iv = (int)(v * m->nv);
    iu = iu < 0 ? 0 : (iu > m->nu - 1 ? m->nu - 1 : iu);
    iv = iv < 0 ? 0 : (iv > m->nv - 1 ? m->nv - 1 : iv);
    if (m->rint[iv] * m->mint == 0.f) return 0.f;
    return (m->func[(size_t)iv * m->nu + iu] * m->rint[iv]) / (m->rint[iv] * m->mint);
}
