/* texture.c -- CPU restatement of pbrt-v2-skin's ImageTexture path (TEST INFRASTRUCTURE ONLY,
 * see oracle.h): the parity checker for the product's texture.h / texture.cpp. Follows:
 *   ImageTexture::GetTexture + convertIn   textures/imagemap.cpp:55-84, imagemap.h:89-96
 *   MIPMap ctor (Lanczos resample, levels)  core/mipmap.h:67-87, 147-220
 *   MIPMap Texel / triangle / Lookup / EWA  core/mipmap.h:223-367
 *   UVMapping2D::Map                        core/texture.cpp:88-98
 * Transcendentals in double rounded once to float (the convention shared with the product). */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static float t_log2(float x) { /* Log2: logf(x) * (1 / logf(2)) */
    float inv = 1.f / (float)log(2.0);
    return (float)log((double)x) * inv;
}
static int t_mod(int a, int b) { int n = a / b; a -= n * b; if (a < 0) a += b; return a; }
static int t_clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

static float lanczos_w(float x) { /* Lanczos(x, tau = 2), core/texture.cpp:266-274 */
    const float tau = 2.f;
    x = fabsf(x);
    if (x < 1e-5) return 1.f;
    if (x > 1.f) return 0.f;
    x *= 3.14159265358979323846f;
    float s = (float)sin((double)(x * tau)) / (x * tau);
    float lz = (float)sin((double)x) / x;
    return s * lz;
}

static unsigned rup2(unsigned v) { unsigned r = 1; while (r < v) r <<= 1; return r; }

typedef struct { int first; float w[4]; } rweight;

static rweight *resample_w(unsigned oldres, unsigned newres) {
    rweight *wt = (rweight *)malloc(newres * sizeof(rweight));
    for (unsigned i = 0; i < newres; ++i) {
        float center = (i + .5f) * oldres / newres;
        wt[i].first = (int)floorf((center - 2.f) + 0.5f);
        for (int j = 0; j < 4; ++j) {
            float pos = wt[i].first + j + .5f;
            wt[i].w[j] = lanczos_w((pos - center) / 2.f);
        }
        float inv = 1.f / (wt[i].w[0] + wt[i].w[1] + wt[i].w[2] + wt[i].w[3]);
        for (int j = 0; j < 4; ++j) wt[i].w[j] *= inv;
    }
    return wt;
}

static const float *texel(const o_tex *t, int level, int s, int u) {
    static const float black[3] = {0.f, 0.f, 0.f};
    int w = t->w[level], h = t->h[level];
    if (t->wrap == 0) { s = t_mod(s, w); u = t_mod(u, h); }
    else if (t->wrap == 2) { s = t_clampi(s, 0, w - 1); u = t_clampi(u, 0, h - 1); }
    else if (s < 0 || s >= w || u < 0 || u >= h) return black;
    return t->lv[level] + (size_t)t->nch * ((size_t)u * w + s);
}

static float g_lut[128];
static void init_lut(void) {
    for (int i = 0; i < 128; ++i) {
        float alpha = 2;
        float r2 = (float)i / (float)(128 - 1);
        g_lut[i] = (float)exp((double)(-alpha * r2)) - (float)exp((double)(-alpha));
    }
}

/* MIPMap ctor over already converted texels (nch floats each) */
static void mipmap_init(o_tex *t, unsigned sres, unsigned tres, const float *img) {
    int nch = t->nch;
    float *res = NULL;
    if ((sres & (sres - 1)) || (tres & (tres - 1))) {
        unsigned sp = rup2(sres), tp = rup2(tres);
        rweight *sw = resample_w(sres, sp);
        res = (float *)calloc((size_t)sp * tp * nch, sizeof(float));
        for (unsigned u = 0; u < tres; ++u)
            for (unsigned s = 0; s < sp; ++s) {
                float *o = res + nch * ((size_t)u * sp + s);
                for (int k = 0; k < nch; ++k) o[k] = 0.f;
                for (int j = 0; j < 4; ++j) {
                    int os = sw[s].first + j;
                    if (t->wrap == 0) os = t_mod(os, (int)sres);
                    else if (t->wrap == 2) os = t_clampi(os, 0, (int)sres - 1);
                    if (os >= 0 && os < (int)sres)
                        for (int k = 0; k < nch; ++k) o[k] += sw[s].w[j] * img[nch * ((size_t)u * sres + os) + k];
                }
            }
        free(sw);
        rweight *tw = resample_w(tres, tp);
        float *work = (float *)malloc((size_t)tp * nch * sizeof(float));
        for (unsigned s = 0; s < sp; ++s) {
            for (unsigned u = 0; u < tp; ++u) {
                for (int k = 0; k < nch; ++k) work[nch * u + k] = 0.f;
                for (int j = 0; j < 4; ++j) {
                    int ot = tw[u].first + j;
                    if (t->wrap == 0) ot = t_mod(ot, (int)tres);
                    else if (t->wrap == 2) ot = t_clampi(ot, 0, (int)tres - 1);
                    if (ot >= 0 && ot < (int)tres)
                        for (int k = 0; k < nch; ++k)
                            work[nch * u + k] += tw[u].w[j] * res[nch * ((size_t)ot * sp + s) + k];
                }
            }
            for (unsigned u = 0; u < tp; ++u)
                for (int k = 0; k < nch; ++k) {
                    float v = work[nch * u + k];
                    res[nch * ((size_t)u * sp + s) + k] = v < 0.f ? 0.f : v;
                }
        }
        free(work);
        free(tw);
        img = res;
        sres = sp;
        tres = tp;
    }
    unsigned mx = sres > tres ? sres : tres;
    t->nlevels = 1 + (int)floorf(t_log2((float)mx));
    t->w[0] = (int)sres;
    t->h[0] = (int)tres;
    t->lv[0] = (float *)malloc((size_t)sres * tres * nch * sizeof(float));
    memcpy(t->lv[0], img, (size_t)sres * tres * nch * sizeof(float));
    for (int i = 1; i < t->nlevels; ++i) {
        int w = t->w[i - 1] / 2, h = t->h[i - 1] / 2;
        t->w[i] = w < 1 ? 1 : w;
        t->h[i] = h < 1 ? 1 : h;
        t->lv[i] = (float *)malloc((size_t)t->w[i] * t->h[i] * nch * sizeof(float));
        for (int u = 0; u < t->h[i]; ++u)
            for (int s = 0; s < t->w[i]; ++s) {
                const float *a = texel(t, i - 1, 2 * s, 2 * u), *b = texel(t, i - 1, 2 * s + 1, 2 * u);
                const float *c = texel(t, i - 1, 2 * s, 2 * u + 1), *d = texel(t, i - 1, 2 * s + 1, 2 * u + 1);
                for (int k = 0; k < nch; ++k)
                    t->lv[i][nch * ((size_t)u * t->w[i] + s) + k] = .25f * (a[k] + b[k] + c[k] + d[k]);
            }
    }
    free(res);
}

int o_tex_build(o_tex *t, int W, int H, const float *texels, int is_float, float shift, float scale, float gamma,
                int wrap, int trilinear, float max_aniso, float su, float sv, float du, float dv) {
    memset(t, 0, sizeof(*t));
    if (!g_lut[0]) init_lut();
    t->nch = is_float ? 1 : 3;
    t->su = su; t->sv = sv; t->du = du; t->dv = dv;
    if (W <= 0 || H <= 0 || !texels) { /* one-valued MIPMap with the MIPMap ctor defaults */
        float one = (float)pow((double)(scale * (1 + shift)), (double)gamma);
        float v[3] = {one, one, one};
        t->wrap = 0; t->trilinear = 0; t->max_aniso = 8.f;
        mipmap_init(t, 1, 1, v);
        return 0;
    }
    t->wrap = wrap; t->trilinear = trilinear; t->max_aniso = max_aniso;
    size_t n = (size_t)W * H;
    float *conv = (float *)malloc(n * t->nch * sizeof(float));
    for (size_t i = 0; i < n; ++i) {
        const float *x = texels + 3 * i;
        if (t->nch == 3) {
            for (int k = 0; k < 3; ++k) conv[3 * i + k] = scale * ((float)pow((double)x[k], (double)gamma) + shift);
        } else {
            float y = 0.212671f * x[0] + 0.715160f * x[1] + 0.072169f * x[2];
            conv[i] = scale * ((float)pow((double)y, (double)gamma) + shift);
        }
    }
    mipmap_init(t, (unsigned)W, (unsigned)H, conv);
    free(conv);
    return 0;
}

void o_tex_free(o_tex *t) {
    for (int i = 0; i < t->nlevels; ++i) free(t->lv[i]);
    memset(t, 0, sizeof(*t));
}

static void triangle(const o_tex *t, int level, float s, float u, float out[3]) {
    level = t_clampi(level, 0, t->nlevels - 1);
    s = s * t->w[level] - 0.5f;
    u = u * t->h[level] - 0.5f;
    int s0 = (int)floorf(s), u0 = (int)floorf(u);
    float ds = s - s0, du = u - u0;
    const float *a = texel(t, level, s0, u0), *b = texel(t, level, s0, u0 + 1);
    const float *c = texel(t, level, s0 + 1, u0), *d = texel(t, level, s0 + 1, u0 + 1);
    for (int k = 0; k < 3; ++k) out[k] = 0.f;
    for (int k = 0; k < t->nch; ++k)
        out[k] = (1.f - ds) * (1.f - du) * a[k] + (1.f - ds) * du * b[k] + ds * (1.f - du) * c[k] + ds * du * d[k];
}

static void ewa(const o_tex *t, int level, float s, float u, float ds0, float dt0, float ds1, float dt1,
                float out[3]) {
    for (int k = 0; k < 3; ++k) out[k] = 0.f;
    if (level >= t->nlevels) {
        const float *x = texel(t, t->nlevels - 1, 0, 0);
        for (int k = 0; k < t->nch; ++k) out[k] = x[k];
        return;
    }
    s = s * t->w[level] - 0.5f;
    u = u * t->h[level] - 0.5f;
    ds0 *= t->w[level];
    dt0 *= t->h[level];
    ds1 *= t->w[level];
    dt1 *= t->h[level];
    float A = dt0 * dt0 + dt1 * dt1 + 1;
    float B = -2.f * (ds0 * dt0 + ds1 * dt1);
    float C = ds0 * ds0 + ds1 * ds1 + 1;
    float invF = 1.f / (A * C - B * B * 0.25f);
    A *= invF;
    B *= invF;
    C *= invF;
    float det = -B * B + 4.f * A * C;
    float invDet = 1.f / det;
    float uSqrt = sqrtf(det * C), vSqrt = sqrtf(A * det);
    int s0 = (int)ceilf(s - 2.f * invDet * uSqrt), s1 = (int)floorf(s + 2.f * invDet * uSqrt);
    int t0 = (int)ceilf(u - 2.f * invDet * vSqrt), t1 = (int)floorf(u + 2.f * invDet * vSqrt);
    float sum[3] = {0.f, 0.f, 0.f}, sumWts = 0.f;
    for (int it = t0; it <= t1; ++it) {
        float tt = it - u;
        for (int is = s0; is <= s1; ++is) {
            float ss = is - s;
            float r2 = A * ss * ss + B * ss * tt + C * tt * tt;
            if (r2 < 1.) {
                int li = (int)(r2 * 128);
                float weight = g_lut[li < 127 ? li : 127];
                const float *x = texel(t, level, is, it);
                for (int k = 0; k < t->nch; ++k) sum[k] += x[k] * weight;
                sumWts += weight;
            }
        }
    }
    for (int k = 0; k < t->nch; ++k) out[k] = sum[k] / sumWts;
}

static void lookup_width(const o_tex *t, float s, float u, float width, float out[3]) {
    float level = (unsigned)(t->nlevels - 1) + t_log2(width < 1e-8f ? 1e-8f : width);
    if (level < 0) {
        triangle(t, 0, s, u, out);
    } else if (level >= (unsigned)(t->nlevels - 1)) {
        const float *x = texel(t, t->nlevels - 1, 0, 0);
        for (int k = 0; k < 3; ++k) out[k] = k < t->nch ? x[k] : 0.f;
    } else {
        int il = (int)floorf(level);
        float delta = level - il, a[3], b[3];
        triangle(t, il, s, u, a);
        triangle(t, il + 1, s, u, b);
        for (int k = 0; k < 3; ++k) out[k] = (1.f - delta) * a[k] + delta * b[k];
    }
}

static void lookup(const o_tex *t, float s, float u, float ds0, float dt0, float ds1, float dt1, float out[3]) {
    if (t->trilinear) {
        float m0 = fabsf(ds0) < fabsf(dt0) ? fabsf(dt0) : fabsf(ds0);
        float m1 = fabsf(ds1) < fabsf(dt1) ? fabsf(dt1) : fabsf(ds1);
        lookup_width(t, s, u, 2.f * (m0 < m1 ? m1 : m0), out);
        return;
    }
    if (ds0 * ds0 + dt0 * dt0 < ds1 * ds1 + dt1 * dt1) {
        float x = ds0; ds0 = ds1; ds1 = x;
        x = dt0; dt0 = dt1; dt1 = x;
    }
    float majorLength = sqrtf(ds0 * ds0 + dt0 * dt0);
    float minorLength = sqrtf(ds1 * ds1 + dt1 * dt1);
    if (minorLength * t->max_aniso < majorLength && minorLength > 0.f) {
        float scale = majorLength / (minorLength * t->max_aniso);
        ds1 *= scale;
        dt1 *= scale;
        minorLength *= scale;
    }
    if (minorLength == 0.f) {
        triangle(t, 0, s, u, out);
        return;
    }
    float lod = t->nlevels - 1.f + t_log2(minorLength);
    if (!(0.f < lod)) lod = 0.f; /* max(0.f, lod) */
    unsigned ilod = (unsigned)floorf(lod);
    float d = lod - ilod, a[3], b[3];
    ewa(t, (int)ilod, s, u, ds0, dt0, ds1, dt1, a);
    ewa(t, (int)ilod + 1, s, u, ds0, dt0, ds1, dt1, b);
    for (int k = 0; k < 3; ++k) out[k] = (1.f - d) * a[k] + d * b[k];
}

void o_tex_eval(const o_tex *t, float u, float v, float dudx, float dvdx, float dudy, float dvdy, float out[3]) {
    float s = t->su * u + t->du, tt = t->sv * v + t->dv;
    lookup(t, s, tt, t->su * dudx, t->sv * dvdx, t->su * dudy, t->sv * dvdy, out);
}

int o_imagemap_lookup(int W, int H, const float *texels, int is_float, float shift, float scale, float gamma,
                      int wrap, int trilinear, float max_aniso, float su, float sv, float du, float dv, int n,
                      const float *uvd, float *out) {
    o_tex t;
    o_tex_build(&t, W, H, texels, is_float, shift, scale, gamma, wrap, trilinear, max_aniso, su, sv, du, dv);
    for (int i = 0; i < n; ++i) {
        const float *a = uvd + 6 * (size_t)i;
        o_tex_eval(&t, a[0], a[1], a[2], a[3], a[4], a[5], out + 3 * (size_t)i);
    }
    o_tex_free(&t);
    return 0;
}
