// texture.h -- ImageTexture lookups of the LayeredSkin textures ("albedo", "bumpmap") on host
// and device, and the surface differentials they are filtered with. Restates, in float with the
// reference's operation order (-ffp-contract=off):
//   MIPMap<T>::Texel / triangle / Lookup(s, t, width) / Lookup(s, t, ds0, dt0, ds1, dt1) / EWA
//                                       core/mipmap.h:223-367 (weight LUT :210-218)
//   UVMapping2D::Map                    core/texture.cpp:88-98
//   ImageTexture::Evaluate/convertOut   textures/imagemap.cpp:180-189, imagemap.h:97-105
//   DifferentialGeometry::ComputeDifferentials   core/diffgeom.cpp:58-111
//   Material::Bump                      core/material.cpp:47-104 (the fork's central differences)
// The pyramid itself (convertIn, Lanczos resampling, box-filtered levels) is built on the host
// (texture.cpp) and uploaded flat: level i at data + off[i], nch floats per texel, row-major.
#pragma once
#include "common.h"
#include "pbrt_math.h"

namespace mpss {

constexpr int kTexMaxLevels = 16;
constexpr int kEwaLut = 128;  // WEIGHT_LUT_SIZE
enum TexWrap : int { TEX_REPEAT = 0, TEX_BLACK = 1, TEX_CLAMP = 2 };

struct TexView {
    const float *data;  // the pyramid (host or device memory)
    const float *lut;   // EWA weight table (kEwaLut floats)
    int nch;            // 3: ImageTexture<RGBSpectrum, Spectrum>; 1: ImageTexture<float, float>
    int nlevels, wrap, trilinear;
    float max_aniso;
    float su, sv, du, dv;  // UVMapping2D
    int lw[kTexMaxLevels], lh[kTexMaxLevels];
    uint32_t off[kTexMaxLevels];
};

MPSS_HD int tex_mod(int a, int b) {  // Mod (pbrt.h:282-287)
    const int n = a / b;
    a -= n * b;
    return a < 0 ? a + b : a;
}

MPSS_HD float tex_log2(float x) {  // Log2 (pbrt.h:300-303): logf(x) * (1 / logf(2))
    const float inv_log2 = 1.f / m_log(2.f);
    return m_log(x) * inv_log2;
}

// MIPMap::Texel (mipmap.h:223-246): out[0..nch) of texel (s, t) of a level under the wrap mode
MPSS_HD void tex_texel(const TexView &T, int level, int s, int t, float out[3]) {
    const int w = T.lw[level], h = T.lh[level];
    if (T.wrap == TEX_REPEAT) {
        s = tex_mod(s, w);
        t = tex_mod(t, h);
    } else if (T.wrap == TEX_CLAMP) {
        s = s < 0 ? 0 : (s > w - 1 ? w - 1 : s);
        t = t < 0 ? 0 : (t > h - 1 ? h - 1 : t);
    } else if (s < 0 || s >= w || t < 0 || t >= h) {
        out[0] = out[1] = out[2] = 0.f;
        return;
    }
    const float *x = T.data + T.off[level] + (size_t)T.nch * ((size_t)t * w + s);
    out[0] = x[0];
    out[1] = T.nch == 3 ? x[1] : 0.f;
    out[2] = T.nch == 3 ? x[2] : 0.f;
}

// MIPMap::triangle (mipmap.h:258-269)
MPSS_HD void tex_triangle(const TexView &T, int level, float s, float t, float out[3]) {
    level = level < 0 ? 0 : (level > T.nlevels - 1 ? T.nlevels - 1 : level);
    s = s * (float)T.lw[level] - 0.5f;
    t = t * (float)T.lh[level] - 0.5f;
    const int s0 = (int)floorf(s), t0 = (int)floorf(t);
    const float ds = s - (float)s0, dt = t - (float)t0;
    const float w00 = (1.f - ds) * (1.f - dt), w01 = (1.f - ds) * dt, w10 = ds * (1.f - dt), w11 = ds * dt;
    float a[3], b[3], c[3], d[3];
    tex_texel(T, level, s0, t0, a);
    tex_texel(T, level, s0, t0 + 1, b);
    tex_texel(T, level, s0 + 1, t0, c);
    tex_texel(T, level, s0 + 1, t0 + 1, d);
    for (int k = 0; k < 3; ++k) out[k] = ((w00 * a[k] + w01 * b[k]) + w10 * c[k]) + w11 * d[k];
}

// MIPMap::EWA (mipmap.h:321-363)
MPSS_HD void tex_ewa(const TexView &T, int level, float s, float t, float ds0, float dt0, float ds1, float dt1,
                     float out[3]) {
    if (level >= T.nlevels) {
        tex_texel(T, T.nlevels - 1, 0, 0, out);
        return;
    }
    const float W = (float)T.lw[level], H = (float)T.lh[level];
    s = s * W - 0.5f;
    t = t * H - 0.5f;
    ds0 *= W;
    dt0 *= H;
    ds1 *= W;
    dt1 *= H;
    float A = dt0 * dt0 + dt1 * dt1 + 1;
    float B = -2.f * (ds0 * dt0 + ds1 * dt1);
    float C = ds0 * ds0 + ds1 * ds1 + 1;
    const float invF = 1.f / (A * C - B * B * 0.25f);
    A *= invF;
    B *= invF;
    C *= invF;
    const float det = -B * B + 4.f * A * C;
    const float invDet = 1.f / det;
    const float uSqrt = sqrtf(det * C), vSqrt = sqrtf(A * det);
    const int s0 = (int)ceilf(s - 2.f * invDet * uSqrt);
    const int s1 = (int)floorf(s + 2.f * invDet * uSqrt);
    const int t0 = (int)ceilf(t - 2.f * invDet * vSqrt);
    const int t1 = (int)floorf(t + 2.f * invDet * vSqrt);
    float sum[3] = {0.f, 0.f, 0.f}, sumWts = 0.f;
    for (int it = t0; it <= t1; ++it) {
        const float tt = (float)it - t;
        for (int is = s0; is <= s1; ++is) {
            const float ss = (float)is - s;
            const float r2 = A * ss * ss + B * ss * tt + C * tt * tt;
            if (r2 < 1.f) {
                int li = (int)(r2 * (float)kEwaLut);
                li = li < kEwaLut - 1 ? li : kEwaLut - 1;
                const float weight = T.lut[li];
                float x[3];
                tex_texel(T, level, is, it, x);
                for (int k = 0; k < 3; ++k) sum[k] += x[k] * weight;
                sumWts += weight;
            }
        }
    }
    for (int k = 0; k < 3; ++k) out[k] = sum[k] / sumWts;
}

// MIPMap::Lookup(s, t, width) (mipmap.h:239-255): trilinear
MPSS_HD void tex_lookup_width(const TexView &T, float s, float t, float width, float out[3]) {
    const float level = (float)(uint32_t)(T.nlevels - 1) + tex_log2(width < 1e-8f ? 1e-8f : width);
    if (level < 0.f) {
        tex_triangle(T, 0, s, t, out);
    } else if (level >= (float)(uint32_t)(T.nlevels - 1)) {
        tex_texel(T, T.nlevels - 1, 0, 0, out);
    } else {
        const int il = (int)floorf(level);
        const float delta = level - (float)il;
        float a[3], b[3];
        tex_triangle(T, il, s, t, a);
        tex_triangle(T, il + 1, s, t, b);
        for (int k = 0; k < 3; ++k) out[k] = (1.f - delta) * a[k] + delta * b[k];
    }
}

// MIPMap::Lookup(s, t, ds0, dt0, ds1, dt1) (mipmap.h:272-318): EWA unless "trilinear"
MPSS_HD void tex_lookup(const TexView &T, float s, float t, float ds0, float dt0, float ds1, float dt1,
                        float out[3]) {
    if (T.trilinear) {
        const float m = fmaxf(fmaxf(fabsf(ds0), fabsf(dt0)), fmaxf(fabsf(ds1), fabsf(dt1)));
        tex_lookup_width(T, s, t, 2.f * m, out);
        return;
    }
    if (ds0 * ds0 + dt0 * dt0 < ds1 * ds1 + dt1 * dt1) {
        float x = ds0;
        ds0 = ds1;
        ds1 = x;
        x = dt0;
        dt0 = dt1;
        dt1 = x;
    }
    const float majorLength = sqrtf(ds0 * ds0 + dt0 * dt0);
    float minorLength = sqrtf(ds1 * ds1 + dt1 * dt1);
    if (minorLength * T.max_aniso < majorLength && minorLength > 0.f) {
        const float scale = majorLength / (minorLength * T.max_aniso);
        ds1 *= scale;
        dt1 *= scale;
        minorLength *= scale;
    }
    if (minorLength == 0.f) {
        tex_triangle(T, 0, s, t, out);
        return;
    }
    float lod = (float)(uint32_t)T.nlevels - 1.f + tex_log2(minorLength);
    lod = lod > 0.f ? lod : 0.f;
    const int ilod = (int)floorf(lod);
    const float d = lod - (float)ilod;
    float a[3], b[3];
    tex_ewa(T, ilod, s, t, ds0, dt0, ds1, dt1, a);
    tex_ewa(T, ilod + 1, s, t, ds0, dt0, ds1, dt1, b);
    for (int k = 0; k < 3; ++k) out[k] = (1.f - d) * a[k] + d * b[k];
}

// Surface (u, v) and its screen-space differentials (DifferentialGeometry u, v, dudx ... dvdy).
struct UVDiff {
    float u, v, dudx, dvdx, dudy, dvdy;
};

// ImageTexture::Evaluate (imagemap.cpp:180-189) with UVMapping2D::Map (texture.cpp:88-98); out is
// the MIPMap value (RGB, or out[0] for a float texture) before convertOut
MPSS_HD void tex_eval(const TexView &T, const UVDiff &g, float out[3]) {
    const float s = T.su * g.u + T.du, t = T.sv * g.v + T.dv;
    tex_lookup(T, s, t, T.su * g.dudx, T.sv * g.dvdx, T.su * g.dudy, T.sv * g.dvdy, out);
}

// SolveLinearSystem2x2 (core/transform.cpp:39-49)
MPSS_HD bool solve2x2(const float A[2][2], const float B[2], float &x0, float &x1) {
    const float det = A[0][0] * A[1][1] - A[0][1] * A[1][0];
    if (fabsf(det) < 1e-10f) return false;
    x0 = (A[1][1] * B[0] - A[0][1] * B[1]) / det;
    x1 = (A[0][0] * B[1] - A[1][0] * B[0]) / det;
    if (x0 != x0 || x1 != x1) return false;
    return true;
}

MPSS_HD float v3_at(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

// DifferentialGeometry::ComputeDifferentials (diffgeom.cpp:58-111) for a ray differential with
// rxOrigin = ryOrigin = o (the pinhole camera's; ScaleDifferentials keeps them): dg's point p,
// normal nn (geometric, oriented), dpdu, dpdv -> dudx, dvdx, dudy, dvdy (0 on failure)
MPSS_HD void compute_differentials(V3 p, V3 nn, V3 dpdu, V3 dpdv, V3 o, V3 rxd, V3 ryd, UVDiff &g) {
    g.dudx = g.dvdx = g.dudy = g.dvdy = 0.f;
    const float d = -dot(nn, p);
    const float tx = -(dot(nn, o) + d) / dot(nn, rxd);
    if (tx != tx) return;
    const V3 px = o + rxd * tx;
    const float ty = -(dot(nn, o) + d) / dot(nn, ryd);
    if (ty != ty) return;
    const V3 py = o + ryd * ty;
    int a0, a1;
    if (fabsf(nn.x) > fabsf(nn.y) && fabsf(nn.x) > fabsf(nn.z)) {
        a0 = 1;
        a1 = 2;
    } else if (fabsf(nn.y) > fabsf(nn.z)) {
        a0 = 0;
        a1 = 2;
    } else {
        a0 = 0;
        a1 = 1;
    }
    const float A[2][2] = {{v3_at(dpdu, a0), v3_at(dpdv, a0)}, {v3_at(dpdu, a1), v3_at(dpdv, a1)}};
    const float Bx[2] = {v3_at(px, a0) - v3_at(p, a0), v3_at(px, a1) - v3_at(p, a1)};
    const float By[2] = {v3_at(py, a0) - v3_at(p, a0), v3_at(py, a1) - v3_at(p, a1)};
    if (!solve2x2(A, Bx, g.dudx, g.dvdx)) g.dudx = g.dvdx = 0.f;
    if (!solve2x2(A, By, g.dudy, g.dvdy)) g.dudy = g.dvdy = 0.f;
}

// Material::Bump (material.cpp:47-104) for a UV-mapped float image texture (its value depends on
// (u, v) and the differentials only). dgs: shading geometry (dpdu, dpdv, dndu, dndv, nn);
// ng: dgGeom.nn; flip: ReverseOrientation ^ TransformSwapsHandedness. Returns the bumped dpdu
// and nn. The fork differences over +-du / +-dv; du and dv are negated before the division, so
// the height gradient enters with the opposite sign of pbrt-v2's, and the -u sample is taken at
// (u - du, v + dv) because dgEval.v is left shifted from the +v sample (both kept as is).
MPSS_HD void bump_frame(const TexView &T, const UVDiff &g, V3 dpdu, V3 dpdv, V3 dndu, V3 dndv, V3 nn, V3 ng,
                        int flip, V3 &dpdu_b, V3 &nn_b) {
    float du = fabsf(g.dudx) + fabsf(g.dudy);
    if (du == 0.f) du = .01f;
    float dv = fabsf(g.dvdx) + fabsf(g.dvdy);
    if (dv == 0.f) dv = .01f;
    float x[3];
    UVDiff e = g;
    e.u = g.u + du;
    tex_eval(T, e, x);
    const float upD = x[0];
    e.u = g.u;
    e.v = g.v + dv;
    tex_eval(T, e, x);
    const float vpD = x[0];
    tex_eval(T, g, x);
    const float disp = x[0];
    du = -du;
    e.u = g.u + du;  // dgEval.v still holds v + dv here: the reference does not reset it
    tex_eval(T, e, x);
    const float unD = x[0];
    dv = -dv;
    e.u = g.u;
    e.v = g.v + dv;
    tex_eval(T, e, x);
    const float vnD = x[0];
    dpdu_b = (dpdu + nn * ((upD - unD) / (2 * du))) + dndu * disp;
    const V3 dpdv_b = (dpdv + nn * ((vpD - vnD) / (2 * dv))) + dndv * disp;
    V3 n = normalize(cross(dpdu_b, dpdv_b));
    if (flip) n = n * -1.f;
    nn_b = dot(n, ng) < 0.f ? -n : n;  // Faceforward(n, dgGeom.nn)
}

}  // namespace mpss
