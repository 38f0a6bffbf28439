// pbrt_math.h -- host/device float math for the render path, written to round exactly like
// pbrt-v2's scalar code (core/geometry.h, core/transform.h, core/montecarlo.h,
// core/reflection.{h,cpp}, shapes/sphere.cpp, shapes/trianglemesh.inl) when compiled with
// -ffp-contract=off:
//   - Cross products are evaluated in double and rounded to float (geometry.h:529-558);
//   - Dot/LengthSquared sum left to right; Normalize multiplies by 1/length (geometry.h:102-106);
//   - transcendentals (sin, cos, exp, log, atan, atan2, acos, pow) are evaluated in double
//     and rounded once to float, the convention the CPU oracle uses too, so host libm and
//     the GPU's OCML agree to the last bit (bar double-rounding ties, ~2^-28 per call).
#pragma once
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>

#define MPSS_HD __host__ __device__ __forceinline__

namespace mpss {

constexpr float kPiF = 3.14159265358979323846f;  // pbrt.h:196 (a float literal)
constexpr float kInvPiF = 0.31830988618379067154f;
constexpr float kInvTwoPiF = 0.15915494309189533577f;
constexpr float kOneMinusEps = 0x1.fffffep-1f;

struct V3 {
    float x, y, z;
};
MPSS_HD V3 v3(float x, float y, float z) { return V3{x, y, z}; }
MPSS_HD V3 operator+(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
MPSS_HD V3 operator-(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
MPSS_HD V3 operator-(V3 a) { return V3{-a.x, -a.y, -a.z}; }
MPSS_HD V3 operator*(V3 a, float s) { return V3{a.x * s, a.y * s, a.z * s}; }
MPSS_HD V3 operator*(float s, V3 a) { return V3{a.x * s, a.y * s, a.z * s}; }
MPSS_HD float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
MPSS_HD float absdot(V3 a, V3 b) { return fabsf(dot(a, b)); }
MPSS_HD float len2(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
MPSS_HD float length(V3 a) { return sqrtf(len2(a)); }
MPSS_HD V3 div(V3 a, float f) {  // VectorBase::operator/ (geometry.h:102-106)
    const float inv = 1.f / f;
    return V3{a.x * inv, a.y * inv, a.z * inv};
}
MPSS_HD V3 normalize(V3 a) { return div(a, length(a)); }
MPSS_HD V3 cross(V3 a, V3 b) {  // geometry.h:529-536, in double
    const double ax = a.x, ay = a.y, az = a.z, bx = b.x, by = b.y, bz = b.z;
    return V3{(float)((ay * bz) - (az * by)), (float)((az * bx) - (ax * bz)), (float)((ax * by) - (ay * bx))};
}
MPSS_HD float dist2(V3 a, V3 b) { return len2(a - b); }

// CoordinateSystem, geometry.h (v1 normalized)
MPSS_HD void coordinate_system(V3 v1, V3 &v2, V3 &v3_) {
    if (fabsf(v1.x) > fabsf(v1.y)) {
        const float inv = 1.f / sqrtf(v1.x * v1.x + v1.z * v1.z);
        v2 = V3{-v1.z * inv, 0.f, v1.x * inv};
    } else {
        const float inv = 1.f / sqrtf(v1.y * v1.y + v1.z * v1.z);
        v2 = V3{0.f, v1.z * inv, -v1.y * inv};
    }
    v3_ = cross(v1, v2);
}

// Double-evaluated transcendentals rounded once to float (see header comment)
MPSS_HD float m_sin(float x) { return (float)sin((double)x); }
MPSS_HD float m_cos(float x) { return (float)cos((double)x); }
MPSS_HD float m_exp(float x) { return (float)exp((double)x); }
MPSS_HD float m_log(float x) { return (float)log((double)x); }
MPSS_HD float m_atan(float x) { return (float)atan((double)x); }
MPSS_HD float m_atan2(float y, float x) { return (float)atan2((double)y, (double)x); }
MPSS_HD float m_acos(float x) { return (float)acos((double)x); }
MPSS_HD float m_pow(float x, float y) { return (float)pow((double)x, (double)y); }

// 4x4 row-major transforms (core/transform.h:190-237)
MPSS_HD V3 xform_point(const float *m, V3 p) {
    const float xp = m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3];
    const float yp = m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7];
    const float zp = m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11];
    const float wp = m[12] * p.x + m[13] * p.y + m[14] * p.z + m[15];
    if (wp == 1.f) return V3{xp, yp, zp};
    const float inv = 1.f / wp;  // PointBase::operator/=
    return V3{xp * inv, yp * inv, zp * inv};
}
MPSS_HD V3 xform_vector(const float *m, V3 v) {
    return V3{m[0] * v.x + m[1] * v.y + m[2] * v.z, m[4] * v.x + m[5] * v.y + m[6] * v.z,
              m[8] * v.x + m[9] * v.y + m[10] * v.z};
}
MPSS_HD V3 xform_normal(const float *minv, V3 n) {  // uses the inverse matrix, transposed
    return V3{minv[0] * n.x + minv[4] * n.y + minv[8] * n.z, minv[1] * n.x + minv[5] * n.y + minv[9] * n.z,
              minv[2] * n.x + minv[6] * n.y + minv[10] * n.z};
}

// ---------------------------------------------------------------- low-discrepancy samples
// montecarlo.h:278-302
MPSS_HD float van_der_corput(uint32_t n, uint32_t scramble) {
    n = __builtin_bitreverse32(n) ^ scramble;
    const float v = (float)((n >> 8) & 0xffffff) / (float)(1 << 24);
    return v < kOneMinusEps ? v : kOneMinusEps;
}
// Sobol2's generator has columns v_0 = 2^31, v_{i+1} = v_i ^ (v_i >> 1): column i is row i of Pascal's
// triangle mod 2, top bit first. By Lucas' theorem, bit 31 - j of the XOR of the columns of n's set
// bits is the parity of n's bits at the positions i that contain j (i & j == j) -- a superset-sum
// transform of n in five shift-xor steps, then bit-reversed: the loop's value for every n, without
// its n-dependent trip count (tests/test_sampler_replay.py checks the transform against the loop for
// every 16-bit n; the GPU image tests against the oracle's loop).
MPSS_HD float sobol2(uint32_t n, uint32_t scramble) {
    n ^= (n >> 1) & 0x55555555u;
    n ^= (n >> 2) & 0x33333333u;
    n ^= (n >> 4) & 0x0f0f0f0fu;
    n ^= (n >> 8) & 0x00ff00ffu;
    n ^= (n >> 16) & 0x0000ffffu;
    scramble ^= __builtin_bitreverse32(n);
    const float r = (float)((scramble >> 8) & 0xffffff) / (float)(1 << 24);
    return r < kOneMinusEps ? r : kOneMinusEps;
}

// Counter-based scrambles (replaces pbrt's per-task MT19937 streams; DESIGN.md "replay mode").
MPSS_HD uint32_t mix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x7feb352du;
    h ^= h >> 15;
    h *= 0x846ca68bu;
    h ^= h >> 16;
    return h;
}
MPSS_HD uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
    return mix32(a ^ mix32(b ^ mix32(c + 0x9e3779b9u)));
}

// Sample dimensions of one camera sample (pbrt's Sample: image, lens, time, then the
// integrator's 1D/2D arrays requested by MultipoleSubsurfaceIntegrator::RequestSamples,
// multipolesubsurface.cpp:238-252 [file lines]).
enum SampleDim : uint32_t {
    DIM_IMAGE = 0,      // 2D
    DIM_LIGHT_POS = 2,  // 2D x nLightSamples, per light
    DIM_LIGHT_COMP = 3, // 1D
    DIM_BSDF_DIR = 4,   // 2D
    DIM_BSDF_COMP = 5,  // 1D
    DIM_IRR_POS = 6,    // irradiance preprocess, per light
    DIM_IRR_COMP = 7,
    DIM_STRIDE = 8
};

}  // namespace mpss
