// rho_gpu.hip -- the LayeredSkin rho_hd table on the GPU (row f1; reference
// src/core/multipole.cpp:488-549 RhoTask / ComputeRhoDataFromBxDF).
//
// One workgroup per table entry (1025 by default). Each entry is one MT19937 stream seeded
// 6428263 * id (core/rng.cpp) whose 2 n^2 draws jitter an n x n stratified grid
// (StratifiedSample2D, montecarlo.cpp:158-168) in the order the reference draws them:
//   - the 624-word state lives in LDS; a twist is the standard three-phase parallel
//     recurrence (k in [0,227) reads only old words; [227,454) reads words [0,227) the first
//     phase wrote; [454,624) reads words [227,397) the second phase wrote), every phase
//     reading all operands before any lane writes;
//   - the 624 tempered outputs of a twist are 312 (jx, jy) pairs = strata 312 t .. 312 t + 311,
//     whose estimator terms (rho.h, the render path's BSDF code) the lanes evaluate in parallel
//     into LDS;
//   - the reference sums the terms in sample order with a Kahan sum: lane 0 adds the 312 terms
//     of each twist in order before the next twist's barriers let anyone overwrite them, so
//     every entry is the host build's float result (transcendentals follow the package's
//     double-then-round convention on both sides). No global scratch.
// rho_hh (ComputeRhoHHFromBxDF) is one entry and stays on the host (material.cpp).
#include <vector>

#include "../../include/mpss.h"
#include "common.h"
#include "material.h"
#include "rho.h"

namespace mpss {

namespace {

constexpr int kRhoThreads = 256;
constexpr uint32_t kSkip = 0x7fbadbadu;  // NaN payload marking "pdf <= 0: not added"

__device__ __forceinline__ uint32_t temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

__device__ __forceinline__ uint32_t twist_word(uint32_t k0, uint32_t k1, uint32_t m) {
    const uint32_t y = (k0 & 0x80000000u) | (k1 & 0x7fffffffu);
    return m ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// mt[k] for k in [lo, hi) from the state as it stands (reads first, then one barrier, then writes)
__device__ __forceinline__ void twist_phase(uint32_t *mt, int lo, int hi) {
    const int k = lo + (int)threadIdx.x;
    uint32_t v = 0;
    if (k < hi) v = twist_word(mt[k], mt[(k + 1) % 624], mt[(k + 397) % 624]);
    __syncthreads();
    if (k < hi) mt[k] = v;
    __syncthreads();
}

__global__ __launch_bounds__(kRhoThreads) void rho_hd_kernel(Microfacet m, int n_entries, int sq, float *hd) {
    __shared__ uint32_t mt[624];
    __shared__ float u[624];
    __shared__ uint32_t terms[312];
    const int id = (int)blockIdx.x;
    const int n = sq * sq;
    if (threadIdx.x == 0) {  // RNG::Seed (sequential recurrence, 623 steps)
        uint32_t s = kRhoSeed * (uint32_t)id;
        mt[0] = s;
        for (int i = 1; i < 624; ++i) {
            s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)i;
            mt[i] = s;
        }
    }
    __syncthreads();
    const V3 wo = rho_wo(rho_costheta(id, n_entries));
    KahanF k;  // lane 0's running sum
    for (int base = 0; base < n; base += 312) {
        twist_phase(mt, 0, 227);
        twist_phase(mt, 227, 454);
        twist_phase(mt, 454, 624);
        for (int j = (int)threadIdx.x; j < 624; j += kRhoThreads)
            u[j] = (float)(temper(mt[j]) & 0xffffffu) / (float)(1 << 24);  // RNG::RandomFloat
        __syncthreads();
        const int cnt = n - base < 312 ? n - base : 312;
        for (int j = (int)threadIdx.x; j < cnt; j += kRhoThreads) {
            const int i = base + j;
            float u1, u2, t;
            rho_stratum(i % sq, i / sq, sq, u[2 * j], u[2 * j + 1], u1, u2);
            terms[j] = rho_term(m, wo, u1, u2, t) ? __float_as_uint(t) : kSkip;
        }
        __syncthreads();
        if (threadIdx.x == 0)  // KahanSum in sample order
            for (int j = 0; j < cnt; ++j)
                if (terms[j] != kSkip) k.add(__uint_as_float(terms[j]));
    }
    if (threadIdx.x == 0) hd[id] = k.sum / (float)n;
}

}  // namespace

void build_rho_table_gpu(float roughness, float eta, bool fixed, int n_entries, int sqrt_samples, RhoTable &out,
                         hipStream_t stream) {
    if (n_entries < 2 || sqrt_samples < 1) throw Error(MPSS_ERR_INVALID, "rho table: bad size");
    const Microfacet m = rho_bxdf(roughness, eta, fixed);
    DevBuf<float> hd;
    hd.alloc((size_t)n_entries);
    hipLaunchKernelGGL(rho_hd_kernel, dim3((unsigned)n_entries), dim3(kRhoThreads), 0, stream, m, n_entries,
                       sqrt_samples, hd.ptr);
    MPSS_HIP(hipGetLastError());
    out.hd.assign(n_entries, 0.f);
    MPSS_HIP(hipMemcpyAsync(out.hd.data(), hd.ptr, sizeof(float) * n_entries, hipMemcpyDeviceToHost, stream));
    MPSS_HIP(hipStreamSynchronize(stream));
    out.hh = rho_hh(roughness, eta, fixed, sqrt_samples);
}

}  // namespace mpss
