// mo_wave.h -- the sharded gather's persistent wave-queue kernel (mo_band_wave_kernel) and its
// launch, shared by the translation units that instantiate it: mo_wave_{plain,cg,rgb,rgb_cg}.hip
// each compile one family of variants (per-band tables / common grid, spectral / rgbprofile) so the
// build runs them in parallel; mo_kernel.hip's launch_band picks the family.
#pragma once
#include "mo_kernel.h"
#include "mo_band.h"

namespace mpss {

// ---------------------------------------------------------------------------------------
// Spectrally sharded gather (mo_band.h), in two launches: mo_sort_kernel sorts each 1024-query
// chunk by a Morton key of its query positions into a permutation, then the persistent
// mo_band_wave_kernel deals 64 sorted queries at a time to waves. Workgroup b starts on band group
// b % 8 (one XCD under the round-robin dispatch), so each XCD's L2 holds only its group's tables.
// Every result goes to its query's own slot, so neither the order nor the stealing changes a bit.
// ---------------------------------------------------------------------------------------

struct BandArgs {
    BandTree t;
    const float *__restrict__ queries3;  // q * 3 (batch API) or null
    const float4 *__restrict__ queries4; // {p, *} (render path) or null
    const int *__restrict__ count;       // device query count (nullable: use nq)
    const uint32_t *__restrict__ hit_s;  // render path with several BSSRDF materials: material filter
    int mat;
    int nq;
    float *__restrict__ out;             // batch: out[q * stride + band]
    float4 *__restrict__ out4;           // render: out4[q * 8 + group]
    int out_stride;
    int32_t *__restrict__ counters;      // batch API COUNT: q * 4 (+= per group)
    unsigned long long *__restrict__ counts;  // render COUNT: [kStatStride * kGroups]
    int *__restrict__ work;              // [kGroups] chunk counters (zeroed before the launch)
    float klo[3], kinv[3];               // Morton key quantization (octree root bounds)
    int *perm;                           // chunk-sorted query ids (-1: none), mo_sort_kernel
    int steal;                           // work stealing across groups (GatherOpts::steal)
};

__device__ __forceinline__ bool band_query(const BandArgs &a, int q, float &px, float &py, float &pz) {
    if (a.queries4) {
        const float4 v = a.queries4[q];
        px = v.x;
        py = v.y;
        pz = v.z;
        bool live = v.w >= 0.f;  // render hit list: w < 0 marks hits without a BSSRDF
        if (live && a.hit_s) live = (int)((a.hit_s[q] >> 16) & 0xffu) == a.mat;
        return live;
    }
    px = a.queries3[3 * (size_t)q];
    py = a.queries3[3 * (size_t)q + 1];
    pz = a.queries3[3 * (size_t)q + 2];
    return true;
}


// Step 2: every wave takes 64 consecutive entries of perm at a time from its group's counter and
// walks them to the end on its own -- no workgroup barrier between chunks, so a wave with a short
// traversal does not wait for the slowest wave of its workgroup. Same traversal, same sums.
// Waves per SIMD the register allocation targets: 8 with two workgroups per CU (the 5088-entry near
// field); the 10236-entry near field fills the LDS with one workgroup (4 waves per SIMD), so up to
// 128 VGPRs are free to use -- the bands' row bases then stay in VGPRs for the whole traversal.
// WGT: threads per workgroup.
template <int KLDS, int WGT>
constexpr int wave_kernel_wpe() {
    return (WGT / 64) * (KLDS > 5088 ? 1 : 2) / 4;
}

template <bool COUNT, int KLDS, bool CG, int WGT = 1024, bool RGB = false>
__global__ __launch_bounds__(WGT) __attribute__((amdgpu_waves_per_eu(wave_kernel_wpe<KLDS, WGT>(),
                                                                     wave_kernel_wpe<KLDS, WGT>())))
void mo_band_wave_kernel(BandArgs a) {
    constexpr int ROWF = near_row<KLDS>();
    constexpr bool VROWS = KLDS > 5088;
    // the near field; RGB: its last 28 floats hold the group's FromRGB weights (RgbK; slot 3 is
    // unused for an rgbprofile, and its common grid's LDS split leaves them free)
    __shared__ float lt[KLDS > 0 ? 4 * ROWF : 1];
    __shared__ int next_grp;
    const int tid = (int)threadIdx.x, lane = tid & 63;
    const int nq = a.count ? *a.count : a.nq;
    // steal: a workgroup whose group queue is dry moves on to the next group with units left
    // (groups g + 1, g + 2, ... in turn), reloading its near field; the XCDs whose groups finish
    // first then take over the tail of the slowest group.
    const int home = (int)(blockIdx.x & (kGroups - 1));
    const bool steal = a.steal != 0;
    for (int ph = 0; ph < (steal ? kGroups : 1); ++ph) {
    int grp = home;
    if (steal) {
        if (ph > 0) {
            __syncthreads();  // every wave is done with the previous group's near field
            if (tid == 0) {
                int g = -1;
                for (int k = ph; k < kGroups && g < 0; ++k) {
                    const int c = (home + k) & (kGroups - 1);
                    if (__hip_atomic_load(&a.work[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) * 64 < nq) g = c;
                }
                next_grp = g;
            }
            __syncthreads();
            grp = next_grp;
            if (grp < 0) break;
            // (the loop index stays ph; later phases search from ph onwards, so a group is tried at
            // most once after it was found dry)
        }
    }
    if (CG) {
        // slot j's exact near field: entries 0..klim_j of its band (CommonGrid::lrow, lcnt = klim_j + 1)
        for (int j = 0; j < 4; ++j) {
            const int c = a.t.lband[grp][j];
            const int o = (int)a.t.cg.lrow[grp][j];
            const int n = a.t.cg.lcnt[grp][j];
            for (int k = tid; k < n; k += WGT) lt[o + k] = c >= 0 ? a.t.table[(size_t)c * a.t.L + k] : 0.f;
        }
    } else if (KLDS > 0) {
        // entries 0..kmax of each band, kmax = min(KLDS, L - 2), zeros after (the last two floats of
        // a row are the zero pair of the lanes past the profile end)
        const int kmax = KLDS < a.t.L - 2 ? KLDS : a.t.L - 2;
        for (int i = tid; i < 4 * ROWF - (RGB ? 28 : 0); i += WGT) {
            const int j = i / ROWF, k = i % ROWF, c = a.t.lband[grp][j];
            lt[i] = (c >= 0 && k <= kmax) ? a.t.table[(size_t)c * a.t.L + k] : 0.f;
        }
    }
    // (the common-grid gather's fused FromRGB takes the weights with FromRGB's .94 folded in: from_rgb4_fused)
    if (RGB && tid < 28) lt[4 * ROWF - 28 + tid] = (&a.t.rgb_k[grp].w[0])[tid] * (CG ? .94f : 1.f);
    __syncthreads();  // the near field is read-only from here on
    for (;;) {
        int u = 0;
        if (lane == 0) u = atomicAdd(&a.work[grp], 1);
        u = __builtin_amdgcn_readfirstlane(__shfl(u, 0));
        const int base = u * 64;
        if (base >= nq) break;
        const int q = a.perm[base + lane];
        float px = 0.f, py = 0.f, pz = 0.f;
        const bool live = q >= 0 && band_query(a, q, px, py, pz);
        float acc[4];
        int kn = 0, kp = 0, wn = 0, wp = 0, hist[kHist] = {};
        mo_band_traverse<COUNT, KLDS, VROWS && !CG, CG, RGB>(a.t, grp, px, py, pz, live, acc, kn, kp, wn, wp, hist,
                                                            lt);
        if (live) {
            if (a.out4) {
                a.out4[(size_t)q * kGroups + grp] = make_float4(acc[0], acc[1], acc[2], acc[3]);
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int c = a.t.groups.band[grp][j];
                    if (c >= 0) a.out[(size_t)q * a.out_stride + c] = acc[j];
                }
            }
        }
        if (COUNT) {
            if (a.counters && live) {
                atomicAdd(&a.counters[4 * (size_t)q + 2], kn);
                atomicAdd(&a.counters[4 * (size_t)q + 3], kp);
            }
            if (a.counts) {
                if (kn) atomicAdd(&a.counts[kStatStride * grp], (unsigned long long)kn);
                if (kp) atomicAdd(&a.counts[kStatStride * grp + 1], (unsigned long long)kp);
                if (lane == 0) {
                    atomicAdd(&a.counts[kStatStride * grp + 2], (unsigned long long)wn);
                    atomicAdd(&a.counts[kStatStride * grp + 3], (unsigned long long)wp);
                }
#pragma unroll
                for (int k = 0; k < kHist; ++k)
                    if (hist[k]) atomicAdd(&a.counts[kStatStride * grp + 4 + k], (unsigned long long)hist[k]);
            }
        }
    }
    }
}

// The sharded gather: the sort launch, then the persistent wave-queue launch. opts.near_field picks
// the LDS near field per band: 10236 entries (one 1024-thread workgroup per CU holding the whole
// 160 KB; 32 workgroups per group) or 5088 (two workgroups per CU, 64 per group). opts.steal: a
// workgroup whose group queue runs dry moves on to the next group with work left (C2: 42.5 ->
// 41.2 ms per launch, profiles/r02j_variants.txt). opts.count_noprune (instrumented pass only):
// the reach pruning off, so each group walks exactly the records the reference's Mo() recursion
// reads (bench.py's SURVEY 8d algorithmic bytes).
template <bool COUNT, int KLDS, bool CG = false, int WGT = 1024, bool RGB = false>
void launch_wave(BandArgs a, dim3 grid, bool steal, hipStream_t stream) {
    a.steal = steal ? 1 : 0;
    hipLaunchKernelGGL((mo_band_wave_kernel<COUNT, KLDS, CG, WGT, RGB>), grid, dim3(WGT), 0, stream, a);
}

// one family's four variants: COUNT (instrumented pass) x the 10236 / 5088 near field
template <bool CG, bool RGB>
void launch_wave_family(BandArgs a, dim3 grid, bool count, bool wide, bool steal, hipStream_t stream) {
    if (count && wide)
        launch_wave<true, 10236, CG, 1024, RGB>(a, grid, steal, stream);
    else if (count)
        launch_wave<true, 5088, CG, 1024, RGB>(a, grid, steal, stream);
    else if (wide)
        launch_wave<false, 10236, CG, 1024, RGB>(a, grid, steal, stream);
    else
        launch_wave<false, 5088, CG, 1024, RGB>(a, grid, steal, stream);
}

// mo_wave_plain.hip, mo_wave_cg.hip, mo_wave_rgb.hip, mo_wave_rgb_cg.hip
void launch_wave_plain(BandArgs a, dim3 grid, bool count, bool wide, bool steal, hipStream_t stream);
void launch_wave_cg(BandArgs a, dim3 grid, bool count, bool wide, bool steal, hipStream_t stream);
void launch_wave_rgb(BandArgs a, dim3 grid, bool count, bool wide, bool steal, hipStream_t stream);
void launch_wave_rgb_cg(BandArgs a, dim3 grid, bool count, bool wide, bool steal, hipStream_t stream);

}  // namespace mpss
