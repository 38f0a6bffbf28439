// profile_gpu.hip -- the LayeredSkin multipole profile built on the GPU.
//
// Same computation as material.cpp::channel_profile (MultipoleProfileTask::Run,
// multipole.cpp:241-295 -> MPC_ComputeDiffusionProfile, MultipoleProfileCalculator.cpp:151-346 ->
// MPC_ResampleForUniformDistanceSquaredDistribution :404-426), all 30 channels at once:
//   grid_fill_kernel   the dipole sums of both layers' R and T on the (i <= j) grid octant,
//                      lerp-on-thin-slab, written to the 8 symmetric cells of a 2M x 2M (M = 2N)
//                      zero-padded, origin-centred complex array (ToFrequencyDomain's layout)
//   fft_rows / fft_cols radix-2 FP64 FFTs in LDS (one row, or 4 columns, per workgroup)
//   combine_kernel     R12 = T1 R2 T1 / (1 - R2 R1) + R1 per frequency (CombineLayerProfiles)
//   readout_kernel     unique d^2 = (i^2 + j^2) step^2 samples, first (i, j) in the reference's
//                      loop order wins (:316-330)
//   total_kernel       Kahan sum of the R12 grid (totalReflectance)
//   resample_kernel    uniform-d^2 resampling to twice the sample count (:355-426)
// FP64 throughout the grids and transforms, like the reference's MPC; results agree with the
// host build (and the kissfft-based oracle) to FP64 rounding of differently ordered FFTs.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "material.h"

namespace mpss {

namespace {

constexpr float kPiMPC = 3.141592654f;  // numutil.h:45
constexpr int kPairs = 11;              // dipole pairs -5..5 (DipoleCalculator)

struct DipoleP {
    float d, zpos, zneg, str, alphap;
};
struct ChanSetup {
    float s2;          // step^2 (float)
    double nf;         // step^2 as double
    double lerp[2];    // lerp-on-thin-slab weight per layer
    DipoleP dip[2][kPairs];
};

float fresnel_diffuse_h(float eta) {  // DipoleCalculator.cpp:38-46
    if (eta >= 1.f) return -1.4399f / (eta * eta) + 0.7099f / eta + 0.6681f + 0.0636f * eta;
    const float e2 = eta * eta;
    return -0.4399f + 0.7099f / eta - 0.3319f / e2 + 0.0636f / (e2 * eta);
}

DipoleP make_dipole(float eta0, float etad, float thick, float sa, float sps, int zi, bool lerp) {
    DipoleP p;
    p.d = thick;
    const float spt = sa + sps;
    p.str = sqrtf(3 * sa * spt);
    p.alphap = sps / spt;
    const float F0 = fresnel_diffuse_h(eta0), Fd = fresnel_diffuse_h(etad);
    const float A0 = (1.f + F0) / (1.f - F0), Ad = (1.f + Fd) / (1.f - Fd);
    const float D = 1.f / (3.f * spt);
    const float zb0 = 2.f * A0 * D, zbd = 2.f * Ad * D;
    float l = 1.f / spt;
    if (lerp && l > p.d * .5f) l = p.d * .5f;
    p.zpos = 2.f * (float)zi * (p.d + zb0 + zbd) + l;
    p.zneg = p.zpos - 2.f * (l + zb0);
    return p;
}

__device__ __forceinline__ float dterm(float str, float z, float dsq) {
    const float r = sqrtf(dsq + z * z);
    return z * (1 + str * r) * expf(-str * r) / (r * r * r);
}

// grids: [nch][4][M * M] double2, 0 = R layer 0, 1 = T layer 0, 2 = R layer 1, 3 = T layer 1
__global__ void grid_fill_kernel(const ChanSetup *__restrict__ cs, int nch, int ext, int M, double2 *grids) {
    const int64_t per = (int64_t)(ext + 1) * (ext + 1);
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= per * 2 * nch) return;
    const int ch = (int)(gid / (per * 2)), l = (int)((gid / per) % 2);
    const int i = (int)((gid % per) / (ext + 1)), j = (int)(gid % (ext + 1));
    if (j < i) return;
    const ChanSetup &s = cs[ch];
    const double r2 = ((double)((unsigned)i * (unsigned)i) + (double)((unsigned)j * (unsigned)j)) * s.s2;
    const float r2f = (float)r2;
    double rr = 0., tt = 0.;
    for (int k = 0; k < kPairs; ++k) {
        const DipoleP &p = s.dip[l][k];
        const float rd = p.alphap * (0.25f / kPiMPC) * (dterm(p.str, p.zpos, r2f) - dterm(p.str, p.zneg, r2f));
        const float td = p.alphap * (0.25f / kPiMPC) * (dterm(p.str, p.d - p.zpos, r2f) - dterm(p.str, p.d - p.zneg, r2f));
        rr += rd * s.nf;
        tt += td * s.nf;
    }
    const double lerp = s.lerp[l];
    if (lerp < 1.) {
        rr *= lerp;
        tt *= lerp;
        if (i == 0 && j == 0) tt += 1. - lerp;
    }
    double2 *R = grids + ((size_t)ch * 4 + 2 * l) * (size_t)M * M;
    double2 *T = R + (size_t)M * M;
    const int ri[2] = {i, (M - i) % M}, rj[2] = {j, (M - j) % M};
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b) {
            R[(size_t)ri[a] * M + rj[b]] = make_double2(rr, 0.);
            T[(size_t)ri[a] * M + rj[b]] = make_double2(tt, 0.);
            R[(size_t)rj[b] * M + ri[a]] = make_double2(rr, 0.);
            T[(size_t)rj[b] * M + ri[a]] = make_double2(tt, 0.);
        }
}

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 cdiv(double2 a, double2 b) {
    const double den = b.x * b.x + b.y * b.y;
    return make_double2((a.x * b.x + a.y * b.y) / den, (a.y * b.x - a.x * b.y) / den);
}

// Iterative radix-2 DIT FFT of n points in LDS (bit-reversed load), 256 threads.
__device__ void lds_fft(double2 *a, int n, int logn, const double2 *__restrict__ tw, bool inverse) {
    for (int len = 2, st = n / 2; len <= n; len <<= 1, st >>= 1) {
        const int half = len >> 1;
        for (int b = threadIdx.x; b < n / 2; b += blockDim.x) {
            const int grp = b / half, k = b % half;
            const int i0 = grp * len + k, i1 = i0 + half;
            double2 w = tw[(size_t)k * st];
            if (inverse) w.y = -w.y;
            const double2 u = a[i0], v = cmul(a[i1], w);
            a[i0] = cadd(u, v);
            a[i1] = csub(u, v);
        }
        __syncthreads();
    }
}

__device__ __forceinline__ int bitrev(int x, int logn) { return (int)(__builtin_bitreverse32((unsigned)x) >> (32 - logn)); }

__global__ __launch_bounds__(256) void fft_rows_kernel(double2 *data, int M, int logM, const double2 *tw, int inverse) {
    extern __shared__ double2 a_row[];
    double2 *row = data + (size_t)blockIdx.x * M;
    for (int k = threadIdx.x; k < M; k += blockDim.x) a_row[bitrev(k, logM)] = row[k];
    __syncthreads();
    lds_fft(a_row, M, logM, tw, inverse != 0);
    for (int k = threadIdx.x; k < M; k += blockDim.x) row[k] = a_row[k];
}

// 'cols' adjacent columns per workgroup; grid = (M / cols) x nmat
__global__ __launch_bounds__(256) void fft_cols_kernel(double2 *data, int M, int logM, int cols, const double2 *tw,
                                                       int inverse) {
    extern __shared__ double2 a_col[];
    double2 *mat = data + (size_t)blockIdx.y * M * M;
    const int c0 = blockIdx.x * cols;
    for (int e = threadIdx.x; e < M * cols; e += blockDim.x) {
        const int r = e / cols, cc = e % cols;
        a_col[cc * M + bitrev(r, logM)] = mat[(size_t)r * M + c0 + cc];
    }
    __syncthreads();
    for (int cc = 0; cc < cols; ++cc) lds_fft(a_col + cc * M, M, logM, tw, inverse != 0);
    for (int e = threadIdx.x; e < M * cols; e += blockDim.x) {
        const int r = e / cols, cc = e % cols;
        mat[(size_t)r * M + c0 + cc] = a_col[cc * M + r];
    }
}

// R12 into slot 0 of each channel (CombineLayerProfiles, MultipoleProfileCalculator.cpp:253-280)
__global__ void combine_kernel(double2 *grids, int nch, int M) {
    const int64_t mm = (int64_t)M * M;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= mm * nch) return;
    const int ch = (int)(gid / mm);
    const int64_t k = gid % mm;
    double2 *g = grids + (size_t)ch * 4 * mm;
    const double2 fR1 = g[k], fT1 = g[mm + k], fR2 = g[2 * mm + k];
    const double2 one = csub(make_double2(1., 0.), cmul(fR2, fR1));
    g[k] = cadd(cdiv(cmul(cmul(fT1, fR2), fT1), one), fR1);
}

// unique d^2 entries: value = Re(R12)(i, j) / M^2 as float * 1 / step^2
__global__ void readout_kernel(const double2 *grids, int nch, int M, const int2 *ij, const uint32_t *nsq, int nent,
                               const float *step, float *d_out, float *r_out) {
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= nent * nch) return;
    const int ch = gid / nent, k = gid % nent;
    const double2 *R = grids + (size_t)ch * 4 * M * M;
    const double s = 1.0 / ((double)M * (double)M);
    const float st = step[ch];
    const float denorm = 1.f / (st * st);
    const int2 p = ij[k];
    r_out[gid] = (float)(R[(size_t)p.x * M + p.y].x * s) * denorm;
    d_out[gid] = (float)nsq[k] * st * st;
}

// totalReflectance = Kahan sum over the N x N time-domain grid (numutil.h:236-246), per channel
__global__ __launch_bounds__(256) void total_kernel(const double2 *grids, int M, int N, double *out) {
    __shared__ double part[256];
    const int ch = blockIdx.x;
    const double2 *R = grids + (size_t)ch * 4 * M * M;
    const double s = 1.0 / ((double)M * (double)M);
    const int c = (N - 1) / 2;
    double sum = 0., comp = 0.;
    for (int e = threadIdx.x; e < N * N; e += blockDim.x) {
        const int i = e / N, j = e % N;
        const double x = R[(size_t)((M - c + i) % M) * M + (M - c + j) % M].x * s;
        const double y = x - comp, t = sum + y;
        comp = (t - sum) - y;
        sum = t;
    }
    part[threadIdx.x] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        double tot = 0., cp = 0.;
        for (int k = 0; k < (int)blockDim.x; ++k) {
            const double y = part[k] - cp, t = tot + y;
            cp = (t - tot) - y;
            tot = t;
        }
        out[ch] = tot;
    }
}

// MPC resample at one d^2 (MultipoleProfileCalculator.cpp:355-402)
__device__ float resample_dev(const float *d, const float *R, unsigned len, float dsq) {
    if (dsq > d[len - 1]) return 0.f;
    unsigned lo = 0, hi = len - 1;
    float d2lo = d[lo];
    if (lo + 32 < hi) {
        float d2hi = d[hi];
        do {
            int m = (int)((dsq - d2lo) / (d2hi - d2lo) * (float)(hi - lo));
            m = m < 0 ? 0 : (m > (int)(hi - lo - 1) ? (int)(hi - lo - 1) : m);
            const unsigned mid = (unsigned)m + lo;
            const float d2mid = d[mid];
            if (dsq > d2mid) {
                lo = mid + 1;
                d2lo = d[lo];
            } else {
                hi = mid;
                d2hi = d2mid;
            }
        } while (lo + 32 < hi);
    }
    while (lo < hi && dsq > d2lo) d2lo = d[++lo];
    if (!lo) return R[0];
    float t = (dsq - d[lo - 1]) / (d[lo] - d[lo - 1]);
    t = t < 0.f ? 0.f : (t > 1.f ? 1.f : t);
    if (t != t) t = 0.5f;
    return (1.f - t) * R[lo - 1] + t * R[lo];
}

__global__ void resample_kernel(const float *d, const float *r, int nent, int nch, int tl, float *table) {
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= tl * nch) return;
    const int ch = gid / tl, i = gid % tl;
    const float *dc = d + (size_t)ch * nent, *rc = r + (size_t)ch * nent;
    const float extent = dc[nent - 1];
    const float q = (float)i * extent / (float)(tl - 1);
    table[gid] = resample_dev(dc, rc, (unsigned)nent, q);
}

// first (i, j) per unique i^2 + j^2 in the reference's loop order (i ascending, j >= i), sorted by
// nsq -- depends only on ext, so it is built once per length
struct UniqueList {
    std::vector<int2> ij;
    std::vector<uint32_t> nsq;
};
const UniqueList &unique_list(unsigned ext) {
    static std::mutex mu;
    static std::map<unsigned, UniqueList> cache;
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find(ext);
    if (it != cache.end()) return it->second;
    std::vector<uint8_t> seen((size_t)ext * ext * 2 + 1, 0);
    std::vector<std::pair<uint32_t, int2>> ents;
    for (unsigned i = 0; i <= ext; ++i)
        for (unsigned j = i; i * i + j * j <= ext * ext; ++j) {
            const unsigned n = i * i + j * j;
            if (seen[n]) continue;
            seen[n] = 1;
            ents.emplace_back(n, make_int2((int)i, (int)j));
        }
    std::sort(ents.begin(), ents.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
    UniqueList &u = cache[ext];
    for (auto &e : ents) {
        u.nsq.push_back(e.first);
        u.ij.push_back(e.second);
    }
    return u;
}

unsigned round_up_pow2_u(unsigned v) {
    v--;
    v |= v >> 1; v |= v >> 2; v |= v >> 4; v |= v >> 8; v |= v >> 16;
    return v + 1;
}

}  // namespace

void build_profile_gpu(const LayerParams &lp, int desired_length, bool lerp_thin, ProfileTables &out,
                       hipStream_t stream, int distinct) {
    if (distinct < 1 || distinct > NB) throw Error(-1, "build_profile_gpu: distinct channels out of range");
    const int NC = distinct;  // channels built; channel c >= NC copies channel c % NC
    const int length = (int)round_up_pow2_u((unsigned)desired_length);
    const int N = 2 * length, M = 2 * N;
    int logM = 0;
    while ((1 << logM) < M) ++logM;
    if (M > 4096) throw Error(-1, "build_profile_gpu: desiredlength above 1024 not supported on the GPU path");
    const int ext = length - 1;
    // per-channel setup (channel_profile / layer_grid, material.cpp)
    std::vector<ChanSetup> cs(NC);
    std::vector<float> steps(NC);
    for (int sc = 0; sc < NC; ++sc) {
        float mfp_total = 0.f;
        for (int l = 0; l < 2; ++l) mfp_total += 1.f / (lp.mua[l][sc] + lp.musp[l][sc]);
        const float mfp = mfp_total / (float)2;
        const float step = 12.f * mfp / (float)desired_length;
        steps[sc] = step;
        ChanSetup &c = cs[sc];
        c.s2 = step * step;
        c.nf = c.s2;
        const float up[2] = {lp.eta[0], lp.eta[1] / lp.eta[0]}, lo[2] = {lp.eta[0] / lp.eta[1], lp.eta[1]};
        for (int l = 0; l < 2; ++l) {
            float thick = lp.thickness[l];
            const float mua = lp.mua[l][sc], musp = lp.musp[l][sc];
            const double mfp2 = 2. / (mua + musp);
            double lerp = 1.;
            if (lerp_thin) {
                lerp = (thick < mfp2) ? (1. - exp(-thick * 2. / mfp2)) / (1. - exp(-2.)) : 1.;
                if (thick < 0.01 * mfp2) thick = (float)(0.01 * mfp2);
            }
            c.lerp[l] = lerp;
            for (int k = 0; k < kPairs; ++k) c.dip[l][k] = make_dipole(up[l], lo[l], thick, mua, musp, k - 5, lerp_thin);
        }
    }
    const UniqueList &ul = unique_list((unsigned)ext);
    const int nent = (int)ul.nsq.size();
    const int tl = 2 * nent;
    // twiddles exp(-2 pi i k / M)
    std::vector<double2> tw(M / 2);
    for (int k = 0; k < M / 2; ++k) {
        const double ph = -2.0 * M_PI * (double)k / (double)M;
        tw[k] = make_double2(cos(ph), sin(ph));
    }
    DevBuf<double2> d_tw;
    d_tw.upload(tw.data(), tw.size());
    DevBuf<ChanSetup> d_cs;
    d_cs.upload(cs.data(), cs.size());
    DevBuf<int2> d_ij;
    d_ij.upload(ul.ij.data(), ul.ij.size());
    DevBuf<uint32_t> d_nsq;
    d_nsq.upload(ul.nsq.data(), ul.nsq.size());
    DevBuf<float> d_step, d_d, d_r, d_table;
    d_step.upload(steps.data(), steps.size());
    d_d.alloc((size_t)NC * nent);
    d_r.alloc((size_t)NC * nent);
    d_table.alloc((size_t)NC * tl);
    DevBuf<double> d_tot;
    d_tot.alloc(NC);
    // channels in batches that keep the 4 complex grids per channel within ~3 GB
    const size_t grid_bytes = (size_t)M * M * sizeof(double2);
    const int batch = (int)std::max<size_t>(1, std::min<size_t>(NC, ((size_t)3 << 30) / (4 * grid_bytes)));
    DevBuf<double2> grids;
    grids.alloc((size_t)batch * 4 * M * M);
    const int cols = std::max(1, std::min(4, 131072 / (M * (int)sizeof(double2))));
    MPSS_HIP(hipFuncSetAttribute((const void *)fft_cols_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 cols * M * (int)sizeof(double2)));
    MPSS_HIP(hipFuncSetAttribute((const void *)fft_rows_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 M * (int)sizeof(double2)));
    for (int c0 = 0; c0 < NC; c0 += batch) {
        const int nch = std::min(batch, NC - c0);
        MPSS_HIP(hipMemsetAsync(grids.ptr, 0, (size_t)nch * 4 * grid_bytes, stream));
        const int64_t cells = (int64_t)(ext + 1) * (ext + 1) * 2 * nch;
        hipLaunchKernelGGL(grid_fill_kernel, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0, stream,
                           d_cs.ptr + c0, nch, ext, M, grids.ptr);
        // forward 2-D transforms of all 4 grids
        hipLaunchKernelGGL(fft_rows_kernel, dim3((unsigned)(M * nch * 4)), dim3(256), M * sizeof(double2), stream,
                           grids.ptr, M, logM, d_tw.ptr, 0);
        hipLaunchKernelGGL(fft_cols_kernel, dim3((unsigned)(M / cols), (unsigned)(nch * 4)), dim3(256),
                           (size_t)cols * M * sizeof(double2), stream, grids.ptr, M, logM, cols, d_tw.ptr, 0);
        const int64_t freq = (int64_t)M * M * nch;
        hipLaunchKernelGGL(combine_kernel, dim3((unsigned)((freq + 255) / 256)), dim3(256), 0, stream, grids.ptr, nch,
                           M);
        // inverse transform of R12 (slot 0 of each channel): rows of the slot-0 matrices only
        for (int ch = 0; ch < nch; ++ch) {
            double2 *g = grids.ptr + (size_t)ch * 4 * M * M;
            hipLaunchKernelGGL(fft_rows_kernel, dim3((unsigned)M), dim3(256), M * sizeof(double2), stream, g, M, logM,
                               d_tw.ptr, 1);
            hipLaunchKernelGGL(fft_cols_kernel, dim3((unsigned)(M / cols), 1u), dim3(256),
                               (size_t)cols * M * sizeof(double2), stream, g, M, logM, cols, d_tw.ptr, 1);
        }
        hipLaunchKernelGGL(readout_kernel, dim3((unsigned)((nent * nch + 255) / 256)), dim3(256), 0, stream, grids.ptr,
                           nch, M, d_ij.ptr, d_nsq.ptr, nent, d_step.ptr + c0, d_d.ptr + (size_t)c0 * nent,
                           d_r.ptr + (size_t)c0 * nent);
        hipLaunchKernelGGL(total_kernel, dim3((unsigned)nch), dim3(256), 0, stream, grids.ptr, M, N, d_tot.ptr + c0);
        MPSS_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(resample_kernel, dim3((unsigned)((tl * NC + 255) / 256)), dim3(256), 0, stream, d_d.ptr,
                       d_r.ptr, nent, NC, tl, d_table.ptr);
    MPSS_HIP(hipGetLastError());
    out.length = tl;
    out.table.resize((size_t)NB * tl);
    std::vector<float> dlast(NC);
    std::vector<double> tot(NC);
    MPSS_HIP(hipMemcpyAsync(out.table.data(), d_table.ptr, sizeof(float) * (size_t)NC * tl, hipMemcpyDeviceToHost,
                            stream));
    MPSS_HIP(hipMemcpyAsync(tot.data(), d_tot.ptr, sizeof(double) * NC, hipMemcpyDeviceToHost, stream));
    for (int c = 0; c < NC; ++c)
        MPSS_HIP(hipMemcpyAsync(&dlast[c], d_d.ptr + (size_t)c * nent + nent - 1, sizeof(float), hipMemcpyDeviceToHost,
                                stream));
    MPSS_HIP(hipStreamSynchronize(stream));
    for (int c = NC; c < NB; ++c)
        memcpy(&out.table[(size_t)c * tl], &out.table[(size_t)(c % NC) * tl], sizeof(float) * tl);
    for (int c = 0; c < NB; ++c) {
        const float extent = dlast[c % NC];
        const float last = (float)(tl - 1) * extent / (float)(tl - 1);
        out.spacing[c] = last / (float)(tl - 1);  // multipole.cpp:274-275
        out.rcp[c] = (float)(tl - 1) / last;
        out.total_reflectance[c] = (float)tot[c % NC];
    }
}

}  // namespace mpss
