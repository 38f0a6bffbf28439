// material.cpp -- LayeredSkin parse-time precompute (host, multithreaded). See material.h
// for the reference functions followed. The layer grids and their frequency-domain
// combination are FP64 exactly as the reference's MPC; the 2-D transforms use this
// file's own radix-2 FFT (not kissfft), so tables agree with the oracle to FP64
// rounding, which tests/test_profile.py bounds.
#include "material.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <complex>
#include <cstring>
#include <thread>

#include "rho.h"
#include "spectral.h"

namespace mpss {

// ------------------------------------------------------------ skin coefficients
namespace {
constexpr int WLD_N = 61;  // core/material.h:96
inline float wld_lambda(int i) { return 400.f + 5.f * (float)i; }

const float kOxy[WLD_N] = {  // skincoeffs.cpp:44-52
    266200, 331450, 466800, 523100, 480400, 351100, 246100, 149050, 102600, 78880, 62820, 51525,
    44480, 38440, 33210, 29480, 26630, 24925, 23680, 22155, 20930, 20185, 20040, 20715, 24200,
    30885, 39960, 48335, 53240, 50985, 43020, 35650, 32610, 35210, 44500, 54425, 50100, 30620,
    14400, 6681.5f, 3200, 1958.5f, 1506, 1166.5f, 942, 740.8f, 610, 495.6f, 442, 397.7f, 368,
    340.3f, 319.6f, 305.6f, 294, 283.8f, 277.6f, 273.6f, 276, 280.6f, 290};
const float kDeoxy[WLD_N] = {  // skincoeffs.cpp:64-72
    223300, 261950, 304000, 353200, 407600, 471500, 528600, 549600, 413300, 259950, 103300,
    33435, 23390, 18700, 16160, 14920, 14550, 15375, 16680, 18650, 20860, 23285, 25770, 28680,
    31590, 35170, 39040, 42840, 46590, 50490, 53410, 54530, 53790, 49700, 45070, 40905, 37020,
    33590, 28320, 21185, 14680, 12040, 9444, 7553.5f, 6510, 5763.5f, 5149, 4666.5f, 4345,
    4026.5f, 3750, 3481.5f, 3227, 3011, 2795, 2591, 2408, 2224.5f, 2052, 1923.5f, 1794};

// WLDValue::FromSampled (core/material.h:118-141): piecewise-linear resampling onto the WLD grid
void wld_resample(const float *vals, float out[WLD_N]) {
    int idx = 0;
    float l0 = 0.f, l1 = wld_lambda(0), v0 = vals[0], v1 = vals[0];
    for (int i = 0; i < WLD_N; ++i) {
        const float lam = wld_lambda(i);
        while (lam > l1 && idx < WLD_N - 1) {
            ++idx;
            l0 = l1;
            l1 = wld_lambda(idx);
            v0 = v1;
            v1 = vals[idx];
        }
        out[i] = (lam <= l1) ? lerpf_((lam - l0) / (l1 - l0), v0, v1) : v1;
    }
}

void wld_to_bands(const float w[WLD_N], float out[NB]) {
    float lam[WLD_N];
    for (int i = 0; i < WLD_N; ++i) lam[i] = wld_lambda(i);
    spectrum_from_sampled(lam, w, WLD_N, out);
}
}  // namespace

void skin_layer_params(const SkinParams &p, LayerParams &out) {
    float base[WLD_N], eu[WLD_N], pheo[WLD_N], sct[WLD_N];
    for (int i = 0; i < WLD_N; ++i) {
        const float wl = wld_lambda(i);
        base[i] = 0.244f + 85.3f * expf(-(wl - 154.f) / 66.2f);            // skincoeffs.h:46-50
        eu[i] = 6.6e11f * powf(wl, -3.33f);                                 // :54-58
        pheo[i] = 2.9e15f * powf(wl, -4.75f);                               // :60-64
        sct[i] = 2e12f * powf(wl, -4.f) + 147.4f * powf(wl, (float)-0.22);  // :79-81,119-130
    }
    float oxy[WLD_N], deo[WLD_N];
    wld_resample(kOxy, oxy);
    wld_resample(kDeoxy, deo);
    const float unit = p.nmperunit / 1e7f;  // layeredskin.cpp:47
    const float kblood = 2.303f / 64500.f * 150.f;
    float ea[WLD_N], es[WLD_N], da[WLD_N], ds[WLD_N];
    for (int i = 0; i < WLD_N; ++i) {
        const float mel = eu[i] * p.f_eu + pheo[i] * (1 - p.f_eu);
        ea[i] = (mel * p.f_mel + base[i] * (1 - p.f_mel)) * unit;                    // mua_epi
        es[i] = sct[i] * unit;                                                        // musp_epi
        const float blood = (oxy[i] * p.f_ohg + deo[i] * (1.f - p.f_ohg)) * kblood;  // mua_blood
        da[i] = (blood * p.f_blood + base[i] * (1 - p.f_blood)) * unit;               // mua_derm
        ds[i] = (sct[i] * 0.5f) * unit;                                               // musp_derm
    }
    wld_to_bands(ea, out.mua[0]);
    wld_to_bands(es, out.musp[0]);
    wld_to_bands(da, out.mua[1]);
    wld_to_bands(ds, out.musp[1]);
    for (int l = 0; l < 2; ++l) {
        out.thickness[l] = p.thickness_nm[l] / p.nmperunit;
        out.eta[l] = p.ior[l];
    }
}

// ------------------------------------------------------------ multipole profile
namespace {

constexpr float kPiMPC = 3.141592654f;  // numutil.h:45 (the MPC's own PI)

float fresnel_diffuse(float eta) {  // DipoleCalculator.cpp:38-46
    if (eta >= 1.f) return -1.4399f / (eta * eta) + 0.7099f / eta + 0.6681f + 0.0636f * eta;
    const float e2 = eta * eta;
    return -0.4399f + 0.7099f / eta - 0.3319f / e2 + 0.0636f / (e2 * eta);
}

struct Dipole {  // DipoleCalculator.cpp:52-91
    float d, zpos, zneg, str, alphap;
    Dipole(float eta0, float etad, float thick, float sa, float sps, int zi, bool lerp) {
        d = thick;
        const float spt = sa + sps;
        str = sqrtf(3 * sa * spt);
        alphap = sps / spt;
        const float F0 = fresnel_diffuse(eta0), Fd = fresnel_diffuse(etad);
        const float A0 = (1.f + F0) / (1.f - F0), Ad = (1.f + Fd) / (1.f - Fd);
        const float D = 1.f / (3.f * spt);
        const float zb0 = 2.f * A0 * D, zbd = 2.f * Ad * D;
        float l = 1.f / spt;
        if (lerp && l > d * .5f) l = d * .5f;
        zpos = 2.f * (float)zi * (d + zb0 + zbd) + l;
        zneg = zpos - 2.f * (l + zb0);
    }
    float term(float z, float dsq) const {
        const float r = sqrtf(dsq + z * z);
        return z * (1 + str * r) * expf(-str * r) / (r * r * r);
    }
    float Rd(float dsq) const { return alphap * (0.25f / kPiMPC) * (term(zpos, dsq) - term(zneg, dsq)); }
    float Td(float dsq) const {
        return alphap * (0.25f / kPiMPC) * (term(d - zpos, dsq) - term(d - zneg, dsq));
    }
};

// Layer grid: N x N doubles, centre (N-1)/2 (MultipoleProfileCalculator.cpp:151-230)
void layer_grid(float ior_up, float ior_lo, float thick, float mua, float musp, float step, bool lerp_thin, int N,
                std::vector<double> &R, std::vector<double> &T) {
    R.assign((size_t)N * N, 0.0);
    T.assign((size_t)N * N, 0.0);
    const double mfp2 = 2. / (mua + musp);
    double lerp = 1.;
    if (lerp_thin) {
        lerp = (thick < mfp2) ? (1. - exp(-thick * 2. / mfp2)) / (1. - exp(-2.)) : 1.;
        if (thick < 0.01 * mfp2) thick = (float)(0.01 * mfp2);
    }
    const int c = (N - 1) / 2, ext = c;
    std::vector<Dipole> dips;
    for (int pair = -5; pair <= 5; ++pair) dips.emplace_back(ior_up, ior_lo, thick, mua, musp, pair, lerp_thin);
    const float s2 = step * step;
    const double nf = s2;
    auto at = [&](std::vector<double> &M, int r, int col) -> double & { return M[(size_t)r * N + col]; };
    for (int i = 0; i <= ext; ++i)
        for (int j = i; j <= ext; ++j) {
            const double r2 = ((double)((unsigned)i * (unsigned)i) + (double)((unsigned)j * (unsigned)j)) * s2;
            double &rr = at(R, c + i, c + j), &tt = at(T, c + i, c + j);
            for (const Dipole &dp : dips) {
                rr += dp.Rd((float)r2) * nf;
                tt += dp.Td((float)r2) * nf;
            }
        }
    if (lerp < 1.) {
        for (int i = 0; i <= ext; ++i)
            for (int j = i; j <= ext; ++j) {
                at(R, c + i, c + j) *= lerp;
                at(T, c + i, c + j) *= lerp;
            }
        at(T, c, c) += 1. - lerp;
    }
    for (int i = 1; i <= ext; ++i)
        for (int j = 0; j < i; ++j) {
            at(R, c + i, c + j) = at(R, c + j, c + i);
            at(T, c + i, c + j) = at(T, c + j, c + i);
        }
    for (int i = 0; i <= ext; ++i)
        for (int j = 0; j <= ext; ++j) {
            const double rv = at(R, c + i, c + j), tv = at(T, c + i, c + j);
            at(R, c - i, c + j) = rv; at(R, c + i, c - j) = rv; at(R, c - i, c - j) = rv;
            at(T, c - i, c + j) = tv; at(T, c + i, c - j) = tv; at(T, c - i, c - j) = tv;
        }
}

using cd = std::complex<double>;

// In-place iterative radix-2 DIT FFT over n points with stride 1.
struct FFT1 {
    int n, logn;
    std::vector<cd> tw;       // e^{-2 pi i k / n}
    std::vector<int> rev;
    explicit FFT1(int n_) : n(n_) {
        logn = 0;
        while ((1 << logn) < n) ++logn;
        tw.resize(n / 2);
        for (int k = 0; k < n / 2; ++k) {
            const double ph = -2.0 * M_PI * (double)k / (double)n;
            tw[k] = cd(cos(ph), sin(ph));
        }
        rev.resize(n);
        for (int i = 0; i < n; ++i) {
            int r = 0;
            for (int b = 0; b < logn; ++b)
                if (i & (1 << b)) r |= 1 << (logn - 1 - b);
            rev[i] = r;
        }
    }
    void run(cd *a, bool inverse) const {
        for (int i = 0; i < n; ++i)
            if (i < rev[i]) std::swap(a[i], a[rev[i]]);
        for (int len = 2; len <= n; len <<= 1) {
            const int half = len >> 1, step = n / len;
            for (int i = 0; i < n; i += len)
                for (int j = 0; j < half; ++j) {
                    cd w = tw[(size_t)j * step];
                    if (inverse) w = std::conj(w);
                    const cd u = a[i + j], v = a[i + j + half] * w;
                    a[i + j] = u + v;
                    a[i + j + half] = u - v;
                }
        }
    }
};

// 2-D FFT of an M x M complex array (rows, then columns through a column buffer).
void fft2(const FFT1 &f, std::vector<cd> &A, int M, bool inverse) {
    for (int r = 0; r < M; ++r) f.run(&A[(size_t)r * M], inverse);
    std::vector<cd> col(M);
    for (int c = 0; c < M; ++c) {
        for (int r = 0; r < M; ++r) col[r] = A[(size_t)r * M + c];
        f.run(col.data(), inverse);
        for (int r = 0; r < M; ++r) A[(size_t)r * M + c] = col[r];
    }
}

// Circularly centre an N x N grid (centre (N-1)/2) on the origin of a 2N x 2N array and transform
// (ToFrequencyDomain + ScaleAndShift, MultipoleProfileCalculator.cpp:233-240, numutil.h:201-213).
void to_freq(const FFT1 &f, const std::vector<double> &P, int N, std::vector<cd> &out) {
    const int M = 2 * N, c = (N - 1) / 2;
    out.assign((size_t)M * M, cd(0, 0));
    for (int i = 0; i < N; ++i) {
        const int ii = (M - c + i) % M;
        for (int j = 0; j < N; ++j) out[(size_t)ii * M + (M - c + j) % M] = cd(P[(size_t)i * N + j], 0);
    }
    fft2(f, out, M, false);
}

// Inverse transform, 1/M^2 scaling and un-centring (ToTimeDomain, :243-250; numutil.h:214-226).
void to_time(const FFT1 &f, std::vector<cd> &F, int N, std::vector<double> &out) {
    const int M = 2 * N, c = (N - 1) / 2;
    fft2(f, F, M, true);
    const double s = 1.0 / ((double)M * (double)M);
    out.assign((size_t)N * N, 0.0);
    for (int i = 0; i < N; ++i) {
        const int ii = (M - c + i) % M;
        for (int j = 0; j < N; ++j) out[(size_t)i * N + j] = F[(size_t)ii * M + (M - c + j) % M].real() * s;
    }
}

double kahan(const std::vector<double> &v) {  // numutil.h:236-246
    double sum = 0, comp = 0;
    for (double x : v) {
        const double y = x - comp, t = sum + y;
        comp = (t - sum) - y;
        sum = t;
    }
    return sum;
}

// resample (MultipoleProfileCalculator.cpp:355-402)
float resample_at(const std::vector<float> &d, const std::vector<float> &R, float dsq) {
    const unsigned len = (unsigned)d.size();
    if (dsq > d[len - 1]) return 0.f;
    unsigned lo = 0, hi = len - 1;
    float d2lo = d[lo];
    if (lo + 32 < hi) {
        float d2hi = d[hi];
        do {
            int m = (int)((dsq - d2lo) / (d2hi - d2lo) * (float)(hi - lo));
            m = std::min(std::max(m, 0), (int)(hi - lo - 1));
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

unsigned round_up_pow2(unsigned v) {
    v--;
    v |= v >> 1; v |= v >> 2; v |= v >> 4; v |= v >> 8; v |= v >> 16;
    return v + 1;
}

// One spectral channel (MultipoleProfileTask::Run, multipole.cpp:241-295)
void channel_profile(const LayerParams &lp, int sc, int desired, bool lerp_thin, std::vector<float> &table,
                     float &rcp, float &spacing, float &total) {
    float mfp_total = 0.f;
    for (int l = 0; l < 2; ++l) mfp_total += 1.f / (lp.mua[l][sc] + lp.musp[l][sc]);
    const float mfp = mfp_total / (float)2;
    const float step = 12.f * mfp / (float)desired;
    const int length = (int)round_up_pow2((unsigned)desired);
    const int N = 2 * length;
    std::vector<double> R0, T0, R1, T1;
    // MPC_ComputeDiffusionProfile, :294-314 (two layers)
    layer_grid(lp.eta[0], lp.eta[0] / lp.eta[1], lp.thickness[0], lp.mua[0][sc], lp.musp[0][sc], step, lerp_thin, N,
               R0, T0);
    layer_grid(lp.eta[1] / lp.eta[0], lp.eta[1], lp.thickness[1], lp.mua[1][sc], lp.musp[1][sc], step, lerp_thin, N,
               R1, T1);
    {  // CombineLayerProfiles, :253-280: R12 = R1 + T1 R2 T1 / (1 - R2 R1)
        FFT1 f(2 * N);
        std::vector<cd> fR1, fR2, fT1, fT2;
        to_freq(f, R0, N, fR1);
        to_freq(f, R1, N, fR2);
        to_freq(f, T0, N, fT1);
        to_freq(f, T1, N, fT2);
        T1.clear();
        R1.clear();
        std::vector<cd> fR12(fR1.size()), &fT12 = fT2;
        for (size_t k = 0; k < fR1.size(); ++k) {
            const cd one = cd(1, 0) - fR2[k] * fR1[k];
            fR12[k] = fT1[k] * fR2[k] * fT1[k] / one + fR1[k];
            fT12[k] = fT1[k] * fT2[k] / one;
        }
        fR1.clear(); fR2.clear(); fT1.clear();
        to_time(f, fR12, N, R0);
        to_time(f, fT12, N, T0);
    }
    // unique d^2 = (i^2 + j^2) step^2 entries, i <= j, first insertion wins (:316-330)
    const unsigned c = (unsigned)length - 1, ext = c;
    const float denorm = 1.f / (step * step);
    std::vector<uint8_t> seen((size_t)ext * ext * 2 + 1, 0);
    std::vector<std::pair<unsigned, float>> ents;
    for (unsigned i = 0; i <= ext; ++i)
        for (unsigned j = i; i * i + j * j <= ext * ext; ++j) {
            const unsigned nsq = i * i + j * j;
            if (seen[nsq]) continue;
            seen[nsq] = 1;
            ents.emplace_back(nsq, (float)R0[(size_t)(c + i) * N + (c + j)] * denorm);
        }
    std::sort(ents.begin(), ents.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
    std::vector<float> d(ents.size()), r(ents.size());
    for (size_t k = 0; k < ents.size(); ++k) {
        d[k] = (float)ents[k].first * step * step;
        r[k] = ents[k].second;
    }
    total = (float)kahan(R0);
    // MPC_ResampleForUniformDistanceSquaredDistribution (:404-426), target = 2 * length
    const unsigned tl = (unsigned)d.size() * 2;
    const float extent = d.back();
    table.resize(tl);
    std::vector<float> nd(tl);
    for (unsigned i = 0; i < tl; ++i) {
        const float q = (float)i * extent / (float)(tl - 1);
        nd[i] = q;
        table[i] = resample_at(d, r, q);
    }
    spacing = nd[tl - 1] / (float)(tl - 1);   // multipole.cpp:274-275
    rcp = (float)(tl - 1) / nd[tl - 1];
}

template <class F>
void parallel_for(int n, int nthreads, F &&fn) {
    if (nthreads <= 0) nthreads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::atomic<int> next{0};
    std::vector<std::thread> th;
    for (int t = 0; t < std::min(nthreads, n); ++t)
        th.emplace_back([&] {
            for (int i; (i = next.fetch_add(1)) < n;) fn(i);
        });
    for (auto &x : th) x.join();
}

// 2-D FFT with the rows, then the columns, spread over threads (the 4096^2 transforms of the
// desiredLength-1024 reference profiles).
void fft2_par(const FFT1 &f, std::vector<cd> &A, int M, bool inverse) {
    parallel_for(M, 0, [&](int r) { f.run(&A[(size_t)r * M], inverse); });
    constexpr int kCols = 8;
    parallel_for(M / kCols, 0, [&](int cb) {
        std::vector<cd> col((size_t)M);
        for (int c = cb * kCols; c < (cb + 1) * kCols; ++c) {
            for (int r = 0; r < M; ++r) col[r] = A[(size_t)r * M + c];
            f.run(col.data(), inverse);
            for (int r = 0; r < M; ++r) A[(size_t)r * M + c] = col[r];
        }
    });
}

void to_freq_par(const FFT1 &f, const std::vector<double> &P, int N, std::vector<cd> &out) {
    const int M = 2 * N, c = (N - 1) / 2;
    out.assign((size_t)M * M, cd(0, 0));
    for (int i = 0; i < N; ++i) {
        const int ii = (M - c + i) % M;
        for (int j = 0; j < N; ++j) out[(size_t)ii * M + (M - c + j) % M] = cd(P[(size_t)i * N + j], 0);
    }
    fft2_par(f, out, M, false);
}

void to_time_par(const FFT1 &f, std::vector<cd> &F, int N, std::vector<double> &out) {
    const int M = 2 * N, c = (N - 1) / 2;
    fft2_par(f, F, M, true);
    const double s = 1.0 / ((double)M * (double)M);
    out.assign((size_t)N * N, 0.0);
    for (int i = 0; i < N; ++i) {
        const int ii = (M - c + i) % M;
        for (int j = 0; j < N; ++j) out[(size_t)i * N + j] = F[(size_t)ii * M + (M - c + j) % M].real() * s;
    }
}

}  // namespace

// MPC_ComputeDiffusionProfile for any layer stack (MultipoleProfileCalculator.cpp:294-346):
// layer grids (ComputeLayerProfile :151-230), pairwise frequency-domain combination with the
// time-domain crop between combinations (CombineLayerProfiles :253-280 via ToTimeDomain
// :243-250), the unique-d^2 readout of R and T (:316-345; the first (i, j) of each d^2 wins) and
// the Kahan totals of both grids.
void mpc_compute(const MpcLayer *L, int n, float step, int desired_length, bool lerp_thin, MpcOutput &out) {
    if (n < 1) throw Error(-1, "mpc: no layers");
    const int length = (int)round_up_pow2((unsigned)desired_length);
    const int N = 2 * length;
    std::vector<double> R0, T0, R1, T1;
    layer_grid(L[0].ior, n > 1 ? L[0].ior / L[1].ior : L[0].ior, L[0].thickness, L[0].mua, L[0].musp, step,
               lerp_thin, N, R0, T0);
    if (n > 1) {
        FFT1 f(2 * N);
        for (int i = 1; i < n; ++i) {
            const float lo = n > i + 1 ? L[i].ior / L[i + 1].ior : L[i].ior;
            layer_grid(L[i].ior / L[i - 1].ior, lo, L[i].thickness, L[i].mua, L[i].musp, step, lerp_thin, N, R1, T1);
            std::vector<cd> fR1, fR2, fT1, fT2;
            to_freq_par(f, R0, N, fR1);
            to_freq_par(f, R1, N, fR2);
            to_freq_par(f, T0, N, fT1);
            to_freq_par(f, T1, N, fT2);
            std::vector<cd> &fR12 = fR2, &fT12 = fT2;  // in place: each k reads its own inputs first
            for (size_t k = 0; k < fR1.size(); ++k) {
                const cd r1 = fR1[k], r2 = fR2[k], t1 = fT1[k], t2 = fT2[k];
                const cd one = cd(1, 0) - r2 * r1;  // fOneR2R1 = 1 - fR2 fR1
                fR12[k] = t1 * r2 * t1 / one + r1;
                fT12[k] = t1 * t2 / one;
            }
            fR1.clear();
            fT1.clear();
            to_time_par(f, fR12, N, R0);
            to_time_par(f, fT12, N, T0);
        }
    }
    const unsigned c = (unsigned)length - 1, ext = c;
    const float denorm = 1.f / (step * step);
    std::vector<uint8_t> seen((size_t)ext * ext * 2 + 1, 0);
    struct Ent {
        unsigned nsq;
        float r, t;
    };
    std::vector<Ent> ents;
    for (unsigned i = 0; i <= ext; ++i)
        for (unsigned j = i; i * i + j * j <= ext * ext; ++j) {
            const unsigned nsq = i * i + j * j;
            if (seen[nsq]) continue;
            seen[nsq] = 1;
            const size_t at = (size_t)(c + i) * N + (c + j);
            ents.push_back(Ent{nsq, (float)R0[at] * denorm, (float)T0[at] * denorm});
        }
    std::sort(ents.begin(), ents.end(), [](const Ent &a, const Ent &b) { return a.nsq < b.nsq; });
    out.dsq.resize(ents.size());
    out.refl.resize(ents.size());
    out.trans.resize(ents.size());
    for (size_t k = 0; k < ents.size(); ++k) {
        out.dsq[k] = (float)ents[k].nsq * step * step;
        out.refl[k] = ents[k].r;
        out.trans[k] = ents[k].t;
    }
    out.total_reflectance = (float)kahan(R0);
    out.total_transmittance = (float)kahan(T0);
}

// MPC_ResampleDistribution (MultipoleProfileCalculator.cpp:429-449): the profile at distances
// samplePoints (d^2 = point * point in float) by the interpolation search of resample().
void mpc_resample_distribution(const MpcOutput &in, int n, const float *points, float *refl, float *trans) {
    for (int i = 0; i < n; ++i) {
        const float dsq = points[i] * points[i];
        refl[i] = resample_at(in.dsq, in.refl, dsq);
        trans[i] = resample_at(in.dsq, in.trans, dsq);
    }
}

// MultipoleReferenceTask::Run (renderers/mcprofile.cpp:381-425): the multipole profile of the
// MC scene's layers at desiredLength 1024 with step extent * 1.01 / 1024, sampled at the ring
// centres (i + .5) * extent / nSegments.
void mc_reference_profile(const MpcLayer *layers, int n, double extent, int nsegments, bool lerp_thin, double *refl,
                          double *trans, double *total_r, double *total_t) {
    MpcOutput o;
    const int desired = 1024;
    mpc_compute(layers, n, (float)(extent * 1.01 / desired), desired, lerp_thin, o);
    *total_r = o.total_reflectance;
    *total_t = o.total_transmittance;
    std::vector<float> pts(nsegments), r(nsegments), t(nsegments);
    for (int i = 0; i < nsegments; ++i) pts[i] = (float)((i + .5) * (extent / nsegments));
    mpc_resample_distribution(o, nsegments, pts.data(), r.data(), t.data());
    for (int i = 0; i < nsegments; ++i) {
        refl[i] = r[i];
        trans[i] = t[i];
    }
}

// ComputeMonteCarloProfile's conversion of one band's ring profile (multipole.cpp:328-355): the
// rings as an MPC_Output at d^2 = (float)(((i + .5) * extent / n)^2), values cast to float,
// resampled to `target` entries uniform in d^2.
void profile_from_rings(const double *refl, int nseg, double extent, int target, std::vector<float> &table,
                        float &rcp, float &spacing) {
    std::vector<float> d(nseg), r(nseg);
    for (int i = 0; i < nseg; ++i) {
        const double x = (i + 0.5) * extent / (double)nseg;
        d[i] = (float)(x * x);
        r[i] = (float)refl[i];
    }
    const float ext = d.back();
    table.resize(target);
    float last = 0.f;
    for (int i = 0; i < target; ++i) {
        const float q = (float)i * ext / (float)(target - 1);
        last = q;
        table[i] = resample_at(d, r, q);
    }
    spacing = last / (float)(target - 1);
    rcp = (float)(target - 1) / last;
}

void build_profile(const LayerParams &lp, int desired_length, bool lerp_thin, ProfileTables &out, int nthreads,
                   int distinct) {
    if (distinct < 1 || distinct > NB) throw Error(-1, "build_profile: distinct channels out of range");
    std::vector<std::vector<float>> tabs(NB);
    parallel_for(distinct, nthreads, [&](int sc) {
        channel_profile(lp, sc, desired_length, lerp_thin, tabs[sc], out.rcp[sc], out.spacing[sc],
                        out.total_reflectance[sc]);
    });
    for (int c = distinct; c < NB; ++c) {
        tabs[c] = tabs[c % distinct];
        out.rcp[c] = out.rcp[c % distinct];
        out.spacing[c] = out.spacing[c % distinct];
        out.total_reflectance[c] = out.total_reflectance[c % distinct];
    }
    out.length = (int)tabs[0].size();
    for (int c = 1; c < NB; ++c)
        if ((int)tabs[c].size() != out.length) throw Error(-2, "profile channel lengths differ");
    out.table.resize((size_t)NB * out.length);
    for (int c = 0; c < NB; ++c) memcpy(&out.table[(size_t)c * out.length], tabs[c].data(), sizeof(float) * out.length);
}

// ------------------------------------------------------------ rho_hd table
namespace {
struct MT {  // MT19937 (core/rng.cpp)
    uint32_t mt[624];
    int i;
    explicit MT(uint32_t s) {
        mt[0] = s;
        for (i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    }
    uint32_t next() {
        if (i >= 624) {
            for (int k = 0; k < 624; ++k) {
                const uint32_t y = (mt[k] & 0x80000000u) | (mt[(k + 1) % 624] & 0x7fffffffu);
                mt[k] = mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
            }
            i = 0;
        }
        uint32_t y = mt[i++];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= y >> 18;
        return y;
    }
    float uniform() { return (float)(next() & 0xffffff) / (float)(1 << 24); }  // RNG::RandomFloat
};

void stratified(std::vector<float> &s, int n, MT &rng) {  // StratifiedSample2D, montecarlo.cpp:158-168
    s.resize((size_t)2 * n * n);
    float *p = s.data();
    for (int y = 0; y < n; ++y)
        for (int x = 0; x < n; ++x) {
            const float jx = rng.uniform(), jy = rng.uniform();
            rho_stratum(x, y, n, jx, jy, p[0], p[1]);
            p += 2;
        }
}
}  // namespace

// ComputeRhoHHFromBxDF, multipole.cpp:466-480; BxDF::rho(n, s1, s2), reflection.cpp:637-652
float rho_hh(float roughness, float eta, bool fixed, int sqrt_samples) {
    const Microfacet m = rho_bxdf(roughness, eta, fixed);
    const int n = sqrt_samples * sqrt_samples;
    MT rng(kRhoSeed * 3u * 7u);
    std::vector<float> s1, s2;
    stratified(s1, sqrt_samples, rng);
    stratified(s2, sqrt_samples, rng);
    KahanF k;
    for (int i = 0; i < n; ++i) {
        const float z = s1[2 * i], r = sqrtf(std::max(0.f, 1.f - z * z)), phi = 2 * kPiF * s1[2 * i + 1];
        const V3 wo = {r * m_cos(phi), r * m_sin(phi), z};  // UniformSampleHemisphere
        V3 wi;
        float pdf = 0.f;
        beckmann_sample(m, wo, s2[2 * i], s2[2 * i + 1], wi, pdf);
        float f = 0.f;
        if (wo.z * wi.z > 0.f) {
            const MfTerms t = microfacet_terms(m, wo, wi);
            if (!t.zero) f = 1.f * t.D * t.G * t.F / t.den;
        }
        if (pdf > 0.) k.add(f * fabsf(wi.z) * fabsf(wo.z) / (kInvTwoPiF * pdf));
    }
    return k.sum / (kPiF * n);
}

void irradiance_points_profile(float radius, ProfileTables &p, RhoTable &rho) {
    const float area = (float)(M_PI * radius * radius);  // float area = M_PI * radius * radius (double product)
    const float v = 1.f / area;                          // fullSpectrum[i] / area, fullSpectrum = Spectrum(1)
    p.length = 2;
    p.table.assign((size_t)NB * 2, v);
    for (int c = 0; c < NB; ++c) {
        p.spacing[c] = radius * radius;
        p.rcp[c] = 1.f / p.spacing[c];
        p.total_reflectance[c] = 1.f;
    }
    rho.hd.assign(2, 0.f);
    rho.hh = 0.f;
}

void build_rho_table(float roughness, float eta, bool fixed, int n_entries, int sqrt_samples, RhoTable &out,
                     int nthreads) {
    const Microfacet m = rho_bxdf(roughness, eta, fixed);
    out.hd.assign(n_entries, 0.f);
    const int n = sqrt_samples * sqrt_samples;
    parallel_for(n_entries, nthreads, [&](int id) {  // RhoTask::Run, multipole.cpp:506-518
        MT rng(kRhoSeed * (uint32_t)id);
        std::vector<float> s;
        stratified(s, sqrt_samples, rng);
        const V3 wo = rho_wo(rho_costheta(id, n_entries));
        KahanF k;
        for (int i = 0; i < n; ++i) {
            float t;
            if (rho_term(m, wo, s[2 * i], s[2 * i + 1], t)) k.add(t);
        }
        out.hd[id] = k.sum / (float)n;
    });
    out.hh = rho_hh(roughness, eta, fixed, sqrt_samples);
}

}  // namespace mpss
