// mo_kernel.hip -- the Mo() hierarchical irradiance gather on CDNA4 (gfx950).
//
// Computes, for each query point p, SubsurfaceOctreeNode::Mo(octreeBounds, p, ...)
// (reference src/integrators/diffusionutil.h:175-210) with the multipole profile
// Rd(d^2) of MultipoleProfileData::reflectance (src/core/multipole.cpp:60-113).
//
// Mapping: one wave64 = two queries; each 32-lane half-wave owns one query and lane
// c = lane & 31 owns spectral band c (30 bands, lanes 30/31 idle). The traversal is
// stackless over the pre-order node array (skip pointers, octree.h), so control flow is
// uniform inside a half-wave. Every node record and every spectral row is read by the
// half-wave as one coalesced 128-B line (Et/E) plus one broadcast 64-B header.
//
// Summation order is the reference's recursion order: S[d][lane] in LDS holds the
// running sum of the children of the open node at depth d-1; a finished subtree is
// folded into its parent level on the way back up. With FP contraction disabled
// (-ffp-contract=off) every product and sum rounds exactly as the reference's scalar
// code, so the result is bit-identical to the CPU oracle.
//
// Exact pruning: sampleProfile returns exactly 0 once d^2 * rcpDsqSpacing >= L-1
// (multipole.cpp:63-66). Every point of a subtree and its clusters' centroids lie inside the
// node's box, so if the box's squared distance to p times the smallest rcp over bands is past
// L-1 (with a 1e-4 relative margin that dominates float rounding of the two distances), the
// whole subtree adds only +0 terms in the reference and is skipped here without changing a
// bit of the result. The COUNT variant reports both the reference traversal's visits and the
// pruned traversal's visits (SURVEY.md 8d counters).
#include "dipole.h"
#include "mo_kernel.h"
#include "spectral.h"
#include "mo_packet.h"
#include "mo_wave.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

namespace mpss {

namespace {

struct MoArgs {
    const NodeHdr *__restrict__ nodes;
    const float *__restrict__ node_et;
    const float4 *__restrict__ pt_hdr;
    const float *__restrict__ pt_e;
    const float *__restrict__ table;    // [NB][L]
    const float *__restrict__ rcp;      // [NB]
    const float *__restrict__ queries;  // q * 3
    float *__restrict__ out;            // q * out_stride
    int32_t *__restrict__ counters;     // COUNT: q * 4
    int L, n_nodes, nq, out_stride;
    float max_error, prune_f;           // prune when d2box * rcp_min >= prune_f
    float rcp_min;
    const float *__restrict__ dipole;   // FN_DIPOLE: [4][NB] zpos, zneg, sigma_tr, k (dipole.h)
    // render path (instead of queries): queries4[i] = {p, w} (w < 0: no BSSRDF), i < *count, and
    // with hit_s the material filter; out[i * out_stride + c]
    const float4 *__restrict__ queries4;
    const int *__restrict__ count;
    const uint32_t *__restrict__ hit_s;
    int mat;
};

// Rd functors of the reference-order gather: the tabulated spectral profile, the closed-form
// single dipole (DiffusionReflectance), and the RGB profile (rgbprofile: three tables, Rd =
// SampledSpectrum::FromRGB(reflectance) of the three lookups, multipole.cpp:85-107).
enum { FN_TABLE = 0, FN_DIPOLE = 1, FN_RGB = 2 };

// rgbRefl2Spect{White, Cyan, Magenta, Yellow, Red, Green, Blue} (spectrum.cpp, SampledSpectrum::Init)
__constant__ float kRefl[7][NB] = {MPSS_BAND_RGBREFL2SPECTWHITE_INIT, MPSS_BAND_RGBREFL2SPECTCYAN_INIT,
                                   MPSS_BAND_RGBREFL2SPECTMAGENTA_INIT, MPSS_BAND_RGBREFL2SPECTYELLOW_INIT,
                                   MPSS_BAND_RGBREFL2SPECTRED_INIT, MPSS_BAND_RGBREFL2SPECTGREEN_INIT,
                                   MPSS_BAND_RGBREFL2SPECTBLUE_INIT};

// Band c of SampledSpectrum::FromRGB(rgb, SPECTRUM_REFLECTANCE) (spectrum.cpp:103-186): the same
// float operations as the 30-band code (spectral.cpp spectrum_from_rgb), one band.
__device__ __forceinline__ float from_rgb_band(float R, float G, float B, int c) {
    enum { W = 0, CY = 1, MG = 2, YE = 3, RD = 4, GR = 5, BL = 6 };
    float r = 0.f;
    if (R <= G && R <= B) {
        r += kRefl[W][c] * R;
        if (G <= B) { r += kRefl[CY][c] * (G - R); r += kRefl[BL][c] * (B - G); }
        else { r += kRefl[CY][c] * (B - R); r += kRefl[GR][c] * (G - B); }
    } else if (G <= R && G <= B) {
        r += kRefl[W][c] * G;
        if (R <= B) { r += kRefl[MG][c] * (R - G); r += kRefl[BL][c] * (B - R); }
        else { r += kRefl[MG][c] * (B - G); r += kRefl[RD][c] * (R - B); }
    } else {
        r += kRefl[W][c] * B;
        if (R <= G) { r += kRefl[YE][c] * (R - B); r += kRefl[GR][c] * (G - R); }
        else { r += kRefl[YE][c] * (G - B); r += kRefl[RD][c] * (R - G); }
    }
    const float v = r * (float).94;
    return v < 0.f ? 0.f : v;  // Clamp(0, INFINITY)
}

__device__ __forceinline__ float rd_lerp(const float *__restrict__ tb, float f) {
    const uint32_t s = (uint32_t)f;
    const float t = f - (float)s;
    const float a = tb[s], b = tb[s + 1];
    return (1.f - t) * a + t * b;
}

// MultipoleProfileData::reflectance with isRGBProfile (multipole.cpp:85-107): sampleProfile of
// the R, G, B tables, then band c of Spectrum::FromRGBSpectrum
__device__ __forceinline__ float rgb_rd(const float *__restrict__ table, int L, const float rcp3[3], float lm1, float d2,
                                        int c) {
    float v[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float f = d2 * rcp3[k];
        v[k] = f < lm1 ? rd_lerp(table + (size_t)k * L, f) : 0.f;
    }
    return from_rgb_band(v[0], v[1], v[2], c);
}

__device__ __forceinline__ float box_d2(float px, float py, float pz, const NodeHdr &h) {
    const float bx = fmaxf(fmaxf(h.bminx - px, px - h.bmaxx), 0.f);
    const float by = fmaxf(fmaxf(h.bminy - py, py - h.bmaxy), 0.f);
    const float bz = fmaxf(fmaxf(h.bminz - pz, pz - h.bmaxz), 0.f);
    return bx * bx + by * by + bz * bz;
}

// FN_DIPOLE: the Rd functor is the closed-form single dipole (DiffusionReflectance, dipole.h)
// instead of the tabulated profile; it never returns an exact 0 past a range, so nothing is
// pruned. FN_RGB: a.table holds the R, G, B profiles ([3][L]) and a.rcp their rcpDsqSpacing; the
// three lookups are wave-uniform per half-wave, each lane converts them to its band.
template <int MAXD, bool COUNT, int FN>
__global__ __launch_bounds__(256) void mo_gather_kernel(MoArgs a) {
    constexpr bool DIP = FN == FN_DIPOLE;
    __shared__ float S[4][MAXD + 1][64];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int c = lane & 31;
    const int q = ((int)blockIdx.x * 4 + wave) * 2 + (lane >> 5);
    bool active = q < a.nq;
    float(*St)[64] = S[wave];

    float px = 0.f, py = 0.f, pz = 0.f;
    if (a.queries4) {  // render path: the compacted hit list (count on the device) and its filter
        if (active) active = q < *a.count;
        if (active) {
            const float4 v = a.queries4[q];
            px = v.x;
            py = v.y;
            pz = v.z;
            active = v.w >= 0.f && (!a.hit_s || (int)((a.hit_s[q] >> 16) & 0xffu) == a.mat);
        }
    } else if (active) {
        px = a.queries[3 * (size_t)q];
        py = a.queries[3 * (size_t)q + 1];
        pz = a.queries[3 * (size_t)q + 2];
    }
    const float rcp = (FN == FN_TABLE && c < NB) ? a.rcp[c] : INFINITY;
    float rcp3[3] = {0.f, 0.f, 0.f};
    if (FN == FN_RGB)
        for (int k = 0; k < 3; ++k) rcp3[k] = a.rcp[k];
    const float lm1 = (float)(a.L - 1);
    const float *__restrict__ tb = a.table + (size_t)(c < NB ? c : 0) * a.L;
    float dzp = 0.f, dzn = 0.f, dtr = 0.f, dk = 0.f;
    if (DIP) {
        const int cc = c < NB ? c : 0;
        dzp = a.dipole[cc];
        dzn = a.dipole[NB + cc];
        dtr = a.dipole[2 * NB + cc];
        dk = a.dipole[3 * NB + cc];
    }

    int node = active ? 0 : a.n_nodes;
    int dlast = 0;
    St[0][lane] = 0.f;
    // COUNT: reference visits (no pruning) and pruned-kernel visits
    int ref_nodes = 0, ref_pts = 0, k_nodes = 0, k_pts = 0, pruned_until = 0;

    while (node < a.n_nodes) {
        const NodeHdr h = a.nodes[node];
        const int d = h.depth;
        while (dlast > d) {  // close finished subtrees (return from the recursion)
            St[dlast - 1][lane] += St[dlast][lane];
            --dlast;
        }
        int next = h.skip;
        const bool prune = box_d2(px, py, pz, h) * a.rcp_min >= a.prune_f;
        if (COUNT) {
            ++ref_nodes;
            if (node >= pruned_until) {
                ++k_nodes;
                if (prune) pruned_until = h.skip;
            }
        } else if (prune) {
            node = next;
            continue;
        }
        if (!(h.flags & NODE_BLACK)) {
            const float dx = px - h.px, dy = py - h.py, dz = pz - h.pz;
            const float d2 = dx * dx + dy * dy + dz * dz;
            const float dw = h.sum_area / d2;
            const bool inside = px >= h.bminx && px <= h.bmaxx && py >= h.bminy && py <= h.bmaxy &&
                                pz >= h.bminz && pz <= h.bmaxz;
            if (dw < a.max_error && !inside) {
                if (DIP) {
                    St[d][lane] += dipole_band(dzp, dzn, dtr, dk, d2) * a.node_et[(size_t)node * ROW + c];
                } else if (FN == FN_RGB) {
                    St[d][lane] += rgb_rd(a.table, a.L, rcp3, lm1, d2, c < NB ? c : 0) * a.node_et[(size_t)node * ROW + c];
                } else {
                    const float f = d2 * rcp;
                    if (f < lm1) St[d][lane] += rd_lerp(tb, f) * a.node_et[(size_t)node * ROW + c];
                }
            } else if (h.leaf_first >= 0) {
                float acc = 0.f;
                for (int i = 0; i < h.leaf_count; ++i) {
                    const int k = h.leaf_first + i;
                    const float4 ph = a.pt_hdr[k];
                    if (__builtin_signbit(ph.w)) continue;  // E is black
                    if (COUNT) {
                        ++ref_pts;
                        if (node >= pruned_until) ++k_pts;
                    }
                    const float ex = px - ph.x, ey = py - ph.y, ez = pz - ph.z;
                    if (DIP) {
                        acc += dipole_band(dzp, dzn, dtr, dk, ex * ex + ey * ey + ez * ez) *
                               a.pt_e[(size_t)k * ROW + c] * ph.w;
                        continue;
                    }
                    if (FN == FN_RGB) {
                        acc += rgb_rd(a.table, a.L, rcp3, lm1, ex * ex + ey * ey + ez * ez, c < NB ? c : 0) *
                               a.pt_e[(size_t)k * ROW + c] * ph.w;
                        continue;
                    }
                    const float f = (ex * ex + ey * ey + ez * ez) * rcp;
                    if (f < lm1) acc += rd_lerp(tb, f) * a.pt_e[(size_t)k * ROW + c] * ph.w;
                }
                St[d][lane] += acc;
            } else {  // open the node: recurse into its children
                next = node + 1;
                St[d + 1][lane] = 0.f;
                dlast = d + 1;
            }
        }
        node = next;
    }
    while (dlast > 0) {
        St[dlast - 1][lane] += St[dlast][lane];
        --dlast;
    }
    if (active && c < NB) a.out[(size_t)q * a.out_stride + c] = St[0][lane];
    if (COUNT && active && c == 0) {
        int4 v = {ref_nodes, ref_pts, k_nodes, k_pts};
        reinterpret_cast<int4 *>(a.counters)[q] = v;
    }
}

// ---------------------------------------------------------------------------------------
// Packet kernel (default): one wave64 = a packet of 8 queries x 8 band-groups of 4 bands.
// The 8 queries (consecutive in the caller's order: samples of one pixel / neighbouring
// shading points) walk the UNION of their pruned traversals once: node headers and leaf
// point headers are wave-uniform scalar loads, Et/E rows are one 128-B line per wave, and
// each lane owns 4 bands of one query. A query that does not open node j (it pruned it,
// took its cluster contribution, or the node is black) sits out until j's skip index.
// Per query the visited node set, the decisions and every product are those of the
// reference; only the order of the final float additions differs (one running sum per
// band instead of the recursion's per-level sums), so results agree with the reference
// order to float reassociation (tests bound it at 2e-5 relative; north star: 1e-4).
// ---------------------------------------------------------------------------------------
template <bool COUNT>
__global__ __launch_bounds__(256) void mo_packet_kernel(MoArgs a, int nblocks) {
    const int lb = xcd_remap((int)blockIdx.x, nblocks);
    const int lane = threadIdx.x & 63;
    const int g = lane >> 3, k = lane & 7;
    const int q = (lb * 4 + (int)(threadIdx.x >> 6)) * 8 + g;
    const bool valid = q < a.nq;
    float px = 0.f, py = 0.f, pz = 0.f;
    if (valid) {
        px = a.queries[3 * (size_t)q];
        py = a.queries[3 * (size_t)q + 1];
        pz = a.queries[3 * (size_t)q + 2];
    }
    PacketTree t{a.nodes, a.node_et, a.pt_hdr, a.pt_e, a.table, a.rcp, a.L, a.n_nodes, a.max_error, a.prune_f,
                 a.rcp_min};
    float acc[4];
    int kn = 0, kp = 0, un = 0;
    mo_packet_traverse<COUNT>(t, px, py, pz, valid, k, acc, kn, kp, &un);
    if (valid) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = 4 * k + j;
            if (c < NB) a.out[(size_t)q * a.out_stride + c] = acc[j];
        }
        if (COUNT && k == 0) {
            int4 v = {un, 0, kn, kp};  // packet: wave (union) iterations, -, own nodes, own points
            reinterpret_cast<int4 *>(a.counters)[q] = v;
        }
    }
}

// Step 1: each 1024-query chunk sorted by the Morton key of its live queries, written as a
// permutation: perm[base + i] = the i-th query
// of the chunk in key order, -1 past the live ones. Chunks at or past the query count write nothing.
__global__ __launch_bounds__(1024) void mo_sort_kernel(BandArgs a) {
    __shared__ unsigned long long keys[1024];
    const int tid = (int)threadIdx.x;
    const int nq = a.count ? *a.count : a.nq;
    const int base = (int)blockIdx.x * 1024;
    if (base >= nq) return;  // uniform over the block
    float px = 0.f, py = 0.f, pz = 0.f;
    const bool in = base + tid < nq && band_query(a, base + tid, px, py, pz);
    const uint32_t key = in ? morton30(px, py, pz, a.klo, a.kinv) : 0xffffffffu;  // dead last
    keys[tid] = ((unsigned long long)key << 32) | (unsigned)tid;
    __syncthreads();
    for (int k = 2; k <= 1024; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            const int ixj = tid ^ j;
            if (ixj > tid) {
                const unsigned long long x = keys[tid], y = keys[ixj];
                if ((x > y) == ((tid & k) == 0)) {
                    keys[tid] = y;
                    keys[ixj] = x;
                }
            }
            __syncthreads();
        }
    const unsigned long long mine = keys[tid];
    a.perm[base + tid] = (mine >> 32) != 0xffffffffull ? base + (int)(mine & 0xffffffffull) : -1;
}

void launch_band(BandArgs a, int nq_max, const DeviceOctree &t, bool count, const GatherOpts &opts,
                 hipStream_t stream) {
    if (nq_max <= 0) return;
    if (!a.perm) throw Error(-2, "launch_band: the sharded gather needs its permutation scratch");
    if (opts.near_field != 10236 && opts.near_field != 5088)
        throw Error(-1, "mo_near_field must be 10236 or 5088");
    for (int k = 0; k < 3; ++k) {
        const float ext = t.bmax[k] - t.bmin[k];
        a.klo[k] = t.bmin[k];
        a.kinv[k] = ext > 0.f ? 1023.99f / ext : 0.f;
    }
    MPSS_HIP(hipMemsetAsync(a.work, 0, sizeof(int) * kGroups, stream));
    if (count && opts.count_noprune) a.t.prune_f = INFINITY;
    const int chunks = (nq_max + 1023) / 1024;
    hipLaunchKernelGGL(mo_sort_kernel, dim3((unsigned)chunks), dim3(1024), 0, stream, a);
    const bool wide = opts.near_field == 10236;
    const int cap = wide ? 32 : 64;  // resident workgroups per group: 1 or 2 per CU of an XCD
    const dim3 grid((unsigned)((chunks < cap ? chunks : cap) * kGroups));
    if (!wide) a.t.cg = a.t.cg_half;  // the grid built for the 5088 layout's LDS split
    const bool cg = opts.common_grid && a.t.cg.on && a.t.cg.tab;
    if (a.t.rgb_refl && cg)  // rgbprofile: three lookups per record, FromRGB into the group's bands
        launch_wave_rgb_cg(a, grid, count, wide, opts.steal, stream);
    else if (a.t.rgb_refl)
        launch_wave_rgb(a, grid, count, wide, opts.steal, stream);
    else if (cg)
        launch_wave_cg(a, grid, count, wide, opts.steal, stream);
    else
        launch_wave_plain(a, grid, count, wide, opts.steal, stream);
    MPSS_HIP(hipGetLastError());
}

// area: null, or the points' headers -- then each value is scaled by the point's area (|w|: its sign
// bit marks a black E), the common-grid gather's E * area (mo_band.h cg_combine)
__global__ void band_permute_kernel(const float *__restrict__ rows, int n, BandGroups g, const float4 *__restrict__ area,
                                    float4 *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)n * kGroups) return;
    const int grp = (int)(i / n), r = (int)(i % n);
    const float *row = rows + (size_t)r * ROW;
    const float w = area ? fabsf(area[r].w) : 1.f;
    float v[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) v[s] = g.band[grp][s] >= 0 ? (area ? row[g.band[grp][s]] * w : row[g.band[grp][s]]) : 0.f;
    out[i] = make_float4(v[0], v[1], v[2], v[3]);
}

BandTree band_tree(const DeviceOctree &t, const BandLayout &l, const DeviceProfile &p, float max_error) {
    if (!same_groups(l.groups, p.groups)) throw Error(-2, "band layout does not match the profile's band groups");
    BandTree bt;
    bt.nodes = t.nodes.ptr;
    bt.band_et = l.et.ptr;
    bt.pt_hdr = t.pt_hdr.ptr;
    bt.band_e = l.e.ptr;
    bt.band_ew = l.ew.ptr;
    bt.table = p.table.ptr;
    bt.groups = p.groups;
    for (int g = 0; g < kGroups; ++g) {
        bt.grcp_max[g] = 0.f;
        for (int s = 0; s < 4; ++s) {
            bt.grcp[g][s] = p.groups.band[g][s] >= 0 ? p.host_rcp[p.groups.band[g][s]] : 0.f;
            bt.grcp_max[g] = bt.grcp[g][s] > bt.grcp_max[g] ? bt.grcp[g][s] : bt.grcp_max[g];
        }
    }
    bt.leaf_r2 = (t.leaf_r2.ptr && t.leaf_r2_error == max_error) ? t.leaf_r2.ptr : nullptr;
    bt.cg = p.cg;
    bt.cg_half = p.cg_half;
    for (int g = 0; g < kGroups; ++g)
        for (int s2 = 0; s2 < 4; ++s2) bt.lband[g][s2] = p.groups.band[g][s2];
    bt.rgb_refl = nullptr;
    if (p.rgb_refl.ptr) {  // rgbprofile: rows 0..2 (R, G, B) in every group, one reach for all
        float rmin = INFINITY, rmax = 0.f;
        for (int k = 0; k < 3; ++k) {
            rmin = std::min(rmin, p.host_rcp[k]);
            rmax = std::max(rmax, p.host_rcp[k]);
        }
        for (int g = 0; g < kGroups; ++g) {
            for (int s2 = 0; s2 < 4; ++s2) {
                bt.lband[g][s2] = s2 < 3 ? s2 : -1;
                bt.grcp[g][s2] = s2 < 3 ? p.host_rcp[s2] : 0.f;
            }
            bt.grcp_max[g] = rmax;
            bt.groups.rcp_min[g] = rmin;
        }
        bt.rgb_refl = p.rgb_refl.ptr;  // (p.cg: the grid of the three profiles, set_rgb)
        // the groups' FromRGB weights: rgbRefl2Spect{White, Cyan, Magenta, Yellow, Red, Green, Blue}
        static const float refl[7][NB] = {MPSS_BAND_RGBREFL2SPECTWHITE_INIT, MPSS_BAND_RGBREFL2SPECTCYAN_INIT,
                                          MPSS_BAND_RGBREFL2SPECTMAGENTA_INIT, MPSS_BAND_RGBREFL2SPECTYELLOW_INIT,
                                          MPSS_BAND_RGBREFL2SPECTRED_INIT, MPSS_BAND_RGBREFL2SPECTGREEN_INIT,
                                          MPSS_BAND_RGBREFL2SPECTBLUE_INIT};
        for (int g = 0; g < kGroups; ++g)
            for (int s2 = 0; s2 < 4; ++s2) {
                const int c = p.groups.band[g][s2];
                auto at = [&](int t) { return c >= 0 ? refl[t][c] : 0.f; };
                bt.rgb_k[g].w[s2] = at(0);
                for (int t = 0; t < 3; ++t) {
                    bt.rgb_k[g].x[t][s2] = at(1 + t);  // Cyan, Magenta, Yellow
                    bt.rgb_k[g].y[t][s2] = at(4 + t);  // Red, Green, Blue
                }
            }
    }
    if (!bt.leaf_r2)
        for (int g = 0; g < kGroups; ++g) bt.cg.lds_r2[g] = bt.cg_half.lds_r2[g] = 0.f;
    bt.L = p.L;
    bt.n_nodes = t.n_nodes;
    bt.n_points = t.n_points;
    bt.max_error = max_error;
    bt.prune_f = (p.rcp_min > 0.f) ? (float)(p.L - 1) * 1.0001f : INFINITY;
    if (!(p.rcp_min > 0.f))
        for (int g = 0; g < kGroups; ++g) bt.groups.rcp_min[g] = 0.f;  // rcp <= 0: no pruning
    return bt;
}

template <int MAXD, int FN>
void launch_t(const MoArgs &a, bool count, hipStream_t s) {
    const int waves = (a.nq + 1) / 2;
    const int blocks = (waves + 3) / 4;
    if (blocks == 0) return;
    if (count)
        hipLaunchKernelGGL((mo_gather_kernel<MAXD, true, FN>), dim3(blocks), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((mo_gather_kernel<MAXD, false, FN>), dim3(blocks), dim3(256), 0, s, a);
}

template <int FN>
void launch_exact(const MoArgs &a, int max_depth, bool count, hipStream_t s) {
    if (max_depth < 16)
        launch_t<16, FN>(a, count, s);
    else if (max_depth < 32)
        launch_t<32, FN>(a, count, s);
    else if (max_depth < 64)
        launch_t<64, FN>(a, count, s);
    else
        throw Error(-2, "octree deeper than 63 levels is not supported by the gather kernel");
    MPSS_HIP(hipGetLastError());
}

}  // namespace

// The device copy moves each leaf's black points (E == 0: every kernel skips them, they add
// nothing) behind its other points, keeping the others' order, and records the count of the
// rest in NodeHdr::pad's low half (a leaf holds at most 8 points), so the sharded gather's leaf loop
// needs no per-point test. (The high half: ensure_leaf_r2's leaf code.)
void DeviceOctree::upload(const FlatOctree &t) {
    std::vector<NodeHdr> hdr = t.hdr;
    std::vector<float> ph(t.pt_hdr.size()), pe(t.pt_e.size());
    std::vector<int> pidx(t.pt_index.size());
    for (NodeHdr &h : hdr) {
        h.pad = 0;
        if (h.leaf_first < 0) continue;
        int o = h.leaf_first;
        for (int pass = 0; pass < 2; ++pass)
            for (int i = 0; i < h.leaf_count; ++i) {
                const size_t k = (size_t)h.leaf_first + i;
                const bool blk = std::signbit(t.pt_hdr[4 * k + 3]);
                if (blk != (pass == 1)) continue;
                memcpy(&ph[4 * (size_t)o], &t.pt_hdr[4 * k], 4 * sizeof(float));
                memcpy(&pe[(size_t)o * ROW], &t.pt_e[k * ROW], ROW * sizeof(float));
                pidx[o] = t.pt_index[k];
                ++o;
                if (pass == 0) ++h.pad;
            }
    }
    layouts.clear();
    leaf_r2_error = -1.f;
    nodes.upload(hdr.data(), hdr.size());
    node_et.upload(t.node_et.data(), t.node_et.size());
    pt_hdr.upload(reinterpret_cast<const float4 *>(ph.data()), ph.size() / 4);
    pt_e.upload(pe.data(), pe.size());
    pt_index.upload(pidx.data(), pidx.size());
    n_nodes = (int)t.hdr.size();
    n_points = (int)t.pt_index.size();
    max_depth = t.max_depth;
    for (int k = 0; k < 3; ++k) {
        bmin[k] = t.bmin[k];
        bmax[k] = t.bmax[k];
    }
}

void DeviceProfile::upload(const float *tab, int len, const float *rcp_, bool snake) {
    // two zero floats after the last band: the sharded gather's read for "past the profile end"
    const size_t n = (size_t)NB * len;
    if (table.n != n + 2) table.alloc(n + 2);
    MPSS_HIP(hipMemcpy(table.ptr, tab, n * sizeof(float), hipMemcpyHostToDevice));
    MPSS_HIP(hipMemset(table.ptr + n, 0, 2 * sizeof(float)));
    rcp.upload(rcp_, NB);
    L = len;
    rcp_min = rcp_[0];
    for (int c = 1; c < NB; ++c) rcp_min = rcp_[c] < rcp_min ? rcp_[c] : rcp_min;
    for (int c = 0; c < NB; ++c) host_rcp[c] = rcp_[c];
    groups = make_band_groups(rcp_, snake);
    rgb_refl.release();
    build_common(tab, groups, 0, false);
}

// The common grid (mo_band.h CommonGrid), on the host from the band tables:
//   * group g's grid is its longest-reach band's own (rg = the smallest rcp), u = d2 * rg;
//   * the LDS budget of the wide kernel (4 x 10239 floats) is split so that every slot's exact near
//     field ends at the same distance: klim_j ~ K0 * rcp_j / rg, and u0lim = min_j klim_j rg / rcp_j
//     (less a 2^-18 margin) guarantees s_j = fl(d2 rcp_j) < klim_j for every lane with u < u0lim;
//   * R_j(u) = band j's lerp at f = u * rcp_j / rg in double (its last segment continued one row past
//     its end, 0 after); on the group rows a lane computes (1 - t) R_j(u0) + t R_j(u0 + 1);
//   * the row range: the far path reads R where the band gather reads T, both piecewise linear, so the
//     largest error lies on a knot of one of the two grids, and at the group grid's knots R is T's own
//     lerp; every band knot s >= u0lim rcp_j / rg - 1 is compared (R's lerp at u = s rg / rcp_j against
//     T[s]), and the rows end one cell before the first knot whose error exceeds kCgRelTol of |T[s]|
//     (unfloored: a zero or a sign change ends it) -- past it every lookup reads the exact tables; for
//     the rgbprofile's R, G, B (rgb) of the largest of the three at that distance instead of |T[s]|;
//   * at most kCgMaxRows rows per group (32 B each: a group's rows stay well inside its XCD's 4 MB L2);
//   * tau_j = the smallest float d2 with fl(d2 * rcp_j) >= L - 1 (sampleProfile's range test).
#ifndef MPSS_CG_MAX_ROWS_DEFAULT  // (A/B builds of the cap only)
#define MPSS_CG_MAX_ROWS_DEFAULT 49152
#endif
constexpr int kCgMaxRows = MPSS_CG_MAX_ROWS_DEFAULT;
// (a diagnostic build, -DMPSS_DIAGNOSTICS, lets MPSS_CG_MAX_ROWS override the cap: row-cap experiments)
static int cg_max_rows() {
#ifdef MPSS_DIAGNOSTICS
    const char *e = getenv("MPSS_CG_MAX_ROWS");
    if (e && atoi(e) > 0) return atoi(e);
#endif
    return kCgMaxRows;
}

bool build_common_grid(const float *tab, int L, const float *host_rcp, const BandGroups &groups, CommonGrid &cg,
                       std::vector<float4> &h, float cg_rel_err[NB], float cg_l1_err[NB], int near_field,
                       int lds_reserve, bool rgb) {
    cg = CommonGrid{};
    for (int g = 0; g < kGroups; ++g) {  // (one row per grid step unless the layout below says otherwise)
        cg.hinv[g] = 1.f;
        cg.hc[g] = 0.f;
        cg.ua[g] = (float)L;
    }
    h.clear();
    for (int c = 0; c < NB; ++c) cg_rel_err[c] = cg_l1_err[c] = 0.f;
    const int kLdsFloats = 4 * (near_field + 3) - lds_reserve;
    if (L < 4) return false;
    for (int g = 0; g < kGroups; ++g)
        for (int j = 0; j < 4; ++j) {
            const int c = groups.band[g][j];
            if (c >= 0 && (!(host_rcp[c] > 0.f) || !std::isfinite(host_rcp[c])))
                return false;  // no uniform grid to resample
        }
    // The groups are independent (their own slots, LDS split, rows and errors): each is built on its
    // own thread into its own row block, then the blocks are laid out in group order. (For the
    // rgbprofile all groups hold the same three slots: one group is built and copied.)
    std::vector<float4> hg[kGroups];
    float relg[kGroups][4] = {}, l1g[kGroups][4] = {};
    bool anyg[kGroups] = {}, failg[kGroups] = {};
    auto build_group = [&](int g) {
        std::vector<float4> &h = hg[g];
        float rg = INFINITY;
        int nfull = 0;
        for (int j = 0; j < 4; ++j)
            if (groups.band[g][j] >= 0) {
                rg = std::min(rg, host_rcp[groups.band[g][j]]);
                ++nfull;
            }
        if (nfull == 0) {  // an unused group: no wave ever walks it
            for (int j = 0; j < 4; ++j) {
                cg.lrow[g][j] = (uint32_t)(2 * j);
                cg.lcnt[g][j] = 2;
            }
            return;
        }
        double r[4] = {0.0, 0.0, 0.0, 0.0}, rsum = 0.0;
        for (int j = 0; j < 4; ++j)
            if (groups.band[g][j] >= 0) {
                r[j] = (double)host_rcp[groups.band[g][j]] / (double)rg;
                rsum += r[j];
            }
        // near-field split: sum_j (klim_j + 1) <= kLdsFloats (empty slots: 2 zero floats)
        int K0 = (int)std::floor((kLdsFloats - 3.0 * nfull - 2.0 * (4 - nfull) - 8.0) / rsum);
        int klim[4], total;
        for (;;) {
            total = 0;
            for (int j = 0; j < 4; ++j) {
                if (groups.band[g][j] < 0) {
                    klim[j] = 1;
                } else {
                    const double want = std::ceil((double)K0 * r[j] * (1.0 + 1e-6)) + 1.0;
                    klim[j] = (int)std::min<double>(want, (double)(L - 2));
                }
                total += klim[j] + 1;
            }
            if (total <= kLdsFloats || K0 <= 1) break;
            --K0;
        }
        if (total > kLdsFloats) {
            failg[g] = true;
            return;
        }
        uint32_t off = 0;
        double u0 = INFINITY;
        for (int j = 0; j < 4; ++j) {
            cg.lrow[g][j] = off;
            cg.lcnt[g][j] = klim[j] + 1;
            off += (uint32_t)(klim[j] + 1);
            if (groups.band[g][j] >= 0) u0 = std::min(u0, (double)klim[j] / r[j] * (1.0 - 0x1p-18));
        }
        float u0f = (float)u0;
        if ((double)u0f > u0) u0f = std::nextafter(u0f, 0.f);
        cg.u0lim[g] = u0f;
        cg.rg[g] = rg;
        // a leaf is LDS-only when every lane's u < u0lim: leaf_r2 * rg below u0lim, with a 1e-5 margin
        // for the rounding of the lanes' d2 (as the band gather's lds_r2_lim)
        cg.lds_r2[g] = (float)((double)u0f / ((double)rg * 1.00001));
        for (int j = 0; j < 4; ++j) {
            const int c = groups.band[g][j];
            if (c < 0) {
                cg.tau[g][j] = INFINITY;  // (its sum is never stored)
                continue;
            }
            const float rc = host_rcp[c];
            const float endf = (float)(L - 1);
            float x = (float)((double)(L - 1) / (double)rc);
            auto past = [&](float d2) {
                volatile float f = d2 * rc;  // the float product of sampleProfile (multipole.cpp:63)
                return f >= endf;
            };
            while (x > 0.f && past(x)) x = std::nextafter(x, 0.f);
            while (!past(x)) x = std::nextafter(x, INFINITY);
            cg.tau[g][j] = x;
        }
        // R_j(u): band j on the group grid (double lerp, rounded once)
        auto R = [&](int j, int64_t u) -> float {
            const int c = groups.band[g][j];
            if (c < 0 || u >= (int64_t)L) return 0.f;
            const double f = (double)u * r[j];
            if (f - r[j] > (double)(L - 1)) return 0.f;  // past the row after the band's end
            const int sidx = std::min((int)std::floor(f), L - 2);
            const double t = f - sidx;
            const float *T = tab + (size_t)c * L;
            return (float)((1.0 - t) * (double)T[sidx] + t * (double)T[sidx + 1]);
        };
        // The row layout. Rows are indexed by v, a piecewise-linear map of u: v = u below ua (one row per
        // grid step), v = ua + (u - ua) / H above it (one row per H steps, H = 1, 2 or 4) -- on the lane
        // v = min(u, fma(u, hinv, hc)), hc = ua (1 - hinv). A cell (rows k, k + 1) is "bad" when some band
        // knot in it is off by more than max(kCgRelTol scale, kCgAbsTol peak) on the rows (the error of
        // two piecewise-linear functions peaks at a knot of one or the other, and at the row positions R is
        // the band's own lerp, rounded once); a bad cell's row carries a NaN in slot 0's first value and
        // its lanes read the bands' own tables instead (cg_fix), so every served value is within the bound.
        // The range [u1start, u1lim), ua and H are chosen to maximise the record weight served by good
        // cells (records per unit u fall off as 1 / u past the near field: the octree's aggregated nodes
        // grow with distance), a bad cell counting against it, within kCgMaxRows rows (+ one pad row).
        double peak[4] = {0.0, 0.0, 0.0, 0.0};  // each band's largest |T|
        for (int j = 0; j < 4; ++j)
            if (groups.band[g][j] >= 0) {
                const float *T = tab + (size_t)groups.band[g][j] * L;
                for (int k = 0; k < L; ++k) peak[j] = std::max(peak[j], std::fabs((double)T[k]));
            }
        // the value a knot's error is relative to: the band's own |T[s]|; for the rgbprofile's R, G, B
        // (rgb) the largest of the three at that distance -- FromRGB's outputs are sums of the three
        // with weights of order one, so each component's error counts against their scale, not its own
        // (B, ~15x shorter reach, falls orders of magnitude under R and G soon past the near field)
        auto scale = [&](int j, int k) -> double {
            const float *T = tab + (size_t)groups.band[g][j] * L;
            double v = std::fabs((double)T[k]);
            if (!rgb) return v;
            const double u = (double)k / r[j];
            for (int q = 0; q < 4; ++q) {
                const int c = groups.band[g][q];
                if (c < 0 || q == j) continue;
                const double f = u * r[q];
                if (f > (double)(L - 1)) continue;
                const int sidx = std::min((int)std::floor(f), L - 2);
                const double t = f - sidx;
                const float *Tq = tab + (size_t)c * L;
                v = std::max(v, std::fabs((1.0 - t) * (double)Tq[sidx] + t * (double)Tq[sidx + 1]));
            }
            return v;
        };
        // |rows - T| at band j's knot k on a grid of H steps (cells [H m, H (m + 1))), inf = bad
        auto knot_err = [&](int j, int k, int H) -> double {
            const float *T = tab + (size_t)groups.band[g][j] * L;
            const double u = (double)k / r[j];
            const int64_t m = (int64_t)std::floor(u / H);
            const double t = (u - (double)(H * m)) / H;
            const double approx = (1.0 - t) * R(j, H * m) + t * R(j, H * (m + 1));
            const double err = std::fabs(approx - (double)T[k]);
            return err > std::max(kCgRelTol * scale(j, k), kCgAbsTol * peak[j]) ? INFINITY : err;
        };
        static constexpr int kH[3] = {1, 2, 4};
        const int ncell = L + 2;  // cells of the fine grid (u < L); coarse grids: ncell / H + 1
        std::vector<uint8_t> bad[3];
        for (int hi = 0; hi < 3; ++hi) bad[hi].assign((size_t)ncell / kH[hi] + 2, 0);
        std::vector<double> fine_bad;  // u of the fine grid's bad knots (the candidate range starts)
        for (int j = 0; j < 4; ++j) {
            if (groups.band[g][j] < 0) continue;
            for (int k = std::max(0, (int)std::floor((double)u0f * r[j]) - 1); k < L - 1; ++k) {
                const double u = (double)k / r[j];
                for (int hi = 0; hi < 3; ++hi)
                    if (knot_err(j, k, kH[hi]) == INFINITY) {
                        bad[hi][(size_t)std::floor(u / kH[hi])] = 1;
                        if (hi == 0) fine_bad.push_back(u);
                    }
            }
        }
        std::sort(fine_bad.begin(), fine_bad.end());
        // a cell within a step of a band's profile end (u_end = (L - 1) / r_j) is flagged too: there the
        // lanes take the own path, whose pairs carry sampleProfile's exact cutoff (multipole.cpp:65-66);
        // past it the band's rows are exactly 0 (R is 0 from u_end + 1 on), before it every lane's f_j is
        // at least one table step below L - 1 -- so the combine needs no range test
        for (int j = 0; j < 4; ++j) {
            if (groups.band[g][j] < 0) continue;
            const double ue = (double)(L - 1) / r[j];
            for (int hi = 0; hi < 3; ++hi) {
                const int H = kH[hi];
                const int64_t m0 = std::max<int64_t>(0, (int64_t)std::floor((ue - 1.0) / H));
                const int64_t m1 = (int64_t)std::floor((ue + 2.0) / H);
                for (int64_t m = m0; m <= m1 && m < (int64_t)bad[hi].size(); ++m) bad[hi][(size_t)m] = 1;
            }
        }
        // prefix scores per grid: a good cell +w, a bad one -w, w = the cell's share of records (~ H / u)
        std::vector<double> P[3], W0(bad[0].size() + 1, 0.0);  // (W0: the fine cells' weights, unsigned)
        for (size_t m = 0; m < bad[0].size(); ++m) W0[m + 1] = W0[m] + 1.0 / std::max(1.0, (double)m + 0.5);
        for (int hi = 0; hi < 3; ++hi) {
            const int H = kH[hi];
            const size_t n = bad[hi].size();
            P[hi].assign(n + 1, 0.0);
            for (size_t m = 0; m < n; ++m) {
                const double w = (double)H / std::max(1.0, (double)H * ((double)m + 0.5));
                P[hi][m + 1] = P[hi][m] + (bad[hi][m] ? -w : w);
            }
        }
        // argmax of P over an index range (sparse table per grid)
        std::vector<std::vector<uint32_t>> sp[3];
        for (int hi = 0; hi < 3; ++hi) {
            const size_t n = P[hi].size();
            sp[hi].push_back(std::vector<uint32_t>(n));
            for (size_t i = 0; i < n; ++i) sp[hi][0][i] = (uint32_t)i;
            for (size_t lv = 1; ((size_t)1 << lv) <= n; ++lv) {
                const std::vector<uint32_t> &a = sp[hi][lv - 1];
                std::vector<uint32_t> b(n - ((size_t)1 << lv) + 1);
                for (size_t i = 0; i < b.size(); ++i) {
                    const uint32_t x = a[i], y = a[i + ((size_t)1 << (lv - 1))];
                    b[i] = P[hi][y] > P[hi][x] ? y : x;
                }
                sp[hi].push_back(std::move(b));
            }
        }
        auto argmax = [&](int hi, size_t lo, size_t hi_incl) -> size_t {  // first index of the max
            size_t lv = 0;
            while (((size_t)2 << lv) <= hi_incl - lo + 1) ++lv;
            const uint32_t x = sp[hi][lv][lo], y = sp[hi][lv][hi_incl + 1 - ((size_t)1 << lv)];
            return P[hi][y] > P[hi][x] ? y : x;
        };
        const int64_t cap = cg_max_rows();
        const int64_t uend = (int64_t)L - 1;  // the rows serve u < u1lim <= L - 1
        // candidate starts: the near field's end, and just past each of the first bad fine knots
        std::vector<double> starts{(double)u0f};
        for (const double b : fine_bad) {
            if (starts.size() >= 64) break;
            const double st = std::floor(b) + 2.0;
            if (st > starts.back() && st < (double)uend) starts.push_back(st);
        }
        double best = 0.0, bstart = u0f;
        int64_t bua = 0, bu1 = 0;
        int bh = 0;
        // (the rows always begin at the near field's end, so that a lane's row path is u0lim <= u < u1lim:
        // one compare; the cells before the chosen start st are flagged)
        const int64_t vbase = std::max<int64_t>(0, (int64_t)std::floor((double)u0f) - 1);
        const int64_t c0 = (int64_t)std::floor((double)u0f);
        for (const double st : starts) {
            const int64_t sb = (int64_t)std::floor(st);
            const double pre = W0[(size_t)sb] - W0[(size_t)c0];  // the flagged cells before st
            // H = 1: fine rows only, [st, u1)
            {
                const int64_t hiu = std::min<int64_t>(uend, vbase + cap);
                if (hiu > sb) {
                    const size_t e = argmax(0, (size_t)sb + 1, (size_t)hiu);
                    const double sc = P[0][e] - P[0][sb] - pre;
                    if (sc > best) {
                        best = sc, bstart = st, bua = (int64_t)e, bu1 = (int64_t)e, bh = 0;
                    }
                }
            }
            // H = 2, 4: fine rows [st, ua), coarse rows [ua, u1), ua a multiple of 64 (so hc is exact)
            for (int hi = 1; hi < 3; ++hi) {
                const int H = kH[hi];
                for (int64_t ua = ((sb + 64) / 64) * 64; ua < uend; ua += 64) {
                    const int64_t left = cap - (ua - vbase);
                    if (left < 2) break;
                    const double sf = P[0][ua] - P[0][sb];
                    const int64_t m0 = ua / H;
                    const int64_t mhi = std::min<int64_t>(m0 + left, uend / H);
                    if (mhi <= m0) continue;
                    const size_t e = argmax(hi, (size_t)m0 + 1, (size_t)mhi);
                    const double sc = sf + P[hi][e] - P[hi][m0] - pre;
                    if (sc > best) best = sc, bstart = st, bua = ua, bu1 = (int64_t)e * H, bh = hi;
                }
            }
        }
        const int H = kH[bh];
        cg.hinv[g] = 1.f;
        cg.hc[g] = 0.f;
        cg.ua[g] = (float)L;
        if (!(best > 0.0) || bu1 <= (int64_t)bstart + 1) {  // no accurate range: the exact tables past the near field
            cg.u1lim[g] = cg.u1start[g] = u0f;
            cg.ubase[g] = 0;
            return;
        }
        const int64_t ua = bh ? bua : bu1;  // (H = 1: every row fine)
        if (bh) {
            cg.hinv[g] = 1.f / (float)H;
            cg.hc[g] = (float)((double)ua * (1.0 - 1.0 / H));  // exact: ua a multiple of 64
            cg.ua[g] = (float)ua;
        }
        const int64_t v1 = ua + (bu1 - ua) / H;  // v(u1); lanes read rows <= v1 (v may round up to v1)
        auto upos = [&](int64_t v) -> int64_t { return v <= ua ? v : ua + (int64_t)H * (v - ua); };
        const int64_t sfirst = (int64_t)std::floor(bstart);  // the first cell the chosen stretch serves
        auto cell_bad = [&](int64_t v) -> bool {
            const int64_t u = upos(v);
            if (u < sfirst && u >= c0) return true;  // (the row below c0 is never read)
            return v < ua ? bad[0][(size_t)u] != 0 : bad[bh][(size_t)(u / H)] != 0;
        };
        cg.ubase[g] = (uint32_t)vbase;
        cg.u1start[g] = (float)bstart;  // (u0f, or an integer below 2^24)
        cg.u1lim[g] = (float)bu1;
        for (int64_t v = vbase; v <= v1; ++v) {
            const int64_t u = upos(v), un = upos(v + 1);
            float vv[4][2];
            for (int j = 0; j < 4; ++j) {
                vv[j][0] = R(j, u);
                vv[j][1] = R(j, un);
            }
            if (cell_bad(v)) vv[0][0] = NAN;  // its lanes read the bands' own tables (cg_fix)
            h.push_back(make_float4(vv[0][0], vv[0][1], vv[1][0], vv[1][1]));
            h.push_back(make_float4(vv[2][0], vv[2][1], vv[3][0], vv[3][1]));
        }
        for (int j = 0; j < 4; ++j) {  // the error over the knots the good rows serve
            const int c = groups.band[g][j];
            if (c < 0) continue;
            const float *T = tab + (size_t)c * L;
            double l1 = 0.0, emax = 0.0, esum = 0.0;
            for (int k = 0; k < L; ++k) l1 += std::fabs(T[k]);
            for (int k = std::max(0, (int)std::floor(bstart * r[j]) - 1); k < L - 1; ++k) {
                const double u = (double)k / r[j];
                if (u < bstart) continue;
                if (u >= (double)bu1) break;
                const int Hk = u < (double)ua ? 1 : H;
                const int64_t v = u < (double)ua ? (int64_t)std::floor(u) : ua + (int64_t)std::floor((u - ua) / H);
                if (cell_bad(v)) continue;
                const double e = knot_err(j, k, Hk);
                // (relative error -- to scale(): the band's own value, or the largest of R, G, B -- where
                // the relative bound governs: scale >= kCgAbsTol / kCgRelTol of the peak)
                const double sc = scale(j, k);
                if (kCgRelTol * sc >= kCgAbsTol * peak[j]) emax = std::max(emax, e / sc);
                esum += e;
            }
            relg[g][j] = (float)emax;
            l1g[g][j] = (float)(l1 > 0.0 ? esum / l1 : 0.0);
        }
        anyg[g] = true;
    };
    bool same = rgb;  // (rgb: every group's slots are the same three profiles)
    for (int g = 1; g < kGroups && same; ++g)
        for (int j = 0; j < 4; ++j) same = same && groups.band[g][j] == groups.band[0][j];
    if (same) {
        build_group(0);
        for (int g = 1; g < kGroups; ++g) {
            hg[g] = hg[0];
            for (int j = 0; j < 4; ++j) {
                cg.lrow[g][j] = cg.lrow[0][j];
                cg.lcnt[g][j] = cg.lcnt[0][j];
                cg.tau[g][j] = cg.tau[0][j];
                relg[g][j] = relg[0][j];
                l1g[g][j] = l1g[0][j];
            }
            cg.u0lim[g] = cg.u0lim[0];
            cg.rg[g] = cg.rg[0];
            cg.lds_r2[g] = cg.lds_r2[0];
            cg.ubase[g] = cg.ubase[0];
            cg.u1start[g] = cg.u1start[0];
            cg.u1lim[g] = cg.u1lim[0];
            cg.ua[g] = cg.ua[0];
            cg.hinv[g] = cg.hinv[0];
            cg.hc[g] = cg.hc[0];
            anyg[g] = anyg[0];
            failg[g] = failg[0];
        }
    } else {
        std::vector<std::thread> th;
        for (int g = 0; g < kGroups; ++g) th.emplace_back(build_group, g);
        for (std::thread &t : th) t.join();
    }
    bool any = false;
    for (int g = 0; g < kGroups; ++g) {
        if (failg[g]) return false;
        cg.row0[g] = (uint32_t)(h.size() / 2);
        h.insert(h.end(), hg[g].begin(), hg[g].end());
        any = any || anyg[g];
        for (int j = 0; j < 4; ++j) {
            const int c = groups.band[g][j];
            if (c < 0) continue;
            cg_rel_err[c] = std::max(cg_rel_err[c], relg[g][j]);
            cg_l1_err[c] = std::max(cg_l1_err[c], l1g[g][j]);
        }
    }
    cg.on = any ? 1 : 0;
    return any;
}

void DeviceProfile::set_rgb(const float *tab) {
    static const float refl[7][NB] = {MPSS_BAND_RGBREFL2SPECTWHITE_INIT, MPSS_BAND_RGBREFL2SPECTCYAN_INIT,
                                      MPSS_BAND_RGBREFL2SPECTMAGENTA_INIT, MPSS_BAND_RGBREFL2SPECTYELLOW_INIT,
                                      MPSS_BAND_RGBREFL2SPECTRED_INIT, MPSS_BAND_RGBREFL2SPECTGREEN_INIT,
                                      MPSS_BAND_RGBREFL2SPECTBLUE_INIT};
    rgb_refl.upload(&refl[0][0], 7 * NB);
    // the common grid of the R, G, B profiles (rows 0..2, the same three slots in every group: the
    // sharded gather reads them in band_tree's lband order)
    BandGroups g3 = groups;
    for (int g = 0; g < kGroups; ++g)
        for (int j = 0; j < 4; ++j) g3.band[g][j] = j < 3 ? j : -1;
    build_common(tab, g3, 28, true);  // (the LDS's last 28 floats: the groups' FromRGB weights)
}

void DeviceProfile::build_common(const float *tab, const BandGroups &slots, int lds_reserve, bool rgb) {
    ctab.release();
    ctab_half.release();
    // the two LDS layouts' grids side by side (host work: each builds its groups on threads of its own)
    std::vector<float4> hh, h;
    bool ok_half = false;
    std::thread half([&] {
        ok_half = build_common_grid(tab, L, host_rcp, slots, cg_half, hh, cg_rel_err[1], cg_l1_err[1], 5088,
                                    lds_reserve, rgb);
    });
    const bool ok = build_common_grid(tab, L, host_rcp, slots, cg, h, cg_rel_err[0], cg_l1_err[0], 10236,
                                      lds_reserve, rgb);
    half.join();
    if (ok_half) {
        ctab_half.upload(hh.data(), hh.size());
        cg_half.tab = ctab_half.ptr;
    } else {
        cg_half.on = 0;
    }
    if (!ok) {
        cg.on = 0;  // the per-band tables stay in use
        return;
    }
    ctab.upload(h.data(), h.size());
    cg.tab = ctab.ptr;
}

namespace {
// Also writes the bound's leaf code into NodeHdr::pad's high half (its low half is the live point count):
// the bound's high 16 bits rounded up, so code < (lim's high 16 bits) => bound < lim -- the sharded
// gather's LDS-only leaf test is then one scalar compare on the header it has loaded anyway.
__global__ void leaf_r2_kernel(NodeHdr *__restrict__ nodes, int n, float max_error, float *__restrict__ r2) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= n) return;
    const NodeHdr h = nodes[i];
    float out = INFINITY;
    if (h.leaf_first >= 0 && h.sum_area > 0.f && max_error > 0.f && isfinite(h.px) && isfinite(h.py) &&
        isfinite(h.pz)) {
        // A query opens the leaf only if |q - c| <= open (dw >= max_error) or q lies in the box. Every point
        // lies in the box, so |q - p_i| <= open + (c's farthest box corner) or <= diag. The centroid c is
        // luminance-weighted and need not lie in the box (mixed-sign E, or a zero weight sum leaving c at
        // the origin), hence the farthest corner from c rather than the diagonal.
        const double dx = (double)h.bmaxx - h.bminx, dy = (double)h.bmaxy - h.bminy, dz = (double)h.bmaxz - h.bminz;
        const double diag = sqrt(dx * dx + dy * dy + dz * dz);
        const double fx = fmax(fabs((double)h.px - h.bminx), fabs((double)h.px - h.bmaxx));
        const double fy = fmax(fabs((double)h.py - h.bminy), fabs((double)h.py - h.bmaxy));
        const double fz = fmax(fabs((double)h.pz - h.bminz), fabs((double)h.pz - h.bmaxz));
        const double corner = sqrt(fx * fx + fy * fy + fz * fz);
        const double open = sqrt((double)h.sum_area / (double)max_error) * (1.0 + 1e-6);
        const double R = (open + corner > diag ? open + corner : diag);
        out = (float)(R * R * (1.0 + 1e-6));
    }
    r2[i] = out;
    const uint32_t code = (__float_as_uint(out) + 0xffffu) >> 16;  // (out > 0; INF -> 0x7f80)
    nodes[i].pad = (h.pad & 0xffffu) | (code << 16);
}
}  // namespace

void DeviceOctree::ensure_leaf_r2(float max_error) {
    if (leaf_r2.ptr && leaf_r2_error == max_error) return;
    leaf_r2.alloc((size_t)(n_nodes > 0 ? n_nodes : 1));
    if (n_nodes > 0)
        hipLaunchKernelGGL(leaf_r2_kernel, dim3((unsigned)((n_nodes + 255) / 256)), dim3(256), 0, 0, nodes.ptr, n_nodes,
                           max_error, leaf_r2.ptr);
    MPSS_HIP(hipGetLastError());
    MPSS_HIP(hipDeviceSynchronize());
    leaf_r2_error = max_error;
}

const BandLayout *DeviceOctree::find_layout(const BandGroups &g) const {
    for (const auto &l : layouts)
        if (same_groups(l->groups, g)) return l.get();
    return nullptr;
}

const BandLayout &DeviceOctree::ensure_layout(const BandGroups &g) {
    if (const BandLayout *l = find_layout(g)) return *l;
    auto lay = std::make_unique<BandLayout>();
    lay->groups = g;
    lay->et.alloc((size_t)(n_nodes > 0 ? n_nodes : 1) * kGroups);
    lay->e.alloc((size_t)(n_points > 0 ? n_points : 1) * kGroups);
    lay->ew.alloc((size_t)(n_points > 0 ? n_points : 1) * kGroups);
    const int64_t tn = (int64_t)n_nodes * kGroups, tp = (int64_t)n_points * kGroups;
    if (tn) hipLaunchKernelGGL(band_permute_kernel, dim3((unsigned)((tn + 255) / 256)), dim3(256), 0, 0, node_et.ptr,
                               n_nodes, g, nullptr, lay->et.ptr);
    if (tp) {
        hipLaunchKernelGGL(band_permute_kernel, dim3((unsigned)((tp + 255) / 256)), dim3(256), 0, 0, pt_e.ptr,
                           n_points, g, nullptr, lay->e.ptr);
        hipLaunchKernelGGL(band_permute_kernel, dim3((unsigned)((tp + 255) / 256)), dim3(256), 0, 0, pt_e.ptr,
                           n_points, g, pt_hdr.ptr, lay->ew.ptr);
    }
    MPSS_HIP(hipGetLastError());
    // synchronous: every stream that launches a gather later sees a complete layout
    MPSS_HIP(hipDeviceSynchronize());
    layouts.push_back(std::move(lay));
    return *layouts.back();
}

void launch_mo_band(const DeviceOctree &t, const BandLayout &layout, const DeviceProfile &p, float max_error,
                    int nq_max, const float4 *queries4, const int *count_dev, float4 *out4, const uint32_t *hit_s,
                    int mat, unsigned long long *counts, int *work, int *perm, const GatherOpts &opts,
                    hipStream_t stream) {
    if (nq_max <= 0 || t.n_nodes <= 0) return;
    BandArgs a{};
    a.t = band_tree(t, layout, p, max_error);
    a.queries4 = queries4;
    a.count = count_dev;
    a.hit_s = hit_s;
    a.mat = mat;
    a.nq = nq_max;
    a.out4 = out4;
    a.counts = counts;
    a.work = work;
    a.perm = perm;
    launch_band(a, nq_max, t, counts != nullptr, opts, stream);
}

void launch_mo_gather(const DeviceOctree &t, const BandLayout *layout, const DeviceProfile &p, float max_error, int nq,
                      const float *queries, float *out, int out_stride, int32_t *counters, int *work, int *perm,
                      int mode, const GatherOpts &opts, hipStream_t stream) {
    const bool exact = mode == 1;
    if (nq <= 0) return;
    if (t.n_nodes <= 0) throw Error(-1, "launch_mo_gather: octree is empty");
    if (p.L < 2) throw Error(-1, "launch_mo_gather: profile table has fewer than 2 entries");
    const bool count = counters != nullptr;
    if (mode == 0) {
        if (!layout || !work) throw Error(-2, "launch_mo_gather: the sharded gather needs a band layout and work counters");
        if (count) MPSS_HIP(hipMemsetAsync(counters, 0, sizeof(int32_t) * 4 * (size_t)nq, stream));
        BandArgs b{};
        b.t = band_tree(t, *layout, p, max_error);
        b.queries3 = queries;
        b.nq = nq;
        b.out = out;
        b.out_stride = out_stride;
        b.counters = counters;
        b.work = work;
        b.perm = perm;
        launch_band(b, nq, t, count, opts, stream);
        return;
    }
    MoArgs a{};  // value-initialized: unused fields (render-path queries, functor tables) are null
    a.nodes = t.nodes.ptr;
    a.node_et = t.node_et.ptr;
    a.pt_hdr = t.pt_hdr.ptr;
    a.pt_e = t.pt_e.ptr;
    a.table = p.table.ptr;
    a.rcp = p.rcp.ptr;
    a.queries = queries;
    a.out = out;
    a.counters = counters;
    a.L = p.L;
    a.n_nodes = t.n_nodes;
    a.nq = nq;
    a.out_stride = out_stride;
    a.max_error = max_error;
    a.rcp_min = p.rcp_min > 0.f ? p.rcp_min : 0.f;  // rcp_min <= 0 disables pruning
    a.prune_f = (a.rcp_min > 0.f) ? (float)(p.L - 1) * 1.0001f : INFINITY;
    if (!exact) {
        const int packets = (nq + 7) / 8, blocks = (packets + 3) / 4;
        if (count)
            hipLaunchKernelGGL((mo_packet_kernel<true>), dim3(blocks), dim3(256), 0, stream, a, blocks);
        else
            hipLaunchKernelGGL((mo_packet_kernel<false>), dim3(blocks), dim3(256), 0, stream, a, blocks);
        MPSS_HIP(hipGetLastError());
        return;
    }
    a.dipole = nullptr;
    launch_exact<FN_TABLE>(a, t.max_depth, count, stream);
}

void launch_mo_dipole(const DeviceOctree &t, const float *dipole_dev, float max_error, int nq, const float *queries,
                      float *out, int out_stride, int32_t *counters, hipStream_t stream) {
    if (nq <= 0) return;
    if (t.n_nodes <= 0) throw Error(-1, "launch_mo_dipole: octree is empty");
    MoArgs a{};
    a.nodes = t.nodes.ptr;
    a.node_et = t.node_et.ptr;
    a.pt_hdr = t.pt_hdr.ptr;
    a.pt_e = t.pt_e.ptr;
    a.queries = queries;
    a.out = out;
    a.counters = counters;
    a.L = 2;
    a.n_nodes = t.n_nodes;
    a.nq = nq;
    a.out_stride = out_stride;
    a.max_error = max_error;
    a.rcp_min = 0.f;
    a.prune_f = INFINITY;
    a.dipole = dipole_dev;
    launch_exact<FN_DIPOLE>(a, t.max_depth, counters != nullptr, stream);
}

void launch_mo_rgb(const DeviceOctree &t, const float *table3, const float *rcp3_dev, const float rcp3[3], int L,
                   float max_error, int nq, const float *queries, const float4 *queries4, const int *count_dev,
                   const uint32_t *hit_s, int mat, float *out, int out_stride, int32_t *counters, hipStream_t stream) {
    if (nq <= 0) return;
    if (t.n_nodes <= 0) throw Error(-1, "launch_mo_rgb: octree is empty");
    if (L < 2) throw Error(-1, "launch_mo_rgb: profile table has fewer than 2 entries");
    MoArgs a{};
    a.nodes = t.nodes.ptr;
    a.node_et = t.node_et.ptr;
    a.pt_hdr = t.pt_hdr.ptr;
    a.pt_e = t.pt_e.ptr;
    a.table = table3;
    a.rcp = rcp3_dev;
    a.queries = queries;
    a.queries4 = queries4;
    a.count = count_dev;
    a.hit_s = hit_s;
    a.mat = mat;
    a.out = out;
    a.counters = counters;
    a.L = L;
    a.n_nodes = t.n_nodes;
    a.nq = nq;
    a.out_stride = out_stride;
    a.max_error = max_error;
    // every band is FromRGB of the three lookups: +0 once all three are past their table's end
    float rmin = rcp3[0] < rcp3[1] ? rcp3[0] : rcp3[1];
    rmin = rcp3[2] < rmin ? rcp3[2] : rmin;
    a.rcp_min = rmin > 0.f ? rmin : 0.f;
    a.prune_f = (a.rcp_min > 0.f) ? (float)(L - 1) * 1.0001f : INFINITY;
    launch_exact<FN_RGB>(a, t.max_depth, counters != nullptr, stream);
}

}  // namespace mpss
