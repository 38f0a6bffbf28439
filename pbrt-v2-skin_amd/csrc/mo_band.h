// mo_band.h -- the spectrally sharded Mo() gather (device), used by the render path and by
// mpss_mo_batch's default mode.
//
// Why: the gather's cost is the Rd(d^2) table lookups. The 30 per-band tables (L floats each,
// 14 MB for skin) are hit at 30 unrelated offsets per (query, record) and do not fit one XCD's
// 4 MB L2, so with every wave touching every band the lookups miss to the fabric (measured:
// 39-61 % L2 hit rate, ~4x the algorithmic bytes through the fabric).
//
// Mapping: the 30 bands are dealt into 8 groups of <= 4 (BandGroups) and group g runs only on
// workgroups with blockIdx % 8 == g, i.e. on one XCD under the round-robin dispatch. Each XCD's
// L2 then holds only its own <= 4 tables (< 2 MB). One wave64 = 64 queries x one group: lane
// = query, 4 bands per lane. Node / point headers and the group's 16-byte Et/E slice are
// wave-uniform scalar loads from a group-major copy of the octree (band_et / band_e, 16 B per
// record per group, so consecutive pre-order records share lines); only the table lookups
// are per-lane gathers.
//
// Each query walks exactly the node set of SubsurfaceOctreeNode::Mo (diffusionutil.h:175-210)
// minus subtrees that lie past the end of all of the group's profiles (they add +0 for these
// bands), in pre-order, with the packet kernel's summation order: results are bit-identical
// to mo_packet_traverse (one running sum per band, a leaf's points summed first).
#pragma once
#include "common.h"
#include "octree.h"

namespace mpss {

constexpr int kGroups = 8;
constexpr int kBandBlock = 1024;  // queries per workgroup (16 waves of one band group)
constexpr int kLdsRd = 4096;      // leading Rd entries of each of the group's 4 bands kept in LDS (64 KB)

// Band -> (group, slot) assignment and per-group pruning scale.
struct BandGroups {
    int band[kGroups][4];    // band index, or -1 for an empty slot
    float rcp_min[kGroups];  // min rcpDsqSpacing over the group's bands
    int pos[NB];             // band c lives at float pos[c] of a group-major row (4 * g + slot)
};

// Deal bands to groups: bands sorted by decreasing profile reach (L-1)/rcp, snake order
// (0..7, 7..0, ...), so every group gets one of the 8 longest-reaching bands (the work a
// group does is set by its longest-reaching band) and the rest spread evenly.
inline BandGroups make_band_groups(const float *rcp) {
    int order[NB];
    for (int c = 0; c < NB; ++c) order[c] = c;
    for (int i = 1; i < NB; ++i)  // insertion sort by increasing rcp (= decreasing reach)
        for (int j = i; j > 0 && rcp[order[j]] < rcp[order[j - 1]]; --j) {
            const int t = order[j];
            order[j] = order[j - 1];
            order[j - 1] = t;
        }
    BandGroups g;
    int fill[kGroups] = {0};
    for (int i = 0; i < kGroups; ++i) {
        g.rcp_min[i] = INFINITY;
        for (int s = 0; s < 4; ++s) g.band[i][s] = -1;
    }
    for (int r = 0; r < NB; ++r) {
        const int round = r / kGroups, k = r % kGroups;
        const int grp = (round & 1) ? kGroups - 1 - k : k;
        const int c = order[r];
        g.band[grp][fill[grp]] = c;
        g.pos[c] = 4 * grp + fill[grp];
        ++fill[grp];
        g.rcp_min[grp] = rcp[c] < g.rcp_min[grp] ? rcp[c] : g.rcp_min[grp];
    }
    return g;
}

struct BandTree {
    const NodeHdr *__restrict__ nodes;
    const float4 *__restrict__ band_et;  // [kGroups][n_nodes]
    const float4 *__restrict__ pt_hdr;   // [n_points] {p, area (sign bit: E black)}
    const float4 *__restrict__ band_e;   // [kGroups][n_points]
    const float *__restrict__ table;     // [NB][L]
    const float *__restrict__ rcp;       // [NB]
    BandGroups groups;
    int L, n_nodes, n_points;
    float max_error, prune_f;
};

#ifdef __HIP__  // device traversal: HIP translation units only (host .cpp files see the layout types)
// The lerp pair (T[s], T[s+1]) as one 8-byte load at 4-byte alignment (gfx950 global loads
// take unaligned dword pairs): one vector-memory instruction per band instead of two.
struct __attribute__((aligned(4))) RdPair {
    float a, b;
};

// Rd lookups of one record for the lane's 4 bands, straight-line: the 4 pair loads are issued
// back to back (lanes past a band's profile read a clamped, valid entry and are masked), then
// consumed -- one memory round trip per record and no divergent branches for the compiler to
// serialize. t = fract(f) equals f - (float)(uint)f exactly for 0 <= f < 2^24.
// acc[j] += Rd_j(d2) * e[j] (* w) exactly as sampleProfile + the Mo() product
// (multipole.cpp:60-73; diffusionutil.h:185,197).
// The first kLdsRd entries of each band (the near field: leaf points and close clusters, about
// 40 % of the red bands' lookups) come from the workgroup's LDS copy, the rest from L2.
template <bool POINT>
__device__ __forceinline__ void band_rd_accumulate(const float *const tb[4], const float rcp[4], float lm1,
                                                   uint32_t smax, float d2, const float e[4], float w,
                                                   float acc[4], const float (*lt)[kLdsRd]) {
    float f[4];
    bool ok[4];
    RdPair v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        f[j] = d2 * rcp[j];
        ok[j] = f[j] < lm1;
        const uint32_t s = ok[j] ? (uint32_t)f[j] : smax;
        // two unconditional loads and a select (a branch here makes the compiler merge both
        // paths into flat loads): lanes served by LDS point their L2 load at one shared line
        const bool in_lds = s + 1 < (uint32_t)kLdsRd;
        const uint32_t sl = in_lds ? s : 0u, sg = in_lds ? smax : s;
        const float la = lt[j][sl], lb = lt[j][sl + 1];
        const RdPair g = *reinterpret_cast<const RdPair *>(tb[j] + sg);
        v[j].a = in_lds ? la : g.a;
        v[j].b = in_lds ? lb : g.b;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float t = __builtin_amdgcn_fractf(f[j]);
        const float rd = (1.f - t) * v[j].a + t * v[j].b;
        const float val = POINT ? rd * e[j] * w : rd * e[j];
        acc[j] += ok[j] ? val : 0.f;  // == the masked add: acc starts at +0 and never becomes -0
    }
}

// sum_area / d2 < max_error decided without an IEEE division in the common case: a * rcp(d)
// (v_rcp_f32, <= 1 ulp; product <= ~2.5 ulp) is trusted when it clears max_error by 2^-20
// relative either way; the rare near-ties (and NaN/inf) take the exact division, so the decision
// is always that of fl(sum_area / d2) < max_error (diffusionutil.h:182).
__device__ __forceinline__ bool dw_below(float a, float d, float m) {
    const float r = a * __builtin_amdgcn_rcpf(d);
    const float lo = m * (1.f - 0x1p-20f), hi = m * (1.f + 0x1p-20f);
    bool below = r < lo;
    const bool sure = below || r > hi;
    if (!sure) below = (a / d) < m;
    return below;
}

template <bool COUNT>
__device__ __forceinline__ void mo_band_traverse(const BandTree &a, int grp, float px, float py, float pz, bool valid,
                                                 float acc[4], int &k_nodes, int &k_pts, const float (*lt)[kLdsRd]) {
    float rcp[4];
    const float *tb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = a.groups.band[grp][j];
        rcp[j] = c >= 0 ? a.rcp[c] : INFINITY;
        tb[j] = a.table + (size_t)(c >= 0 ? c : 0) * a.L;
        acc[j] = 0.f;
    }
    const float rcp_min = a.groups.rcp_min[grp];
    const float4 *__restrict__ et_g = a.band_et + (size_t)grp * a.n_nodes;
    const float4 *__restrict__ e_g = a.band_e + (size_t)grp * a.n_points;
    const float lm1 = (float)(a.L - 1);
    const uint32_t smax = (uint32_t)(a.L - 2);  // clamped (masked) index for out-of-range bands
    int resume = valid ? 0 : 0x7fffffff;
    int node = 0;
    while (node < a.n_nodes) {
        node = __builtin_amdgcn_readfirstlane(node);
        const NodeHdr h = a.nodes[node];
        const int skip = h.skip;
        bool open = false;
        if (node >= resume) {
            if (COUNT) ++k_nodes;
            const float bx = fmaxf(fmaxf(h.bminx - px, px - h.bmaxx), 0.f);
            const float by = fmaxf(fmaxf(h.bminy - py, py - h.bmaxy), 0.f);
            const float bz = fmaxf(fmaxf(h.bminz - pz, pz - h.bmaxz), 0.f);
            const bool prune = (bx * bx + by * by + bz * bz) * rcp_min >= a.prune_f;
            if (prune || (h.flags & NODE_BLACK)) {
                resume = skip;
            } else {
                const float dx = px - h.px, dy = py - h.py, dz = pz - h.pz;
                const float d2 = dx * dx + dy * dy + dz * dz;
                const bool inside = px >= h.bminx && px <= h.bmaxx && py >= h.bminy && py <= h.bmaxy &&
                                    pz >= h.bminz && pz <= h.bmaxz;
                if (dw_below(h.sum_area, d2, a.max_error) && !inside) {
                    resume = skip;
                    const float4 et = et_g[node];
                    const float e[4] = {et.x, et.y, et.z, et.w};
                    band_rd_accumulate<false>(tb, rcp, lm1, smax, d2, e, 1.f, acc, lt);
                } else {
                    open = true;
                }
            }
        }
        const bool any_open = __builtin_amdgcn_ballot_w64(open) != 0;
        if (h.leaf_first >= 0) {
            if (any_open) {
                // the leaf's non-black points only (DeviceOctree::upload puts them first, h.pad)
                float lacc[4] = {0.f, 0.f, 0.f, 0.f};
                const int live = (int)h.pad;
                for (int i = 0; i < live; ++i) {
                    const int kp = h.leaf_first + i;
                    const float4 ph = a.pt_hdr[kp];
                    if (!open) continue;
                    if (COUNT) ++k_pts;
                    const float ex = px - ph.x, ey = py - ph.y, ez = pz - ph.z;
                    const float d2 = ex * ex + ey * ey + ez * ez;
                    const float4 ev = e_g[kp];
                    const float e[4] = {ev.x, ev.y, ev.z, ev.w};
                    band_rd_accumulate<true>(tb, rcp, lm1, smax, d2, e, ph.w, lacc, lt);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[j] += lacc[j];
            }
            if (open) resume = skip;
            node = skip;
        } else if (any_open) {
            node = node + 1;
        } else {
            node = skip;
        }
    }
}
#endif

}  // namespace mpss
