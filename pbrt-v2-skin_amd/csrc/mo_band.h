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
constexpr int kLdsRd = 4096;      // leading Rd entries per band kept in LDS (64 KB: two workgroups per CU)
constexpr int kLdsRdBig = 10224;  // the same filling one CU's 160 KB (one workgroup per CU)

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
    const float *__restrict__ table;     // [NB][L] + 2 trailing zeros (DeviceProfile::upload)
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
typedef float f2v __attribute__((ext_vector_type(2)));  // v_pk_{add,mul}_f32 operands
typedef __attribute__((address_space(3))) const float lds_float;  // ds_read, never a flat load

// The lane's view of its group's 4 bands.
struct BandLane {
    const float *tb[4];  // band tables (an empty slot reads band 0's with rcp 0; its sum is unused)
    float rcp[4];
    uint32_t zero[4];    // tb[j] + zero[j] = the table's trailing zero pair
    float lm1;           // L - 1: sampleProfile's range end
    float klim;          // min(KLDS, L) - 1: f < klim <=> the lerp pair is in LDS and in range
};

// Rd lookups of one record for the lane's 4 bands, accumulated:
// acc[j] += Rd_j(d2) * e[j] (* w), as sampleProfile + the Mo() product (multipole.cpp:60-73;
// diffusionutil.h:185,197) -- the same IEEE operations in the same order as the scalar code.
// lt: the workgroup's LDS copy of the first KLDS entries of each band, rows of KLDS + 2 floats
// (the last two zero). Per band one wave-uniform choice: if every active lane's pair is in the
// LDS copy (or the lane is past the profile end), all read LDS; otherwise all read the table
// (L2). A lane past the profile end reads a zero pair, so its term is (0 * e) * w = +-0 and the
// running sum (which starts at +0 and is never -0) is unchanged: no masking instruction. The
// pairs of all 4 bands are requested before any is consumed (one memory round trip per
// record); the lerp and the products run as packed f32 (two values per instruction).
template <bool POINT, int KLDS, bool FLAT>
__device__ __forceinline__ void band_rd_accumulate(const BandLane &b, float d2, const float e[4], float w, f2v acc[2],
                                                   const float *lt) {
    float f[4];
    RdPair v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        f[j] = d2 * b.rcp[j];
        const uint32_t s = (uint32_t)f[j];  // fSegId (the double product is exact: multipole.cpp:63-65)
        const bool ok = f[j] < b.lm1;
        const bool in_lds = f[j] < b.klim;  // implies ok
        if (FLAT) {  // per lane: one flat load whose address is in LDS or in the table
            const float *src = in_lds ? lt + j * (KLDS + 2) + s : b.tb[j] + (ok ? s : b.zero[j]);
            v[j] = *reinterpret_cast<const RdPair *>(src);
        } else if (__builtin_amdgcn_ballot_w64(ok && !in_lds) == 0) {
            const lds_float *row =
                (const lds_float *)lt + j * (KLDS + 2) + (in_lds ? s : (uint32_t)KLDS);
            v[j].a = row[0];
            v[j].b = row[1];
        } else {
            v[j] = *reinterpret_cast<const RdPair *>(b.tb[j] + (ok ? s : b.zero[j]));
        }
    }
    float rd[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float t = __builtin_amdgcn_fractf(f[j]);  // == f - (float)(uint)f for 0 <= f < 2^24
        const f2v p = f2v{1.f - t, t} * f2v{v[j].a, v[j].b};
        rd[j] = p.x + p.y;  // (1 - t) * T[s] + t * T[s + 1]
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        f2v val = f2v{rd[2 * h], rd[2 * h + 1]} * f2v{e[2 * h], e[2 * h + 1]};
        if (POINT) val = val * f2v{w, w};
        acc[h] += val;
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

template <bool COUNT, int KLDS, bool FLAT>
__device__ __forceinline__ void mo_band_traverse(const BandTree &a, int grp, float px, float py, float pz, bool valid,
                                                 float out[4], int &k_nodes, int &k_pts, const float *lt) {
    BandLane b;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = a.groups.band[grp][j];
        const int cc = c >= 0 ? c : 0;
        b.rcp[j] = c >= 0 ? a.rcp[c] : 0.f;
        b.tb[j] = a.table + (size_t)cc * a.L;
        b.zero[j] = (uint32_t)(NB - cc) * (uint32_t)a.L;
    }
    b.lm1 = (float)(a.L - 1);
    b.klim = (float)((a.L < KLDS ? a.L : KLDS) - 1);
    f2v acc[2] = {f2v{0.f, 0.f}, f2v{0.f, 0.f}};
    const float rcp_min = a.groups.rcp_min[grp];
    const float4 *__restrict__ et_g = a.band_et + (size_t)grp * a.n_nodes;
    const float4 *__restrict__ e_g = a.band_e + (size_t)grp * a.n_points;
    int resume = valid ? 0 : 0x7fffffff;
    int node = 0;
    while (node < a.n_nodes) {
        node = __builtin_amdgcn_readfirstlane(node);
        const NodeHdr h = a.nodes[node];
        const int skip = h.skip;
        bool open = false;
        if (node >= resume) {
            if (COUNT) ++k_nodes;
            // distance from p to the node box per axis (0 inside the slab)
            const float bx = fmaxf(fmaxf(h.bminx - px, px - h.bmaxx), 0.f);
            const float by = fmaxf(fmaxf(h.bminy - py, py - h.bmaxy), 0.f);
            const float bz = fmaxf(fmaxf(h.bminz - pz, pz - h.bmaxz), 0.f);
            const bool prune = (bx * bx + by * by + bz * bz) * rcp_min >= a.prune_f;
            if (prune || (h.flags & NODE_BLACK)) {
                resume = skip;
            } else {
                const float dx = px - h.px, dy = py - h.py, dz = pz - h.pz;
                const float d2 = dx * dx + dy * dy + dz * dz;
                // nodeBound.Inside(p) <=> every per-axis distance is 0 (the subtractions' signs are exact)
                const bool inside = fmaxf(fmaxf(bx, by), bz) == 0.f;
                if (dw_below(h.sum_area, d2, a.max_error) && !inside) {
                    resume = skip;
                    const float4 et = et_g[node];
                    const float e[4] = {et.x, et.y, et.z, et.w};
                    band_rd_accumulate<false, KLDS, FLAT>(b, d2, e, 1.f, acc, lt);
                } else {
                    open = true;
                }
            }
        }
        const bool any_open = __builtin_amdgcn_ballot_w64(open) != 0;
        if (h.leaf_first >= 0) {
            if (any_open) {
                // the leaf's non-black points only (DeviceOctree::upload puts them first, h.pad)
                f2v lacc[2] = {f2v{0.f, 0.f}, f2v{0.f, 0.f}};
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
                    band_rd_accumulate<true, KLDS, FLAT>(b, d2, e, ph.w, lacc, lt);
                }
                acc[0] += lacc[0];
                acc[1] += lacc[1];
            }
            if (open) resume = skip;
            node = skip;
        } else if (any_open) {
            node = node + 1;
        } else {
            node = skip;
        }
    }
    out[0] = acc[0].x;
    out[1] = acc[0].y;
    out[2] = acc[1].x;
    out[3] = acc[1].y;
}
#endif

}  // namespace mpss
