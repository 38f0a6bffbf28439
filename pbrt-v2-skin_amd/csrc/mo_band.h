// mo_band.h -- the spectrally sharded Mo() gather (device), used by the render path and by
// mpss_mo_batch's default mode.
//
// Why sharded: the gather's memory traffic is the Rd(d^2) table lookups. The 30 per-band
// tables (L floats each, 14 MB for skin) are hit at 30 unrelated offsets per (query, record)
// and do not fit one XCD's 4 MB L2, so with every wave touching every band the lookups miss
// to the fabric (measured: 39-61 % L2 hit rate, ~4x the algorithmic bytes through the fabric).
//
// Mapping: the 30 bands are dealt into 8 groups of <= 4 (BandGroups) and group g runs only on
// workgroups with blockIdx % 8 == g, i.e. on one XCD under the round-robin dispatch. Each XCD's
// L2 then holds only its own <= 4 tables (< 2 MB). One wave64 = 64 queries x one group: lane
// = query, 4 bands per lane. Node / point headers and the group's 16-byte Et/E slice are
// wave-uniform scalar loads from a group-major copy of the octree (BandLayout, 16 B per record
// per group, so consecutive pre-order records share lines); only the table lookups are per-lane
// gathers (one 8-byte load per band: the lerp pair).
//
// What bounds it: with the common grid (the default, CommonGrid below) two resources together -- the
// vector-memory path's L2 request rate (0.84 of the rate tools/microbench/l2_width.hip sustains for the
// grid's row loads) and VALU issue (0.80 of the rate tools/microbench/valu_issue.hip measures for this
// record loop's instruction mix; SQ_ACTIVE_INST_VALU busy 0.82), DESIGN.md §4 "Round 5"; with the
// per-band tables (mo_common_grid 0) the L2 request rate of the per-lane table gathers alone. The traversal is the UNION of
// the wave's 64 pruned traversals, so the 64 queries of a wave should be neighbours: each 1024-query
// chunk is sorted by a Morton key of the query position before queries are dealt to lanes
// (mo_kernel.hip), and the per-record work below is kept to a few VALU on 32-bit table offsets.
//
// Each query walks exactly the node set of SubsurfaceOctreeNode::Mo (diffusionutil.h:175-210)
// minus subtrees that lie past the end of all of the group's profiles (they add +0 for these
// bands), in pre-order, with the packet kernel's summation order. With the per-band tables the
// results are bit-identical to mo_packet_traverse (one running sum per band, a leaf's points summed
// first); the common grid resamples the far lookups (within kCgRelTol / kCgAbsTol per value) and forms
// each term with FMAs (cg_combine), so its sums are within the float-summation bound of the reference
// (tests/test_mo_gpu.py) rather than bit-identical to it.
#pragma once
#include <cstdlib>

#include "common.h"
#include "octree.h"

namespace mpss {

constexpr int kGroups = 8;
// Per-lane traversal counters of the instrumented (COUNT) gather, summed into mo_kernel.h's counts:
// 0 table lookups inside the profile (lane x band), 1..3 those at entries < 4096, 8192, 16384;
// common grid only: 4..6 lane-records by path (group rows, LDS near field, the bands' own tables);
// 7..8 distinct 32-byte sectors and 9..10 distinct 128-byte lines the path's loads touch, summed
// over wave fetches (rows, own tables: what the vector-memory path asks of L2); 11..12 wave fetches
// with a lane on the path (rows, own tables).
constexpr int kHist = 13;

// Band -> (group, slot) assignment and per-group pruning scale.
struct BandGroups {
    int band[kGroups][4];    // band index, or -1 for an empty slot
    float rcp_min[kGroups];  // min rcpDsqSpacing over the group's bands
    int pos[NB];             // band c lives at float pos[c] of a group-major row (4 * g + slot)
};

// Deal bands to groups: bands sorted by decreasing profile reach (L-1)/rcp, then either runs of
// adjacent reach (default: group g's bands share one prune radius, so few of its lookups fall
// past a band's profile end) or, with `snake` (mpss_config.mo_band_dealing = 1), snake rounds
// (0..7, 7..0, ...: every group gets one of the 8 longest-reaching bands, equal work per group).
inline BandGroups make_band_groups(const float *rcp, bool snake = false) {
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
    // Groups of adjacent reach (6 x 4 + 2 x 3 bands, by decreasing reach): each group's prune radius
    // fits all of its bands, 29 % fewer record visits than dealing the bands in snake rounds; the
    // groups' unequal work is evened out by the gather's work stealing (C2: 41.1 -> 37.3 ms per
    // frame, profiles/r02j_variants.txt r02bf).
    const bool contig = !snake;
    for (int r = 0; r < NB; ++r) {
        const int round = r / kGroups, k = r % kGroups;
        const int grp = contig ? (r < 24 ? r / 4 : 6 + (r - 24) / 3) : ((round & 1) ? kGroups - 1 - k : k);
        const int c = order[r];
        g.band[grp][fill[grp]] = c;
        g.pos[c] = 4 * grp + fill[grp];
        ++fill[grp];
        g.rcp_min[grp] = rcp[c] < g.rcp_min[grp] ? rcp[c] : g.rcp_min[grp];
    }
    return g;
}

inline bool same_groups(const BandGroups &a, const BandGroups &b) {
    for (int g = 0; g < kGroups; ++g)
        for (int s = 0; s < 4; ++s)
            if (a.band[g][s] != b.band[g][s]) return false;
    return true;
}

// The common grid of a band group (mpss_config.mo_common_grid; DeviceProfile::build_common): a
// lookup of all <= 4 bands of the group past their LDS near fields from ONE interleaved table. The
// group's tables are resampled onto the grid of its longest-reach band (rg = its rcpDsqSpacing, for
// which the resampling is the identity), u = d2 * rg, and stored as 32-byte pair rows
// {R_0(u_k), R_0(u_k+1), R_1(u_k), R_1(u_k+1)}, {R_2(u_k), ...}: a lookup is two 16-byte loads from one
// 32-byte-aligned sector per lane instead of four 8-byte lerp pairs from four unrelated offsets (the
// gather is bound by the L2 request rate of these per-lane loads). Row k sits at u_k = k
// below ua and at ua + H (k - ua) above it (H = 1, 2 or 4 per group): the lane's row coordinate is
// v = min(u, fma(u, hinv, hc)), hc = ua (1 - hinv), its row floor(v) and its lerp parameter fract(v), so
// a group's rows can reach its profile end inside kCgMaxRows where the tables are smooth enough for
// the coarser steps. Each lane takes one of three paths by u:
//   u < u0lim          every band's exact pair from its LDS near field (as the per-band gather);
//   u0lim <= u < u1lim the group rows -- accurate wherever they are read: build_common measures the
//                      error at every band's own knots, and a cell (row) holding a knot off by more
//                      than the bound carries a NaN in its first value: its lanes read the bands' own
//                      tables instead (cg_fix). So does a cell within a step of a band's profile end
//                      (sampleProfile's exact cutoff, multipole.cpp:65-66, is the own path's) and one
//                      before the stretch the rows serve (u1start). The range is the one serving the
//                      most records from good cells (the far tails of the longest-reach bands carry
//                      the MPC resampler's float noise, which no coarser grid follows: every cell bad);
//   otherwise          every band's exact pair from its own table in HBM/L2 (as the per-band gather),
//                      a band past its profile end from the table's trailing zero pair.
struct CommonGrid {
    const float4 *tab;          // pair rows, two float4 each; group g's row for u at 2 * (row0[g] + u - ubase[g])
    uint32_t row0[kGroups];     // group g's first pair row
    uint32_t ubase[kGroups];    // the v (row coordinate) of that row
    float rg[kGroups];          // the group's grid: u = d2 * rg (its smallest rcp)
    float u0lim[kGroups];       // u < u0lim => every band's pair (s, s + 1) lies in its LDS near field
    float u1lim[kGroups];       // u0lim <= u < u1lim: the pair rows (u1lim = u0lim: none)
    float u1start[kGroups];     // the rows' cells below it are flagged (bands the rows cannot serve)
    float ua[kGroups];          // rows one grid step apart below ua, H steps apart above (L: none)
    float hinv[kGroups];        // 1 / H
    float hc[kGroups];          // ua (1 - 1 / H): v = min(u, fma(u, hinv, hc)) (exact: ua a multiple of 64)
    float tau[kGroups][4];      // d2 >= tau <=> fl(d2 * rcp) >= L - 1: the band is past its profile end
    uint32_t lrow[kGroups][4];  // float offset of slot j's near-field row in LDS (entries 0..klim_j)
    int lcnt[kGroups][4];       // its length, klim_j + 1 floats (2 zeros for an empty slot)
    float lds_r2[kGroups];      // a leaf with leaf_r2 below this is read from LDS only (0: never)
    int on;                     // 1: some group has a non-empty row range (the three-path gather runs)
};

// A band group's FromRGB weights (SampledSpectrum::FromRGB, spectrum.cpp:103-186) for its four
// output bands (0 for an empty slot): out = .94 (W min + X (mid - min) + Y (max - mid)) with X the
// secondary spectrum of the smallest component and Y the primary of the largest.
struct RgbK {
    float w[4];     // rgbRefl2SpectWhite
    float x[3][4];  // Cyan (R smallest), Magenta (G), Yellow (B)
    float y[3][4];  // Red (R largest), Green (G), Blue (B)
};

struct BandTree {
    const NodeHdr *__restrict__ nodes;
    const float4 *__restrict__ band_et;  // [kGroups][n_nodes]
    const float4 *__restrict__ pt_hdr;   // [n_points] {p, area (sign bit: E black)}
    const float4 *__restrict__ band_e;   // [kGroups][n_points]
    const float4 *__restrict__ band_ew;  // [kGroups][n_points]: E * area (the common-grid gather)
    const float *__restrict__ table;     // [NB][L] + 2 trailing zeros (DeviceProfile::upload)
    BandGroups groups;
    float grcp[kGroups][4];              // rcpDsqSpacing of each group slot (0 for an empty slot)
    float grcp_max[kGroups];             // the largest of a group's rcp (its shortest reach)
    const float *leaf_r2;                // DeviceOctree::leaf_r2, non-null when its leaf codes (NodeHdr::pad's
                                         // high half) hold for max_error (null: no LDS-only point loops)
    int L, n_nodes, n_points;
    float max_error, prune_f;
    CommonGrid cg;       // the grid the launch uses (launch_band: cg_half for the 5088 layout)
    CommonGrid cg_half;
    // The table row each group slot looks up: groups.band for a spectral profile; for an rgbprofile
    // material (RGB = 1) rows 0, 1, 2 (its R, G, B profiles) in every group, slot 3 unused -- the
    // group's four OUTPUT bands stay groups.band (Rd_c = FromRGB of the three lookups, band c).
    int lband[kGroups][4];
    const float *rgb_refl;  // RGB: rgbRefl2Spect{White, Cyan, Magenta, Yellow, Red, Green, Blue} [7][NB]
    RgbK rgb_k[kGroups];    // RGB: each group's weights (band_tree, from the same tables)
};

#ifdef __HIP__  // device traversal: HIP translation units only (host .cpp files see the layout types)
// The lerp pair (T[s], T[s+1]) as one 8-byte load at 4-byte alignment (gfx950 global loads
// take unaligned dword pairs): one vector-memory instruction per band instead of two.
struct __attribute__((aligned(4))) RdPair {
    float a, b;
};
typedef float f2v __attribute__((ext_vector_type(2)));  // v_pk_{add,mul}_f32 operands
typedef float f4v __attribute__((ext_vector_type(4)));
// The octree is read-only while a gather runs. Reading it through the constant address space
// says so to the compiler: with stores of results earlier in the same (persistent) kernel it
// otherwise cannot prove the node records unclobbered and turns the wave-uniform header loads
// into vector loads (a full L2 round trip at the top of every node iteration).
#if defined(__HIP_DEVICE_COMPILE__)
template <class T>
using cptr = const __attribute__((address_space(4))) T *;
#else  // the host pass of a HIP translation unit never runs these functions
template <class T>
using cptr = const T *;
#endif
template <class T>
__device__ __forceinline__ cptr<T> as_const(const T *p) {
    return (cptr<T>)p;
}

typedef __attribute__((address_space(3))) const float lds_float;  // ds_read, never a flat load

// The lane's view of its group's 4 bands: table offsets (floats from BandTree::table), rcp, and
// the workgroup's LDS copy of the first entries of each band (the near field).
// LDS rows hold KLDS + 3 floats per band slot: entries 0..klim of the band (klim = min(KLDS, L - 2)),
// zeros after, and a zero pair at row offset KLDS + 1. Lanes with klim <= s < L - 1 read the table
// in L2; all others read LDS -- s < klim the near field, s >= L - 1 (past the profile end:
// sampleProfile returns 0) the zero pair. The LDS/L2 choice is one unsigned range test.
struct BandLane {
    uint32_t off[4];  // c * L (an empty slot reads band 0 with rcp 0; its sum is never stored)
    float rcp[4];
    uint32_t lm1;     // L - 1: sampleProfile's range end
    uint32_t klim;    // min(KLDS, L - 2): s < klim <=> the pair (s, s + 1) is in the LDS copy
    uint32_t gspan;   // L - 1 - klim: s - klim < gspan (unsigned) <=> the pair is read from L2
    const float *lt;  // LDS rows (generic pointer)
    lds_float *ltl;   // the same rows through the LDS address space (ds_read only)
    const float *tb[4];  // the bands' table rows
};
// Row length (floats) of a band's LDS near field.
template <int KLDS>
__host__ __device__ constexpr int near_row() {
    return KLDS + 3;
}

// Rd lookups of one record for the lane's 4 bands, accumulated:
// acc[j] += Rd_j(d2) * e[j] (* w), as sampleProfile + the Mo() product (multipole.cpp:60-73;
// diffusionutil.h:185,197) -- the same IEEE operations in the same order as the scalar code:
// f = d2 * rcp in float (the reference multiplies two floats and widens the product), s = floor
// f, t = f - s, (1 - t) * T[s] + t * T[s + 1]. s < L - 1 <=> f < L - 1 (sampleProfile's range
// test); a lane past the end reads the zero pair, so its term is (0 * e) * w = +0 and the
// running sum (which starts at +0 and is never -0) is unchanged: no masking instruction. All
// four lookups are issued before any is consumed; the products run as packed f32.
// Each lane's pair is one flat load whose address lies in LDS or in the table: the L2 request
// rate is what bounds the gather, and only lanes outside the near field make requests.
// COUNT: hist[0] += lookups inside the profile, hist[1..3] += those with s < 4096, 8192, 16384
// (how much a near-field copy of that many entries per band in LDS would absorb).
// The fetch half: f per band and the four pair loads (issued, not consumed).
template <bool COUNT, int KLDS>
__device__ __forceinline__ void band_rd_fetch(const BandLane &b, float d2, float f[4], RdPair v[4], int hist[kHist]) {
    const f2v f01 = f2v{d2, d2} * f2v{b.rcp[0], b.rcp[1]};
    const f2v f23 = f2v{d2, d2} * f2v{b.rcp[2], b.rcp[3]};
    f[0] = f01.x;
    f[1] = f01.y;
    f[2] = f23.x;
    f[3] = f23.y;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t s = (uint32_t)f[j];  // saturating convert: f >= 2^32 -> 0xffffffff >= lm1
        const bool glob = s - b.klim < b.gspan;  // unsigned: s < klim wraps past gspan
        const uint32_t li = s < (uint32_t)(KLDS + 1) ? s : (uint32_t)(KLDS + 1);
        const float *src = glob ? b.tb[j] + s : b.lt + j * near_row<KLDS>() + li;
        v[j] = *reinterpret_cast<const RdPair *>(src);
        if (COUNT && s < b.lm1 && b.rcp[j] > 0.f) {
            ++hist[0];
            hist[1] += s < 4096u;
            hist[2] += s < 8192u;
            hist[3] += s < 16384u;
        }
    }
}

// band_rd_fetch for a point the caller has proven inside the near field of all four bands (s <
// klim: DeviceOctree::leaf_r2): the pairs come straight from LDS (ds_read), the vector-memory path
// -- the gather's binding resource -- never sees them. Same f, same pairs, so the same terms.
template <int KLDS>
__device__ __forceinline__ void band_rd_fetch_lds(const BandLane &b, float d2, float f[4], RdPair v[4]) {
    const f2v f01 = f2v{d2, d2} * f2v{b.rcp[0], b.rcp[1]};
    const f2v f23 = f2v{d2, d2} * f2v{b.rcp[2], b.rcp[3]};
    f[0] = f01.x;
    f[1] = f01.y;
    f[2] = f23.x;
    f[3] = f23.y;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t s = (uint32_t)f[j];
        lds_float *q = b.ltl + j * near_row<KLDS>() + s;  // one ds_read2_b32 per band
        v[j].a = q[0];
        v[j].b = q[1];
    }
}

// A wave-uniform pointer held in VGPRs for the whole traversal (opaque to rematerialization): the
// per-lane address select of the near-field fetch then reads the band's row base straight from registers instead
// of re-copying it from SGPRs (v_cndmask takes one SGPR operand at most) for every lookup.
__device__ __forceinline__ const float *in_vgprs(const float *p) {
    const uint64_t u = (uint64_t)(uintptr_t)p;
    uint32_t lo, hi;
    asm volatile("v_mov_b32 %0, %1" : "=v"(lo) : "s"((uint32_t)u));
    asm volatile("v_mov_b32 %0, %1" : "=v"(hi) : "s"((uint32_t)(u >> 32)));
    return (const float *)(uintptr_t)(((uint64_t)hi << 32) | lo);
}

// A wave-uniform float held in a VGPR (an operand that would otherwise need a v_mov per use beside
// another SGPR operand).
__device__ __forceinline__ float in_vgpr(float x) {
    float v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "s"(x));
    return v;
}

// The Mo() products and the running sums of one record's four Rd values: acc += (Rd * e) (* w).
template <bool POINT>
__device__ __forceinline__ void band_rd_products(const float rd[4], const float e[4], float w, f2v acc[2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        f2v val = f2v{rd[2 * h], rd[2 * h + 1]} * f2v{e[2 * h], e[2 * h + 1]};
        if (POINT) val = val * f2v{w, w};
        acc[h] += val;
    }
}

// sampleProfile's lerp of the four pairs: rd[j] = (1 - t) * T[s] + t * T[s + 1], t = fract(f[j]).
__device__ __forceinline__ void band_rd_lerp(const float f[4], const RdPair v[4], float rd[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float t = __builtin_amdgcn_fractf(f[j]);  // == f - (float)(uint)f for 0 <= f < 2^24
        const f2v p = f2v{1.f - t, t} * f2v{v[j].a, v[j].b};
        // (1 - t) * T[s] + t * T[s + 1]: one v_add_f32 of the product pair's halves (the IEEE add the
        // compiler would emit; written out because its SLP pass otherwise pairs the adds of two bands
        // into a v_pk_add_f32 fed by three v_mov_b32 swizzles)
        asm("v_add_f32 %0, %1, %2" : "=v"(rd[j]) : "v"(p.x), "v"(p.y));
    }
}

// SampledSpectrum::FromRGB(rgb, SPECTRUM_REFLECTANCE) (spectrum.cpp:103-186; mo_kernel.hip
// from_rgb_band restates its branches) for the group's four output bands. Its six cases only pick
// which component is the minimum, middle and maximum, and two weight spectra by which component is
// the minimum (X: Cyan, Magenta, Yellow) and the maximum (Y: Red, Green, Blue):
//   out = .94 (W min + X (mid - min) + Y (max - mid)), clamped at 0.
// Here min / mid / max are v_min3 / v_med3 / v_max3 (the same values), and X, Y rows are read from
// the group's weights in LDS (rk: W[4], X[3][4], Y[3][4], RgbK's layout) by the lanes' own minimum and
// maximum components: no per-band selects and no weights held in registers. Where two components
// tie the reference's case order and this choice may name different X (or Y) rows, but the
// difference they weigh is then exactly 0, so the result is the same. The float operations are the
// reference's, the clamp is max(v, 0) (Clamp's v < 0 ? 0 : v but for v = -0 and NaN).
__device__ __forceinline__ void from_rgb4(lds_float *rk, float R, float G, float B, float o[4]) {
    const float mn = __builtin_fminf(R, __builtin_fminf(G, B));
    const float mx = __builtin_fmaxf(R, __builtin_fmaxf(G, B));
    const float md = __builtin_amdgcn_fmed3f(R, G, B);
    const uint32_t xs = R == mn ? 0u : (G == mn ? 1u : 2u);
    const uint32_t ys = R == mx ? 0u : (G == mx ? 1u : 2u);
    typedef __attribute__((address_space(3))) const f4v lds_f4v;
    const f4v w = *(lds_f4v *)rk, x = *(lds_f4v *)(rk + 4 + 4 * xs), y = *(lds_f4v *)(rk + 16 + 4 * ys);
    const float d1 = md - mn, d2 = mx - md;
    const f2v wv[2] = {f2v{w.x, w.y}, f2v{w.z, w.w}};
    const f2v xv[2] = {f2v{x.x, x.y}, f2v{x.z, x.w}};
    const f2v yv[2] = {f2v{y.x, y.y}, f2v{y.z, y.w}};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        f2v r = wv[h] * f2v{mn, mn};
        r = r + xv[h] * f2v{d1, d1};
        r = r + yv[h] * f2v{d2, d2};
        r = r * f2v{(float).94, (float).94};
        o[2 * h] = __builtin_fmaxf(r.x, 0.f);
        o[2 * h + 1] = __builtin_fmaxf(r.y, 0.f);
    }
}

// from_rgb4 for the common-grid gather (cg_combine): rk holds the weights times .94, the LDS offsets of
// the X and Y rows come from two selects each, and each band is .94 W min + .94 X (mid - min) + .94 Y
// (max - mid) as one multiply and two FMAs (packed, two bands per instruction), clamped at 0 -- within an
// ulp or two of FromRGB's own sum (the far values are a resampling already).
__device__ __forceinline__ void from_rgb4_fused(lds_float *rk, float R, float G, float B, float o[4]) {
    const float mn = __builtin_fminf(R, __builtin_fminf(G, B));
    const float mx = __builtin_fmaxf(R, __builtin_fmaxf(G, B));
    const float md = __builtin_amdgcn_fmed3f(R, G, B);
    const uint32_t ox = R == mn ? 4u : (G == mn ? 8u : 12u);   // X: Cyan, Magenta, Yellow
    const uint32_t oy = R == mx ? 16u : (G == mx ? 20u : 24u);  // Y: Red, Green, Blue
    typedef __attribute__((address_space(3))) const f4v lds_f4v;
    const f4v w = *(lds_f4v *)rk, x = *(lds_f4v *)(rk + ox), y = *(lds_f4v *)(rk + oy);
    const float d1 = md - mn, d2 = mx - md;
    const f2v wv[2] = {f2v{w.x, w.y}, f2v{w.z, w.w}};
    const f2v xv[2] = {f2v{x.x, x.y}, f2v{x.z, x.w}};
    const f2v yv[2] = {f2v{y.x, y.y}, f2v{y.z, y.w}};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        f2v r = wv[h] * f2v{mn, mn};
        r = __builtin_elementwise_fma(xv[h], f2v{d1, d1}, r);
        r = __builtin_elementwise_fma(yv[h], f2v{d2, d2}, r);
        o[2 * h] = __builtin_fmaxf(r.x, 0.f);
        o[2 * h + 1] = __builtin_fmaxf(r.y, 0.f);
    }
}

// The combine half: lerp, the Mo() products and the running sums (one point or node). RGB: the
// slots hold the R, G, B lookups, and the group's output bands take FromRGB (rk: their weights).
template <bool POINT, bool RGB = false>
__device__ __forceinline__ void band_rd_combine(const float f[4], const RdPair v[4], const float e[4], float w,
                                                f2v acc[2], lds_float *rk = nullptr) {
    float rd[4];
    band_rd_lerp(f, v, rd);
    if (RGB) {
        float o[4];
        from_rgb4(rk, rd[0], rd[1], rd[2], o);
        band_rd_products<POINT>(o, e, w, acc);
        return;
    }
    band_rd_products<POINT>(rd, e, w, acc);
}

// ---- the common-grid gather (CommonGrid) ----
// The lane's (wave-uniform) view of its group's grid.
struct CgLane {
    const float4 *tab;    // the pair rows, indexed by floor(v) + rowoff
    uint32_t rowoff;      // row0 - ubase (mod 2^32)
    float rg, u0lim, u1lim;
    float hinv, hc;       // v = min(u, fma(u, hinv, hc)) (hinv in a VGPR: one SGPR operand per fma)
    uint32_t lrow[4];     // LDS float offsets of the slots' exact near-field rows
    uint32_t off[4];      // c_j * L: the bands' own tables (the u >= u1lim path)
    uint32_t lm1;         // L - 1: sampleProfile's range end
    uint32_t zoff;        // byte offset of the table's trailing zero pair (NB * L floats in)
};

// One record's lookups: band j's pair (T[s], T[s + 1]) -- or (R(u0), R(u0 + 1)) on the group rows --
// in lanes {2j, 2j + 1} of the tuples p01 (bands 0, 1) and p23 (bands 2, 3), its lerp parameter in
// f[j] (d2 * rcp_j, or u on the group rows). Every path writes the two 128-bit tuples whole (a row
// half is one 16-byte load, an LDS or table pair fills one half), so the three paths share registers
// without moves -- a move after a load would wait for it to return.
// (Returned as a value: stores through a reference in the arms of the branch get sunk into one store
// to a phi of their addresses, which keeps the record in scratch memory.)
struct CgRec {
    float f[4];
    f4v p01, p23;
};
typedef const __attribute__((address_space(1))) float gfloat;
typedef const __attribute__((address_space(1))) f4v gf4v;
typedef const __attribute__((address_space(1))) f2v gf2v __attribute__((aligned(4)));

template <bool COUNT>
__device__ __forceinline__ void cg_count(const BandLane &b, const CgLane &c, float d2, int path, int hist[kHist]) {
    if (!COUNT) return;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t s = (uint32_t)(d2 * b.rcp[j]);
        if (!(b.rcp[j] > 0.f) || s >= c.lm1) continue;
        ++hist[0];
        hist[1] += s < 4096u;
        hist[2] += s < 8192u;
        hist[3] += s < 16384u;
    }
    hist[4 + path] += 1;  // 4: group rows, 5: LDS, 6: the bands' own tables
}

// COUNT: how many distinct keys (sector or line numbers) the active lanes hold, each lane holding k0 and,
// if it differs, k1 (a load that straddles two) -- counted once per wave, by its first active lane.
__device__ inline int wave_distinct(uint64_t k0, uint64_t k1) {
    uint64_t m0 = __builtin_amdgcn_ballot_w64(true);
    uint64_t m1 = __builtin_amdgcn_ballot_w64(k1 != k0);
    int n = 0;
    while (m0 | m1) {
        const uint64_t m = m0 ? m0 : m1;
        const int l = __builtin_ctzll(m);
        const bool from0 = m0 != 0;
        const uint64_t mine = from0 ? k0 : k1;
        const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)mine, l);
        const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(mine >> 32), l);
        const uint64_t key = ((uint64_t)hi << 32) | lo;
        m0 &= ~__builtin_amdgcn_ballot_w64(k0 == key);
        m1 &= ~__builtin_amdgcn_ballot_w64(k1 == key);
        ++n;
    }
    return n;
}
__device__ __forceinline__ bool first_active_lane() {
    return (int)(threadIdx.x & 63) == __builtin_ctzll(__builtin_amdgcn_ballot_w64(true));
}

__device__ __forceinline__ f2v lds_pair(const BandLane &b, uint32_t k) {
    lds_float *q = b.ltl + k;
    return f2v{q[0], q[1]};
}

// the per-band indices d2 * rcp_j (multipole.cpp:63: the float product)
__device__ __forceinline__ void band_f(const BandLane &b, float d2, float f[4]) {
    const f2v f01 = f2v{d2, d2} * f2v{b.rcp[0], b.rcp[1]};
    const f2v f23 = f2v{d2, d2} * f2v{b.rcp[2], b.rcp[3]};
    f[0] = f01.x;
    f[1] = f01.y;
    f[2] = f23.x;
    f[3] = f23.y;
}

template <bool COUNT>
__device__ __forceinline__ void cg_count_rows(uint64_t addr, int hist[kHist]) {
    const int ns = wave_distinct(addr >> 5, addr >> 5), nl = wave_distinct(addr >> 7, addr >> 7);
    if (first_active_lane()) {
        hist[7] += ns;
        hist[9] += nl;
        hist[11] += 1;
    }
}
template <bool COUNT>
__device__ __forceinline__ void cg_count_own(const uint64_t addr[4], int hist[kHist]) {
    int ns = 0, nl = 0;
    for (int j = 0; j < 4; ++j) {  // one 8-byte load per band
        ns += wave_distinct(addr[j] >> 5, (addr[j] + 7) >> 5);
        nl += wave_distinct(addr[j] >> 7, (addr[j] + 7) >> 7);
    }
    if (first_active_lane()) {
        hist[8] += ns;
        hist[10] += nl;
        hist[12] += 1;
    }
}

// every band's exact pair from its own table (the u >= u1lim path, and cg_fix)
template <bool COUNT>
__device__ __forceinline__ void cg_own(const BandLane &b, const CgLane &c, const float *table, float d2, CgRec &r,
                                       int hist[kHist]) {
    band_f(b, d2, r.f);
    uint32_t otp[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        // sampleProfile's range test (multipole.cpp:65-66): s >= L - 1 <=> fl(d2 rcp) >= L - 1 (the saturating
        // convert takes f >= 2^32 there too): the zero pair, so the term is exactly +0
        const uint32_t sj = (uint32_t)r.f[j];
        otp[j] = sj < c.lm1 ? 4u * (c.off[j] + sj) : c.zoff;
    }
    const __attribute__((address_space(1))) char *tb = (const __attribute__((address_space(1))) char *)table;
    const f2v q0 = *(gf2v *)(tb + otp[0]), q1 = *(gf2v *)(tb + otp[1]);
    const f2v q2 = *(gf2v *)(tb + otp[2]), q3 = *(gf2v *)(tb + otp[3]);
    if (COUNT) {
        const uint64_t ad[4] = {(uint64_t)(uintptr_t)table + otp[0], (uint64_t)(uintptr_t)table + otp[1],
                                (uint64_t)(uintptr_t)table + otp[2], (uint64_t)(uintptr_t)table + otp[3]};
        cg_count_own<COUNT>(ad, hist);
    }
    r.p01 = f4v{q0.x, q0.y, q1.x, q1.y};
    r.p23 = f4v{q2.x, q2.y, q3.x, q3.y};
#pragma unroll
    for (int j = 0; j < 4; ++j) r.f[j] = __builtin_amdgcn_fractf(r.f[j]);
}

template <bool COUNT>
__device__ __forceinline__ CgRec cg_fetch(const BandLane &b, const CgLane &c, const float *table, float d2,
                                          int hist[kHist]) {
    // Each path forms its own lerp parameters (CgRec::f holds t on return): the rows one fract(u) for
    // the four bands, the LDS and own-table lanes fract(d2 rcp_j) per band, the per-band indices
    // d2 * rcp_j only inside the steps that use them -- a wave whose lanes all read rows forms none.
    CgRec r;
    const float u = d2 * c.rg;
    // Three sequential masked steps, LDS first: a later step's loads may overwrite registers an
    // earlier step's loads target only once those have returned, and LDS returns first (the
    // opposite order made every LDS lane wait for the global loads). The two global steps write in
    // issue order (vector memory returns in order), so the second does not wait for the first. The
    // own-table step goes before the row step: its address arithmetic reuses the record's registers
    // as temporaries, which, behind the row step, waited for the row loads in flight to them (and,
    // for a pair's second point, for the first point's loads too) -- the row step's only VALU work
    // writes CgRec::f, which no load targets (C2 gather 42.8 -> 41.5 ms, profiles/r06_grid_ab.txt r06s).
    // The paths as lane masks: two compares, the rest scalar mask logic (written as plain bools, the
    // negation of a compare becomes a third compare)
    const uint64_t m_lds = __builtin_amdgcn_ballot_w64(u < c.u0lim);
    const uint64_t m_in = __builtin_amdgcn_ballot_w64(u < c.u1lim);
    const bool p_lds = __builtin_amdgcn_inverse_ballot_w64(m_lds);
    const bool p_row = __builtin_amdgcn_inverse_ballot_w64(m_in & ~m_lds);
    const bool p_own = __builtin_amdgcn_inverse_ballot_w64(~(m_in | m_lds));
    const int path = p_lds ? 1 : (p_row ? 0 : 2);  // (COUNT only)
    // the row step's address up front, as a 32-bit byte offset from the (wave-uniform) grid base: one
    // VGPR, a global load in saddr form. (The own-table step's four addresses are formed in its branch:
    // with the gather VALU-bound, a wave whose lanes all take the rows or the LDS does not pay them.)
    const float v = __builtin_fminf(u, __builtin_fmaf(u, c.hinv, c.hc));
    uint32_t orow = 32u * ((uint32_t)v + c.rowoff);
    asm volatile("" : "+v"(orow));
    if (p_lds) {  // s_j < klim_j for every band: inside its LDS row
        band_f(b, d2, r.f);
        const f2v q0 = lds_pair(b, c.lrow[0] + (uint32_t)r.f[0]), q1 = lds_pair(b, c.lrow[1] + (uint32_t)r.f[1]);
        const f2v q2 = lds_pair(b, c.lrow[2] + (uint32_t)r.f[2]), q3 = lds_pair(b, c.lrow[3] + (uint32_t)r.f[3]);
        r.p01 = f4v{q0.x, q0.y, q1.x, q1.y};
        r.p23 = f4v{q2.x, q2.y, q3.x, q3.y};
#pragma unroll
        for (int j = 0; j < 4; ++j) r.f[j] = __builtin_amdgcn_fractf(r.f[j]);
    }
    // (keeps the LDS step ahead of the global ones: the compiler otherwise orders the three steps its
    // own way and puts the LDS step last)
    asm volatile("" : "+v"(r.p01), "+v"(r.p23)::"memory");
    if (p_own) cg_own<COUNT>(b, c, table, d2, r, hist);
    asm volatile("" ::: "memory");  // (an order barrier only: an operand would wait for the loads)
    if (p_row) {
        gf4v *row = (gf4v *)((const __attribute__((address_space(1))) char *)c.tab + orow);
        r.p01 = row[0];
        r.p23 = row[1];
        if (COUNT) cg_count_rows<COUNT>((uint64_t)(uintptr_t)c.tab + orow, hist);
        const float t = __builtin_amdgcn_fractf(v);  // one lerp parameter for the four bands
#pragma unroll
        for (int j = 0; j < 4; ++j) r.f[j] = t;
    }
    cg_count<COUNT>(b, c, d2, path, hist);
    return r;
}

// A lane whose group row is flagged bad (a NaN first value: build_common_grid) reads every band's exact
// pair from its own table instead -- after the row has arrived, so only waves with such a lane wait a
// second round trip. Called for a record's (or a point pair's) fetches before they are combined. (The
// tables hold no NaN, so a lane of the LDS or own-table path never takes it.)
template <bool COUNT>
__device__ __forceinline__ void cg_fix(const BandLane &b, const CgLane &c, const float *table, float d2, CgRec &r,
                                       int hist[kHist]) {
    const bool bad = r.p01.x != r.p01.x;
    if (__builtin_amdgcn_ballot_w64(bad) != 0 && bad) cg_own<COUNT>(b, c, table, d2, r, hist);
}
template <bool COUNT>
__device__ __forceinline__ void cg_fix2(const BandLane &b, const CgLane &c, const float *table, float d2a,
                                        CgRec &ra, float d2b, CgRec &rb, int hist[kHist]) {
    const bool bad_a = ra.p01.x != ra.p01.x, bad_b = rb.p01.x != rb.p01.x;
    if (__builtin_amdgcn_ballot_w64(bad_a || bad_b) != 0) {
        if (bad_a) cg_own<COUNT>(b, c, table, d2a, ra, hist);
        if (bad_b) cg_own<COUNT>(b, c, table, d2b, rb, hist);
    }
}

// A record the caller has proven near for every lane (leaf_r2 < CommonGrid::lds_r2): LDS only.
__device__ __forceinline__ CgRec cg_fetch_near(const BandLane &b, const CgLane &c, float d2) {
    CgRec r;
    const f2v f01 = f2v{d2, d2} * f2v{b.rcp[0], b.rcp[1]};
    const f2v f23 = f2v{d2, d2} * f2v{b.rcp[2], b.rcp[3]};
    r.f[0] = f01.x;
    r.f[1] = f01.y;
    r.f[2] = f23.x;
    r.f[3] = f23.y;
    const f2v q0 = lds_pair(b, c.lrow[0] + (uint32_t)r.f[0]), q1 = lds_pair(b, c.lrow[1] + (uint32_t)r.f[1]);
    const f2v q2 = lds_pair(b, c.lrow[2] + (uint32_t)r.f[2]), q3 = lds_pair(b, c.lrow[3] + (uint32_t)r.f[3]);
    r.p01 = f4v{q0.x, q0.y, q1.x, q1.y};
    r.p23 = f4v{q2.x, q2.y, q3.x, q3.y};
#pragma unroll
    for (int j = 0; j < 4; ++j) r.f[j] = __builtin_amdgcn_fractf(r.f[j]);
    return r;
}

// sampleProfile's lerp with t = fract(f[j]) -- the LDS and own-table paths' exactly as the per-band
// gather's, the group rows' on the group grid. Its range test (multipole.cpp:65-66) is already in the
// pairs: an LDS lane is never past a band's end, an own-table lane past it read the zero pair, and a row
// cell within a step of a band's end is flagged (its lanes took the own path), past it the rows are 0.
// e is E * area for a point (BandTree::band_ew) and Et for a node, w unused.
template <bool POINT, bool RGB = false>
__device__ __forceinline__ void cg_combine(const CgLane &c, const CgRec &r, float d2, const float e[4], float w,
                                           f2v acc[2], lds_float *rk = nullptr) {
    float rd[4];
    const RdPair v[4] = {{r.p01.x, r.p01.y}, {r.p01.z, r.p01.w}, {r.p23.x, r.p23.y}, {r.p23.z, r.p23.w}};
    // a + t (b - a), one rounding after the product: within an ulp or two of the reference's
    // (1 - t) a + t b (the far values are a resampling already)
    // (written out: packed, the four bands' (a, b) pairs would first be shuffled into (a0, a1), (b0, b1)
    // register pairs -- three v_mov per two bands, more than the packing saves)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float t = r.f[j];  // (cg_fetch returns t)
        float d;
        asm("v_sub_f32 %0, %1, %2" : "=v"(d) : "v"(v[j].b), "v"(v[j].a));
        asm("v_fma_f32 %0, %1, %2, %3" : "=v"(rd[j]) : "v"(t), "v"(d), "v"(v[j].a));
    }
    (void)d2;
    float o[4];
    if (RGB) from_rgb4_fused(rk, rd[0], rd[1], rd[2], o);  // slots 0..2: the R, G, B profiles on the grid
    const float *x = RGB ? o : rd;
    (void)w;
#pragma unroll
    for (int h = 0; h < 2; ++h)  // acc += Rd * (E area), one packed FMA per two bands
        acc[h] = __builtin_elementwise_fma(f2v{x[2 * h], x[2 * h + 1]}, f2v{e[2 * h], e[2 * h + 1]}, acc[h]);
}

template <bool POINT, bool COUNT, int KLDS, bool RGB = false>
__device__ __forceinline__ void band_rd_accumulate(const BandLane &b, float d2, const float e[4], float w, f2v acc[2],
                                                   int hist[kHist], lds_float *rk = nullptr) {
    float f[4];
    RdPair v[4];
    band_rd_fetch<COUNT, KLDS>(b, d2, f, v, hist);
    band_rd_combine<POINT, RGB>(f, v, e, w, acc, rk);
}

// sum_area / d2 < max_error decided without an IEEE division in the common case: a against the products
// d m_lo and d m_hi (m_lo, m_hi = m (1 -+ 2^-20)): a < fl(d m_lo) puts the true quotient below m (1 - 2^-21),
// a > fl(d m_hi) above m (1 + 2^-21) -- two plain multiplies and compares (a v_rcp_f32 issues at a quarter of
// a multiply's rate: the multiplies measured 0.7 % faster once the gather was VALU-bound,
// profiles/r06_grid_ab.txt r06n). The rare near-ties (and NaN / inf) take the exact division, so the
// decision is always that of fl(sum_area / d2) < max_error (diffusionutil.h:182).
__device__ __forceinline__ bool dw_below(float a, float d, float m, float m_lo, float m_hi) {
    // (the masks as ballots: two compares, the rest scalar mask logic)
    const uint64_t m_below = __builtin_amdgcn_ballot_w64(a < d * m_lo);
    const uint64_t m_above = __builtin_amdgcn_ballot_w64(a > d * m_hi);
    bool below = __builtin_amdgcn_inverse_ballot_w64(m_below);
    if (__builtin_amdgcn_inverse_ballot_w64(~(m_below | m_above))) below = (a / d) < m;
    return below;
}

// COUNT: k_nodes / k_pts = this lane's node / point visits; w_nodes / w_pts = the wave's node-loop
// and point-loop iterations (uniform).
// A leaf's points are taken two at a time -- both points' eight pair loads issued before either's
// terms are formed (the same terms, summed in the same order), so a wave waits out one L2 round
// trip per two points.
// CG: far lookups from the group's common grid (CommonGrid; the LDS holds the exact near field in
// CommonGrid::lrow's per-slot rows), else every band from its own table (bit-identical to the packet
// kernel).
template <bool COUNT, int KLDS, bool VROWS, bool CG = false, bool RGB = false>
__device__ __forceinline__ void mo_band_traverse(const BandTree &a, int grp, float px, float py, float pz, bool valid,
                                                 float out[4], int &k_nodes, int &k_pts, int &w_nodes, int &w_pts,
                                                 int hist[kHist], const float *lt) {
    BandLane b;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = a.lband[grp][j];
        b.rcp[j] = a.grcp[grp][j];
        b.off[j] = (uint32_t)(c >= 0 ? c : 0) * (uint32_t)a.L;
    }
    lds_float *rk = (lds_float *)lt + 4 * near_row<KLDS>() - 28;  // RGB: the group's FromRGB weights (LDS)
    b.lm1 = (uint32_t)(a.L - 1);
    const uint32_t lm2 = b.lm1 - 1u;  // L >= 2
    b.klim = (uint32_t)KLDS < lm2 ? (uint32_t)KLDS : lm2;
    b.gspan = b.lm1 - b.klim;
#pragma unroll
    for (int j = 0; j < 4; ++j) b.tb[j] = VROWS ? in_vgprs(a.table + b.off[j]) : a.table + b.off[j];
    b.lt = lt;
    b.ltl = (lds_float *)lt;
    CgLane cl;
    if (CG) {
        cl.tab = a.cg.tab;
        cl.rowoff = a.cg.row0[grp] - a.cg.ubase[grp];
        cl.rg = a.cg.rg[grp];
        cl.u0lim = a.cg.u0lim[grp];
        cl.u1lim = a.cg.u1lim[grp];
        cl.hinv = in_vgpr(a.cg.hinv[grp]);
        cl.hc = a.cg.hc[grp];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            cl.lrow[j] = a.cg.lrow[grp][j];
            cl.off[j] = b.off[j];
        }
        cl.lm1 = (uint32_t)a.L - 1u;
        cl.zoff = 4u * (uint32_t)NB * (uint32_t)a.L;
    }
    f2v acc[2] = {f2v{0.f, 0.f}, f2v{0.f, 0.f}};
    // a leaf whose points all lie within the near field of every band of the group, for any query that
    // opens it: leaf_r2 * rcp_max < klim (with a 1e-5 margin for the roundings of d2 and f)
    const float lds_r2_lim = !a.leaf_r2 ? 0.f : CG ? a.cg.lds_r2[grp] : (float)b.klim / (a.grcp_max[grp] * 1.00001f);
    // as a leaf code (NodeHdr::pad's high half, DeviceOctree::ensure_leaf_r2: leaf_r2's high 16 bits
    // rounded up): code < lim_code => leaf_r2 < lds_r2_lim (a leaf within a rounding of the limit
    // takes the general loop)
    const uint32_t lds_code = __float_as_uint(lds_r2_lim) >> 16;
    // box2 * rcp_min >= prune_f as one compare: prune_f carries a 1e-4 margin over the profile end,
    // far above the rounding of the quotient (rcp_min 0: pruning off, INF)
    const float box_lim = a.prune_f / a.groups.rcp_min[grp];
    const cptr<float4> et_g = as_const(a.band_et + (size_t)grp * a.n_nodes);
    // (the common-grid gather's fused products read E * area)
    const cptr<float4> e_g = as_const((CG ? a.band_ew : a.band_e) + (size_t)grp * a.n_points);
    const cptr<NodeHdr> nodes = as_const(a.nodes);
    const cptr<float4> pt_hdr = as_const(a.pt_hdr);
    int resume = valid ? 0 : 0x7fffffff;
    const float m_lo = a.max_error * (1.f - 0x1p-20f), m_hi = a.max_error * (1.f + 0x1p-20f);  // (dw_below)
    int node = 0;
    while (node < a.n_nodes) {
        node = __builtin_amdgcn_readfirstlane(node);
        if (COUNT) ++w_nodes;
        const NodeHdr h = nodes[node];
        // the whole 64-B header (one scalar-cache line) in one load, waited for once, instead of
        // pieces loaded as the decisions below need them (each a further scalar-cache round trip);
        // all 16 words named, so that it is one s_load_dwordx16 rather than x8 + x4 + x2 for the 14 the
        // walk reads (C2 gather -0.6 %, profiles/r06_grid_ab.txt r06z)
        asm volatile("" ::"s"(h.px), "s"(h.py), "s"(h.pz), "s"(h.sum_area), "s"(h.bminx), "s"(h.bminy),
                     "s"(h.bminz), "s"(h.bmaxx), "s"(h.bmaxy), "s"(h.bmaxz), "s"(h.skip), "s"(h.leaf_first),
                     "s"(h.flags), "s"(h.pad), "s"(h.leaf_count), "s"(h.depth));
        const int skip = h.skip;
        bool open = false;
        if (node >= resume) {
            if (COUNT) ++k_nodes;
            // distance from p to the node box per axis (0 inside the slab)
            const float bx = fmaxf(fmaxf(h.bminx - px, px - h.bmaxx), 0.f);
            const float by = fmaxf(fmaxf(h.bminy - py, py - h.bmaxy), 0.f);
            const float bz = fmaxf(fmaxf(h.bminz - pz, pz - h.bmaxz), 0.f);
            // exact-zero pruning with a 1e-4 margin (prune_f), so the test may round freely
            const float box2 = __builtin_fmaf(bz, bz, __builtin_fmaf(by, by, bx * bx));
            if (box2 >= box_lim || (h.flags & NODE_BLACK)) {
                resume = skip;
            } else {
                const float dx = px - h.px, dy = py - h.py, dz = pz - h.pz;
                const float d2 = dx * dx + dy * dy + dz * dz;
                // nodeBound.Inside(p) <=> every per-axis distance is 0 (the subtractions' signs are exact)
                const bool inside = fmaxf(fmaxf(bx, by), bz) == 0.f;
                if (dw_below(h.sum_area, d2, a.max_error, m_lo, m_hi) && !inside) {
                    resume = skip;
                    if (CG) {
                        CgRec r = cg_fetch<COUNT>(b, cl, a.table, d2, hist);
                        // Et's scalar load issued behind the record's table loads: issued before them,
                        // the wait for the LDS step's reads (lgkmcnt) would wait for it too
                        int nd = node;
                        asm volatile("" : "+s"(nd)::"memory");
                        const float4 et = et_g[nd];
                        const float e[4] = {et.x, et.y, et.z, et.w};
                        cg_fix<COUNT>(b, cl, a.table, d2, r, hist);
                        cg_combine<false, RGB>(cl, r, d2, e, 1.f, acc, rk);
                    } else {
                        const float4 et = et_g[node];
                        const float e[4] = {et.x, et.y, et.z, et.w};
                        band_rd_accumulate<false, COUNT, KLDS, RGB>(b, d2, e, 1.f, acc, hist, rk);
                    }
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
                const int live = (int)(h.pad & 0xffffu);
                if (COUNT) w_pts += live;
                int i0 = 0;
                if (!COUNT && KLDS > 0 && (h.pad >> 16) < lds_code) {
                    for (; i0 + 1 < live; i0 += 2) {
                        const int ka = h.leaf_first + i0, kb = ka + 1;
                        const float4 pa = pt_hdr[ka], pb = pt_hdr[kb];
                        const float4 ea = e_g[ka], eb = e_g[kb];
                        if (!open) continue;
                        const float ax = px - pa.x, ay = py - pa.y, az = pz - pa.z;
                        const float bx2 = px - pb.x, by2 = py - pb.y, bz2 = pz - pb.z;
                        const float d2a = ax * ax + ay * ay + az * az;
                        const float d2b = bx2 * bx2 + by2 * by2 + bz2 * bz2;
                        const float e0[4] = {ea.x, ea.y, ea.z, ea.w}, e1[4] = {eb.x, eb.y, eb.z, eb.w};
                        if (CG) {
                            const CgRec ra = cg_fetch_near(b, cl, d2a), rb = cg_fetch_near(b, cl, d2b);
                            cg_combine<true, RGB>(cl, ra, d2a, e0, pa.w, lacc, rk);
                            cg_combine<true, RGB>(cl, rb, d2b, e1, pb.w, lacc, rk);
                            continue;
                        }
                        float fa[4], fb[4];
                        RdPair va[4], vb[4];
                        band_rd_fetch_lds<KLDS>(b, d2a, fa, va);
                        band_rd_fetch_lds<KLDS>(b, d2b, fb, vb);
                        band_rd_combine<true, RGB>(fa, va, e0, pa.w, lacc, rk);
                        band_rd_combine<true, RGB>(fb, vb, e1, pb.w, lacc, rk);
                    }
                }
                for (; i0 + 1 < live; i0 += 2) {
                        const int ka = h.leaf_first + i0, kb = ka + 1;
                        const float4 pa = pt_hdr[ka], pb = pt_hdr[kb];
                        const float4 ea = e_g[ka], eb = e_g[kb];
                        // both points' headers and E in one scalar round trip: loaded later, the wait for
                        // them would also wait out the table loads already in flight (a flat load counts in
                        // lgkmcnt too) and split the pair's lookups into two round trips
                        if (!COUNT)
                            asm volatile("" ::"s"(pa.x), "s"(pa.y), "s"(pa.z), "s"(pa.w), "s"(pb.x), "s"(pb.y),
                                         "s"(pb.z), "s"(pb.w), "s"(ea.x), "s"(ea.y), "s"(ea.z), "s"(ea.w),
                                         "s"(eb.x), "s"(eb.y), "s"(eb.z), "s"(eb.w));
                        if (!open) continue;
                        if (COUNT) k_pts += 2;
                        const float ax = px - pa.x, ay = py - pa.y, az = pz - pa.z;
                        const float bx2 = px - pb.x, by2 = py - pb.y, bz2 = pz - pb.z;
                        const float d2a = ax * ax + ay * ay + az * az;
                        const float d2b = bx2 * bx2 + by2 * by2 + bz2 * bz2;
                        if (CG) {
                            CgRec ra = cg_fetch<COUNT>(b, cl, a.table, d2a, hist);
                            CgRec rb = cg_fetch<COUNT>(b, cl, a.table, d2b, hist);
                            cg_fix2<COUNT>(b, cl, a.table, d2a, ra, d2b, rb, hist);
                            const float e0[4] = {ea.x, ea.y, ea.z, ea.w}, e1[4] = {eb.x, eb.y, eb.z, eb.w};
                            cg_combine<true, RGB>(cl, ra, d2a, e0, pa.w, lacc, rk);
                            cg_combine<true, RGB>(cl, rb, d2b, e1, pb.w, lacc, rk);
                            continue;
                        }
                        float fa[4], fb[4];
                        RdPair va[4], vb[4];
                        band_rd_fetch<COUNT, KLDS>(b, d2a, fa, va, hist);
                        band_rd_fetch<COUNT, KLDS>(b, d2b, fb, vb, hist);
                        // all eight lookups in flight before the first is consumed
                        if (!COUNT)
                            asm volatile("" ::"v"(va[0].a), "v"(va[0].b), "v"(va[1].a), "v"(va[1].b), "v"(va[2].a),
                                         "v"(va[2].b), "v"(va[3].a), "v"(va[3].b), "v"(vb[0].a), "v"(vb[0].b),
                                         "v"(vb[1].a), "v"(vb[1].b), "v"(vb[2].a), "v"(vb[2].b), "v"(vb[3].a),
                                         "v"(vb[3].b));
                        const float e0[4] = {ea.x, ea.y, ea.z, ea.w}, e1[4] = {eb.x, eb.y, eb.z, eb.w};
                        band_rd_combine<true, RGB>(fa, va, e0, pa.w, lacc, rk);
                        band_rd_combine<true, RGB>(fb, vb, e1, pb.w, lacc, rk);
                    }
                for (int i = i0; i < live; ++i) {
                    const int kp = h.leaf_first + i;
                    const float4 ph = pt_hdr[kp];
                    if (!open) continue;
                    if (COUNT) ++k_pts;
                    const float ex = px - ph.x, ey = py - ph.y, ez = pz - ph.z;
                    const float d2 = ex * ex + ey * ey + ez * ez;
                    if (CG) {
                        CgRec r = cg_fetch<COUNT>(b, cl, a.table, d2, hist);
                        int kq = kp;  // (E's scalar load behind the table loads, as Et's)
                        asm volatile("" : "+s"(kq)::"memory");
                        const float4 ev = e_g[kq];
                        const float e[4] = {ev.x, ev.y, ev.z, ev.w};
                        cg_fix<COUNT>(b, cl, a.table, d2, r, hist);
                        cg_combine<true, RGB>(cl, r, d2, e, ph.w, lacc, rk);
                    } else {
                        const float4 ev = e_g[kp];
                        const float e[4] = {ev.x, ev.y, ev.z, ev.w};
                        band_rd_accumulate<true, COUNT, KLDS, RGB>(b, d2, e, ph.w, lacc, hist, rk);
                    }
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

// 30-bit Morton code of a point in [lo, lo + 1/inv) per axis (10 bits per axis, clamped).
__device__ __forceinline__ uint32_t morton_expand10(uint32_t v) {
    v &= 0x3ffu;
    v = (v | (v << 16)) & 0x030000ffu;
    v = (v | (v << 8)) & 0x0300f00fu;
    v = (v | (v << 4)) & 0x030c30c3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}
__device__ __forceinline__ uint32_t morton30(float x, float y, float z, const float lo[3], const float inv[3]) {
    const float q[3] = {(x - lo[0]) * inv[0], (y - lo[1]) * inv[1], (z - lo[2]) * inv[2]};
    uint32_t c[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) c[k] = (uint32_t)fminf(fmaxf(q[k], 0.f), 1023.f);
    return (morton_expand10(c[0]) << 2) | (morton_expand10(c[1]) << 1) | morton_expand10(c[2]);
}
#endif

}  // namespace mpss
