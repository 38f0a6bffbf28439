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
#include "mo_kernel.h"
#include "mo_packet.h"

#include <cstring>
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
};

__device__ __forceinline__ float rd_lerp(const float *__restrict__ tb, float f) {
    const uint32_t s = (uint32_t)f;
    const float t = f - (float)s;
    const float a = tb[s], b = tb[s + 1];
    return (1.f - t) * a + t * b;
}

__device__ __forceinline__ float box_d2(float px, float py, float pz, const NodeHdr &h) {
    const float bx = fmaxf(fmaxf(h.bminx - px, px - h.bmaxx), 0.f);
    const float by = fmaxf(fmaxf(h.bminy - py, py - h.bmaxy), 0.f);
    const float bz = fmaxf(fmaxf(h.bminz - pz, pz - h.bmaxz), 0.f);
    return bx * bx + by * by + bz * bz;
}

template <int MAXD, bool COUNT>
__global__ __launch_bounds__(256) void mo_gather_kernel(MoArgs a) {
    __shared__ float S[4][MAXD + 1][64];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int c = lane & 31;
    const int q = ((int)blockIdx.x * 4 + wave) * 2 + (lane >> 5);
    const bool active = q < a.nq;
    float(*St)[64] = S[wave];

    float px = 0.f, py = 0.f, pz = 0.f;
    if (active) {
        px = a.queries[3 * (size_t)q];
        py = a.queries[3 * (size_t)q + 1];
        pz = a.queries[3 * (size_t)q + 2];
    }
    const float rcp = c < NB ? a.rcp[c] : INFINITY;
    const float lm1 = (float)(a.L - 1);
    const float *__restrict__ tb = a.table + (size_t)(c < NB ? c : 0) * a.L;

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
                const float f = d2 * rcp;
                if (f < lm1) St[d][lane] += rd_lerp(tb, f) * a.node_et[(size_t)node * ROW + c];
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

// ---------------------------------------------------------------------------------------
// Spectrally sharded gather (mo_band.h): block b runs band group b % 8 for queries
// [1024 * (b / 8), +1024); query count read on the device (render path: compacted list).
// ---------------------------------------------------------------------------------------
struct BandArgs {
    BandTree t;
    const float *__restrict__ queries3;  // q * 3 (batch API) or null
    const float4 *__restrict__ queries4; // {p, *} (render path) or null
    const int *__restrict__ count;       // device query count (nullable: use nq)
    int nq;
    float *__restrict__ out;             // mode 0: out[q * stride + band]
    float4 *__restrict__ out4;           // mode 1: out4[q * 8 + group]
    int out_stride;
    int32_t *__restrict__ counters;      // batch API COUNT: q * 4 (+= per group)
    unsigned long long *__restrict__ counts;  // render COUNT: [2 * kGroups]
};

template <bool COUNT, int KLDS, bool FLAT>
__device__ __forceinline__ void mo_band_body(const BandArgs &a, float *lt) {
    const int grp = (int)(blockIdx.x & (kGroups - 1));
    const int base = (int)(blockIdx.x / kGroups) * kBandBlock;
    const int nq = a.count ? *a.count : a.nq;
    if (base >= nq) return;
    // the group's near-field Rd entries, KLDS per band + a zero pair
    for (int i = (int)threadIdx.x; i < 4 * (KLDS + 2); i += kBandBlock) {
        const int j = i / (KLDS + 2), k = i % (KLDS + 2), c = a.t.groups.band[grp][j];
        lt[i] = (c >= 0 && k < KLDS && k < a.t.L) ? a.t.table[(size_t)c * a.t.L + k] : 0.f;
    }
    __syncthreads();
    const int q = base + (int)threadIdx.x;
    const bool valid = q < nq;
    float px = 0.f, py = 0.f, pz = 0.f;
    bool live = valid;
    if (valid) {
        if (a.queries4) {
            const float4 v = a.queries4[q];
            px = v.x;
            py = v.y;
            pz = v.z;
            live = v.w >= 0.f;  // render hit list: w < 0 marks hits without a BSSRDF
        } else {
            px = a.queries3[3 * (size_t)q];
            py = a.queries3[3 * (size_t)q + 1];
            pz = a.queries3[3 * (size_t)q + 2];
        }
    }
    float acc[4];
    int kn = 0, kp = 0;
    mo_band_traverse<COUNT, KLDS, FLAT>(a.t, grp, px, py, pz, live, acc, kn, kp, lt);
    if (!live) return;
    if (a.out4) {
        a.out4[(size_t)q * kGroups + grp] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = a.t.groups.band[grp][j];
            if (c >= 0) a.out[(size_t)q * a.out_stride + c] = acc[j];
        }
    }
    if (COUNT) {
        if (a.counters) {
            atomicAdd(&a.counters[4 * (size_t)q + 2], kn);
            atomicAdd(&a.counters[4 * (size_t)q + 3], kp);
        }
        if (a.counts) {
            atomicAdd(&a.counts[2 * grp], (unsigned long long)kn);
            atomicAdd(&a.counts[2 * grp + 1], (unsigned long long)kp);
        }
    }
}

// Variants of one body: 64 KB of LDS (two workgroups = 32 waves a CU) with wave-uniform LDS /
// table reads; the same with one per-lane flat load (address in LDS or in the table); one
// workgroup a CU with 160 KB of LDS (a larger near field in LDS).
template <bool COUNT>
__global__ __launch_bounds__(kBandBlock) void mo_band_kernel(BandArgs a) {
    __shared__ float lt[4 * (kLdsRd + 2)];
    mo_band_body<COUNT, kLdsRd, false>(a, lt);
}
template <bool COUNT>
__global__ __launch_bounds__(kBandBlock) void mo_band_kernel_flat(BandArgs a) {
    __shared__ float lt[4 * (kLdsRd + 2)];
    mo_band_body<COUNT, kLdsRd, true>(a, lt);
}
template <bool COUNT>
__global__ __launch_bounds__(kBandBlock) void mo_band_kernel_big(BandArgs a) {
    __shared__ float lt[4 * (kLdsRdBig + 2)];
    mo_band_body<COUNT, kLdsRdBig, false>(a, lt);
}

// MPSS_MO_BAND selects the variant (0 default, 1 flat, 2 big LDS) -- a tuning knob
int band_variant() {
    const char *v = getenv("MPSS_MO_BAND");
    return v ? atoi(v) : 0;
}

void launch_band(const BandArgs &a, unsigned blocks, bool count, hipStream_t stream) {
    const int var = band_variant();
    if (var == 1) {
        if (count)
            hipLaunchKernelGGL(mo_band_kernel_flat<true>, dim3(blocks), dim3(kBandBlock), 0, stream, a);
        else
            hipLaunchKernelGGL(mo_band_kernel_flat<false>, dim3(blocks), dim3(kBandBlock), 0, stream, a);
    } else if (var == 2) {
        if (count)
            hipLaunchKernelGGL(mo_band_kernel_big<true>, dim3(blocks), dim3(kBandBlock), 0, stream, a);
        else
            hipLaunchKernelGGL(mo_band_kernel_big<false>, dim3(blocks), dim3(kBandBlock), 0, stream, a);
    } else {
        if (count)
            hipLaunchKernelGGL(mo_band_kernel<true>, dim3(blocks), dim3(kBandBlock), 0, stream, a);
        else
            hipLaunchKernelGGL(mo_band_kernel<false>, dim3(blocks), dim3(kBandBlock), 0, stream, a);
    }
    MPSS_HIP(hipGetLastError());
}

__global__ void band_permute_kernel(const float *__restrict__ rows, int n, BandGroups g, float4 *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)n * kGroups) return;
    const int grp = (int)(i / n), r = (int)(i % n);
    const float *row = rows + (size_t)r * ROW;
    float v[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) v[s] = g.band[grp][s] >= 0 ? row[g.band[grp][s]] : 0.f;
    out[i] = make_float4(v[0], v[1], v[2], v[3]);
}

BandTree band_tree(const DeviceOctree &t, const DeviceProfile &p, float max_error) {
    BandTree bt;
    bt.nodes = t.nodes.ptr;
    bt.band_et = t.band_et.ptr;
    bt.pt_hdr = t.pt_hdr.ptr;
    bt.band_e = t.band_e.ptr;
    bt.table = p.table.ptr;
    bt.rcp = p.rcp.ptr;
    bt.groups = p.groups;
    bt.L = p.L;
    bt.n_nodes = t.n_nodes;
    bt.n_points = t.n_points;
    bt.max_error = max_error;
    bt.prune_f = (p.rcp_min > 0.f) ? (float)(p.L - 1) * 1.0001f : INFINITY;
    if (!(p.rcp_min > 0.f))
        for (int g = 0; g < kGroups; ++g) bt.groups.rcp_min[g] = 0.f;  // rcp <= 0: no pruning
    return bt;
}

template <int MAXD>
void launch_t(const MoArgs &a, bool count, hipStream_t s) {
    const int waves = (a.nq + 1) / 2;
    const int blocks = (waves + 3) / 4;
    if (blocks == 0) return;
    if (count)
        hipLaunchKernelGGL((mo_gather_kernel<MAXD, true>), dim3(blocks), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((mo_gather_kernel<MAXD, false>), dim3(blocks), dim3(256), 0, s, a);
}

}  // namespace

// The device copy moves each leaf's black points (E == 0: every kernel skips them, they add
// nothing) behind its other points, keeping the others' order, and records the count of the
// rest in NodeHdr::pad, so the sharded gather's leaf loop needs no per-point test.
void DeviceOctree::upload(const FlatOctree &t) {
    std::vector<NodeHdr> hdr = t.hdr;
    std::vector<float> ph(t.pt_hdr.size()), pe(t.pt_e.size());
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
                ++o;
                if (pass == 0) ++h.pad;
            }
    }
    nodes.upload(hdr.data(), hdr.size());
    node_et.upload(t.node_et.data(), t.node_et.size());
    pt_hdr.upload(reinterpret_cast<const float4 *>(ph.data()), ph.size() / 4);
    pt_e.upload(pe.data(), pe.size());
    band_valid = false;
    n_nodes = (int)t.hdr.size();
    n_points = (int)t.pt_index.size();
    max_depth = t.max_depth;
}

void DeviceProfile::upload(const float *tab, int len, const float *rcp_) {
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
    groups = make_band_groups(rcp_);
}

void DeviceOctree::ensure_band_layout(const BandGroups &g, hipStream_t stream) {
    if (band_valid && memcmp(g.band, band_groups.band, sizeof(g.band)) == 0) return;
    band_et.alloc((size_t)n_nodes * kGroups);
    band_e.alloc((size_t)(n_points > 0 ? n_points : 1) * kGroups);
    const int64_t tn = (int64_t)n_nodes * kGroups, tp = (int64_t)n_points * kGroups;
    if (tn) hipLaunchKernelGGL(band_permute_kernel, dim3((unsigned)((tn + 255) / 256)), dim3(256), 0, stream,
                               node_et.ptr, n_nodes, g, band_et.ptr);
    if (tp) hipLaunchKernelGGL(band_permute_kernel, dim3((unsigned)((tp + 255) / 256)), dim3(256), 0, stream,
                               pt_e.ptr, n_points, g, band_e.ptr);
    MPSS_HIP(hipGetLastError());
    band_groups = g;
    band_valid = true;
}

void launch_mo_band(DeviceOctree &t, const DeviceProfile &p, float max_error, int nq_max, const float4 *queries4,
                    const int *count_dev, float4 *out4, unsigned long long *counts, hipStream_t stream) {
    if (nq_max <= 0) return;
    t.ensure_band_layout(p.groups, stream);
    BandArgs a{};
    a.t = band_tree(t, p, max_error);
    a.queries4 = queries4;
    a.count = count_dev;
    a.nq = nq_max;
    a.out4 = out4;
    a.counts = counts;
    const unsigned blocks = (unsigned)((nq_max + kBandBlock - 1) / kBandBlock) * kGroups;
    launch_band(a, blocks, counts != nullptr, stream);
}

void launch_mo_gather(const DeviceOctree &t_, const DeviceProfile &p, float max_error, int nq, const float *queries,
                      float *out, int out_stride, int32_t *counters, hipStream_t stream, int mode) {
    DeviceOctree &t = const_cast<DeviceOctree &>(t_);  // band layout is a cache of the octree
    const bool exact = mode == 1;
    if (nq <= 0) return;
    if (t.n_nodes <= 0) throw Error(-1, "launch_mo_gather: octree is empty");
    if (p.L < 2) throw Error(-1, "launch_mo_gather: profile table has fewer than 2 entries");
    MoArgs a;
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
    const bool count = counters != nullptr;
    if (mode == 0) {
        t.ensure_band_layout(p.groups, stream);
        if (count) MPSS_HIP(hipMemsetAsync(counters, 0, sizeof(int32_t) * 4 * (size_t)nq, stream));
        BandArgs b{};
        b.t = band_tree(t, p, max_error);
        b.queries3 = queries;
        b.nq = nq;
        b.out = out;
        b.out_stride = out_stride;
        b.counters = counters;
        const unsigned blocks = (unsigned)((nq + kBandBlock - 1) / kBandBlock) * kGroups;
        launch_band(b, blocks, count, stream);
        return;
    }
    if (!exact) {
        const int packets = (nq + 7) / 8, blocks = (packets + 3) / 4;
        if (count)
            hipLaunchKernelGGL((mo_packet_kernel<true>), dim3(blocks), dim3(256), 0, stream, a, blocks);
        else
            hipLaunchKernelGGL((mo_packet_kernel<false>), dim3(blocks), dim3(256), 0, stream, a, blocks);
        MPSS_HIP(hipGetLastError());
        return;
    }
    if (t.max_depth < 16)
        launch_t<16>(a, count, stream);
    else if (t.max_depth < 32)
        launch_t<32>(a, count, stream);
    else if (t.max_depth < 64)
        launch_t<64>(a, count, stream);
    else
        throw Error(-2, "octree deeper than 63 levels is not supported by the gather kernel");
    MPSS_HIP(hipGetLastError());
}

}  // namespace mpss
