// mo_packet.h -- the packet traversal of the Mo() gather (device), shared by the Mo batch
// kernel (mo_kernel.hip) and the render shading kernel (render.hip).
//
// One wave64 = a packet of 8 queries x 8 band-groups of 4 bands (lane = 8*g + k). The 8
// queries walk the UNION of their pruned traversals of the pre-order octree once: node and
// leaf-point headers are wave-uniform scalar loads, Et/E rows one 128-B line per wave, and
// each lane owns bands 4k..4k+3 of query g. A query that does not open node j (it pruned
// it, took its cluster contribution, or the node is black) sits out until j's skip index.
// Per query the visited node set, the decisions and every product are those of
// SubsurfaceOctreeNode::Mo (integrators/diffusionutil.h:175-210); only the order of the
// float additions differs (one running sum per band instead of the recursion's per-level
// sums), so results agree with the reference order to float reassociation (tests bound it
// at 2e-5 relative; the north-star tolerance is 1e-4).
#pragma once
#include "common.h"
#include "octree.h"

namespace mpss {

struct PacketTree {
    const NodeHdr *__restrict__ nodes;
    const float *__restrict__ node_et;
    const float4 *__restrict__ pt_hdr;
    const float *__restrict__ pt_e;
    const float *__restrict__ table;   // [NB][L] channel-major Rd table
    const float *__restrict__ rcp;
    int L, n_nodes;
    float max_error, prune_f, rcp_min;
};

// Bijective XCD-aware block remap (cdna_hip_programming.md 5.5 T1): logical blocks b and b+1
// (neighbouring queries) land on the same XCD, so they share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int b, int nblocks) {
    const int xcd = b & 7, qn = nblocks >> 3, rn = nblocks & 7;
    return (xcd < rn ? xcd * (qn + 1) : rn * (qn + 1) + (xcd - rn) * qn) + (b >> 3);
}

__device__ __forceinline__ float packet_box_d2(float px, float py, float pz, const NodeHdr &h) {
    const float bx = fmaxf(fmaxf(h.bminx - px, px - h.bmaxx), 0.f);
    const float by = fmaxf(fmaxf(h.bminy - py, py - h.bmaxy), 0.f);
    const float bz = fmaxf(fmaxf(h.bminz - pz, pz - h.bmaxz), 0.f);
    return bx * bx + by * by + bz * bz;
}

template <bool COUNT>
__device__ __forceinline__ void mo_packet_traverse(const PacketTree &a, float px, float py, float pz, bool valid,
                                                   int k, float acc[4], int &k_nodes, int &k_pts,
                                                   int *union_nodes = nullptr) {
    float rcp[4];
    const float *tb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = 4 * k + j;
        rcp[j] = c < NB ? a.rcp[c] : INFINITY;
        tb[j] = a.table + (size_t)(c < NB ? c : 0) * a.L;
        acc[j] = 0.f;
    }
    const float lm1 = (float)(a.L - 1);
    int resume = valid ? 0 : 0x7fffffff;
    int node = 0;
    while (node < a.n_nodes) {
        node = __builtin_amdgcn_readfirstlane(node);
        if (COUNT && union_nodes) ++*union_nodes;
        const NodeHdr h = a.nodes[node];
        const int skip = h.skip;
        bool open = false;
        if (node >= resume) {
            if (COUNT) ++k_nodes;
            const bool prune = packet_box_d2(px, py, pz, h) * a.rcp_min >= a.prune_f;
            if (prune || (h.flags & NODE_BLACK)) {
                resume = skip;
            } else {
                const float dx = px - h.px, dy = py - h.py, dz = pz - h.pz;
                const float d2 = dx * dx + dy * dy + dz * dz;
                const float dw = h.sum_area / d2;
                const bool inside = px >= h.bminx && px <= h.bmaxx && py >= h.bminy && py <= h.bmaxy &&
                                    pz >= h.bminz && pz <= h.bmaxz;
                if (dw < a.max_error && !inside) {
                    resume = skip;
                    const float4 et = reinterpret_cast<const float4 *>(a.node_et + (size_t)node * ROW)[k];
                    const float e[4] = {et.x, et.y, et.z, et.w};
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const float f = d2 * rcp[j];
                        if (f < lm1) {
                            const uint32_t s = (uint32_t)f;
                            const float t = f - (float)s;
                            const float ta = tb[j][s], tbb = tb[j][s + 1];
                            acc[j] += ((1.f - t) * ta + t * tbb) * e[j];
                        }
                    }
                } else {
                    open = true;  // leaf: evaluate its points; interior: descend
                }
            }
        }
        const bool any_open = __builtin_amdgcn_ballot_w64(open) != 0;
        if (h.leaf_first >= 0) {
            if (any_open) {
                float lacc[4] = {0.f, 0.f, 0.f, 0.f};
                for (int i = 0; i < h.leaf_count; ++i) {
                    const int kp = h.leaf_first + i;
                    const float4 ph = a.pt_hdr[kp];
                    if (__builtin_signbit(ph.w)) continue;  // E is black
                    if (!open) continue;
                    if (COUNT) ++k_pts;
                    const float ex = px - ph.x, ey = py - ph.y, ez = pz - ph.z;
                    const float d2 = ex * ex + ey * ey + ez * ez;
                    const float4 ev = reinterpret_cast<const float4 *>(a.pt_e + (size_t)kp * ROW)[k];
                    const float e[4] = {ev.x, ev.y, ev.z, ev.w};
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const float f = d2 * rcp[j];
                        if (f < lm1) {
                            const uint32_t s = (uint32_t)f;
                            const float t = f - (float)s;
                            const float ta = tb[j][s], tbb = tb[j][s + 1];
                            lacc[j] += ((1.f - t) * ta + t * tbb) * e[j] * ph.w;
                        }
                    }
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

}  // namespace mpss
