// octree.h -- irradiance-point octree: host build + HBM layout for the Mo() gather kernel.
//
// Build follows SubsurfaceOctreeNode::Insert / InitHierarchy (reference
// src/integrators/diffusionutil.h:94-173) and the Preprocess loop
// (src/integrators/multipolesubsurface.cpp:301-321), inserting points in index order.
//
// HBM layout (pre-order, children in octant order 0..7, so every subtree is contiguous):
//   NodeHdr[N]   64 B each: cluster centroid p, sumArea, node bounds, skip (= index after the
//                subtree), leaf point range, depth, flags (bit0: Et is black)
//   node_et[N][32]   Et per band, 30 bands + 2 pad lanes -> one 128-B line per node
//   pt_hdr[M]    float4 {p.x, p.y, p.z, area}; area's sign bit set  <=> point E is black
//   pt_e[M][32]  E per band (same 128-B row layout)
// Points are stored in leaf order (leaf k's points are contiguous, in the leaf's ips[] order).
#pragma once
#include <vector>
#include "common.h"

namespace mpss {

struct alignas(16) NodeHdr {
    float px, py, pz, sum_area;
    float bminx, bminy, bminz, bmaxx;
    float bmaxy, bmaxz;
    int32_t skip, leaf_first;  // leaf_first < 0 for interior nodes
    int32_t leaf_count, depth;
    uint32_t flags, pad;
};
static_assert(sizeof(NodeHdr) == 64, "NodeHdr must be one 64-B record");

enum : uint32_t { NODE_BLACK = 1u };

struct FlatOctree {
    std::vector<NodeHdr> hdr;
    std::vector<float> node_et;  // N * ROW
    std::vector<float> pt_hdr;   // M * 4
    std::vector<float> pt_e;     // M * ROW
    std::vector<int32_t> pt_index;  // leaf slot -> original point index
    int max_depth = 0;
    float bmin[3], bmax[3];
};

// p, n: npts*3; E: npts*NB; area: npts.  Throws Error on degenerate input.
void build_octree(int npts, const float *p, const float *n, const float *E, const float *area, FlatOctree &out);

}  // namespace mpss
