// octree_gpu.hip -- the irradiance-point octree built on the device, level by level.
//
// SubsurfaceOctreeNode::Insert (reference src/integrators/diffusionutil.h:94-132) inserts the
// points one at a time in index order: a leaf holds up to 8 points and splits on the 9th, re-placing
// its points in arrival order. The final tree therefore does not depend on the insertion
// sequence except through two facts this build reproduces exactly:
//   * a node is interior iff at least 9 points fall in its box (octant tests against the float
//     midpoint .5*pMin + .5*pMax of the box, child boxes as octreeChildBound, core/octree.h:87-97);
//     a child exists iff some point falls in it;
//   * a leaf's points are in increasing point index (the order they arrived in).
// Each level is one stable radix sort of the points by (position of their node's first point,
// octant): a stable segmented partition that keeps every finished leaf's points in place and the
// points of a split node in index order within each octant. The point array then holds the
// leaves in pre-order, children in octant order -- the FlatOctree order (octree.cpp).
// InitHierarchy (diffusionutil.h:133-173) runs bottom-up one level per launch, one thread per node,
// with the host build's float operations in the same order (children / points in slot order), and
// the pre-order numbering top-down from the subtree sizes. Output: the DeviceOctree arrays
// (mo_kernel.h), bit-identical to DeviceOctree::upload of the host build (tests/test_octree_gpu.py).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>

#include "mo_kernel.h"
#include "spectral.h"

namespace mpss {

namespace {

__constant__ float kCieY[NB] = MPSS_BAND_CIE_Y_INIT;

__device__ __forceinline__ float band_y(const float *s) {  // spectrum_y (spectral.h), same operation order
    float yy = 0.f;
#pragma unroll
    for (int i = 0; i < NB; ++i) yy += kCieY[i] * s[i];
    return yy * (float)(700 - 400) / (float)(MPSS_CIE_Y_INTEGRAL * NB);
}

// Build-order node arrays (level by level; within a level in point-array order).
struct Nodes {
    int *start, *count, *parent, *level, *first_child, *nchild, *size, *pre;
    float4 *lo, *hi;  // box (w unused)
    float *et;        // [g * NB]
    float4 *pn;       // {p, sum_area}
    float4 *nn;       // {n, -}
};

__device__ __forceinline__ void mid_of(const float4 &lo, const float4 &hi, float m[3]) {
    m[0] = .5f * lo.x + .5f * hi.x;
    m[1] = .5f * lo.y + .5f * hi.y;
    m[2] = .5f * lo.z + .5f * hi.z;
}

// key = (first point position of the node << 3) | octant for points of a node that splits (>= 9
// points), (own position << 3) for every other point: a stable sort by key partitions each split
// node by octant and moves nothing else.
__global__ void level_keys_kernel(int n, const float *__restrict__ P, const int *__restrict__ orig,
                                  const int *__restrict__ nid, Nodes nd, uint32_t *__restrict__ key) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= n) return;
    const int g = nid[i];
    uint32_t k = (uint32_t)i << 3;
    if (g >= 0 && nd.count[g] > 8) {
        float m[3];
        mid_of(nd.lo[g], nd.hi[g], m);
        const float *p = P + 3 * (size_t)orig[i];
        const int c = (p[0] > m[0] ? 4 : 0) + (p[1] > m[1] ? 2 : 0) + (p[2] > m[2] ? 1 : 0);
        k = ((uint32_t)nd.start[g] << 3) | (uint32_t)c;
    }
    key[i] = k;
}

// head[i] = 1 where a child node's points start (inside split nodes only)
__global__ void level_heads_kernel(int n, const int *__restrict__ nid, Nodes nd, const uint32_t *__restrict__ key,
                                   int *__restrict__ head) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= n) return;
    const int g = nid[i];
    int h = 0;
    if (g >= 0 && nd.count[g] > 8) h = (i == nd.start[g] || key[i] != key[i - 1]) ? 1 : 0;
    head[i] = h;
}

// One new node per head: box = octreeChildBound of the parent's box for the octant.
__global__ void level_nodes_kernel(int n, int base, int lvl, const int *__restrict__ nid, const uint32_t *__restrict__ key,
                                   const int *__restrict__ head, const int *__restrict__ idx, Nodes nd) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= n || !head[i]) return;
    const int j = base + idx[i], par = nid[i], c = (int)(key[i] & 7u);
    const float4 lo = nd.lo[par], hi = nd.hi[par];
    float m[3];
    mid_of(lo, hi, m);
    const bool ux = (c >> 2) & 1, uy = (c >> 1) & 1, uz = c & 1;
    nd.lo[j] = make_float4(ux ? m[0] : lo.x, uy ? m[1] : lo.y, uz ? m[2] : lo.z, 0.f);
    nd.hi[j] = make_float4(ux ? hi.x : m[0], uy ? hi.y : m[1], uz ? hi.z : m[2], 0.f);
    nd.start[j] = i;
    nd.parent[j] = par;
    nd.level[j] = lvl;
    nd.first_child[j] = -1;
    nd.nchild[j] = 0;
    if (i == nd.start[par]) nd.first_child[par] = j;  // the parent's first point starts its first child
    atomicAdd(&nd.nchild[par], 1);
}

// Each point of a split node moves to its child (the run of its head); the others are done. The
// run's last point writes the child's count (no atomics: a level-1 node holds ~n / 8 points).
__global__ void level_assign_kernel(int n, int base, const int *__restrict__ nid, const int *__restrict__ head,
                                    const int *__restrict__ idx, Nodes nd, int *__restrict__ nid_out) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= n) return;
    const int g = nid[i];
    int o = -1;
    if (g >= 0 && nd.count[g] > 8) {
        o = base + idx[i] + head[i] - 1;  // inclusive scan - 1: this point's run
        const bool tail = i + 1 == nd.start[g] + nd.count[g] || head[i + 1];
        if (tail) nd.count[o] = i + 1 - nd.start[o];
    }
    nid_out[i] = o;
}

// InitHierarchy for one level (diffusionutil.h:133-173; octree.cpp Builder::init): a leaf sums its
// points, an interior node its children, in slot order; p, n weighted by luminance.
__global__ void init_level_kernel(int lo_g, int hi_g, Nodes nd, const int *__restrict__ orig, const float *__restrict__ P,
                                  const float *__restrict__ N, const float *__restrict__ E,
                                  const float *__restrict__ A) {
    const int g = lo_g + (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (g >= hi_g) return;
    float et[NB], p[3] = {0.f, 0.f, 0.f}, nrm[3] = {0.f, 0.f, 0.f}, sum_wt = 0.f, sum_area = 0.f;
    for (int c = 0; c < NB; ++c) et[c] = 0.f;
    const bool leaf = nd.nchild[g] == 0;
    const int k0 = leaf ? nd.start[g] : nd.first_child[g];
    const int cnt = leaf ? nd.count[g] : nd.nchild[g];
    int size = 1;
    for (int k = 0; k < cnt; ++k) {
        float e[NB], pp[3], nn[3], area;
        if (leaf) {
            const int ip = orig[k0 + k];
            area = A[ip];
            for (int c = 0; c < NB; ++c) e[c] = E[(size_t)ip * NB + c] * area;
            for (int a = 0; a < 3; ++a) {
                pp[a] = P[3 * (size_t)ip + a];
                nn[a] = N[3 * (size_t)ip + a];
            }
        } else {
            const int ch = k0 + k;
            for (int c = 0; c < NB; ++c) e[c] = nd.et[(size_t)ch * NB + c];
            const float4 cp = nd.pn[ch], cn = nd.nn[ch];
            pp[0] = cp.x; pp[1] = cp.y; pp[2] = cp.z;
            nn[0] = cn.x; nn[1] = cn.y; nn[2] = cn.z;
            area = cp.w;
            size += nd.size[ch];
        }
        const float wt = band_y(e);
        for (int c = 0; c < NB; ++c) et[c] += e[c];
        for (int a = 0; a < 3; ++a) {
            p[a] += pp[a] * wt;
            nrm[a] += nn[a] * wt;
        }
        sum_wt += wt;
        sum_area += area;
    }
    if (sum_wt > 0.f) {
        const float inv = 1.f / sum_wt;
        for (int a = 0; a < 3; ++a) {
            p[a] *= inv;
            nrm[a] *= inv;
        }
    }
    for (int c = 0; c < NB; ++c) nd.et[(size_t)g * NB + c] = et[c];
    nd.pn[g] = make_float4(p[0], p[1], p[2], sum_area);
    nd.nn[g] = make_float4(nrm[0], nrm[1], nrm[2], 0.f);
    nd.size[g] = size;
}

// Pre-order numbers of one level's children: children in octant order after their parent.
__global__ void preorder_level_kernel(int lo_g, int hi_g, Nodes nd) {
    const int g = lo_g + (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (g >= hi_g || nd.nchild[g] == 0) return;
    int run = nd.pre[g] + 1;
    for (int k = 0; k < nd.nchild[g]; ++k) {
        const int ch = nd.first_child[g] + k;
        nd.pre[ch] = run;
        run += nd.size[ch];
    }
}

__device__ __forceinline__ bool row_black(const float *s) {
    for (int c = 0; c < NB; ++c)
        if (s[c] != 0.f) return false;
    return true;
}

// NodeHdr / node_et at the pre-order slot; a leaf also writes its points (non-black first, in slot
// order, then the black ones: DeviceOctree::upload's device order) and their original indices.
__global__ void emit_kernel(int n_nodes, Nodes nd, const int *__restrict__ orig, const float *__restrict__ P,
                            const float *__restrict__ E, const float *__restrict__ A, NodeHdr *__restrict__ hdr,
                            float *__restrict__ node_et, float4 *__restrict__ pt_hdr, float *__restrict__ pt_e,
                            int *__restrict__ pt_index) {
    const int g = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (g >= n_nodes) return;
    const int me = nd.pre[g];
    const float4 pn = nd.pn[g], lo = nd.lo[g], hi = nd.hi[g];
    const float *et = nd.et + (size_t)g * NB;
    NodeHdr h;
    h.px = pn.x;
    h.py = pn.y;
    h.pz = pn.z;
    h.sum_area = pn.w;
    h.bminx = lo.x;
    h.bminy = lo.y;
    h.bminz = lo.z;
    h.bmaxx = hi.x;
    h.bmaxy = hi.y;
    h.bmaxz = hi.z;
    h.skip = me + nd.size[g];
    h.depth = nd.level[g];
    h.flags = row_black(et) ? NODE_BLACK : 0u;
    h.pad = 0;
    float *row = node_et + (size_t)me * ROW;
    for (int c = 0; c < NB; ++c) row[c] = et[c];
    for (int c = NB; c < ROW; ++c) row[c] = 0.f;
    if (nd.nchild[g] == 0) {
        h.leaf_first = nd.start[g];
        h.leaf_count = nd.count[g];
        int o = nd.start[g];
        for (int pass = 0; pass < 2; ++pass)
            for (int k = 0; k < nd.count[g]; ++k) {
                const int ip = orig[nd.start[g] + k];
                const float *e = E + (size_t)ip * NB;
                const bool blk = row_black(e);
                if (blk != (pass == 1)) continue;
                const float a = A[ip];
                pt_hdr[o] = make_float4(P[3 * (size_t)ip], P[3 * (size_t)ip + 1], P[3 * (size_t)ip + 2],
                                        blk ? copysignf(a, -1.f) : a);
                float *pr = pt_e + (size_t)o * ROW;
                for (int c = 0; c < NB; ++c) pr[c] = e[c];
                for (int c = NB; c < ROW; ++c) pr[c] = 0.f;
                pt_index[o] = ip;
                ++o;
                if (pass == 0) ++h.pad;
            }
    } else {
        h.leaf_first = -1;
        h.leaf_count = 0;
    }
    hdr[me] = h;
}

inline unsigned grid_of(int64_t n) { return (unsigned)((n + 255) / 256); }

// Node arrays with a growable capacity (device-to-device copy on growth).
struct NodeStore {
    DevBuf<int> start, count, parent, level, first_child, nchild, size, pre;
    DevBuf<float4> lo, hi, pn, nn;
    DevBuf<float> et;
    size_t cap = 0;
    template <class T>
    static void grow(DevBuf<T> &b, size_t used, size_t cap) {
        DevBuf<T> nb;
        nb.alloc(cap);
        if (used) MPSS_HIP(hipMemcpy(nb.ptr, b.ptr, used * sizeof(T), hipMemcpyDeviceToDevice));
        std::swap(b.ptr, nb.ptr);
        std::swap(b.n, nb.n);
    }
    void reserve(size_t used, size_t want) {
        if (want <= cap) return;
        size_t c = std::max(want, cap * 2);
        grow(start, used, c); grow(count, used, c); grow(parent, used, c); grow(level, used, c);
        grow(first_child, used, c); grow(nchild, used, c); grow(lo, used, c); grow(hi, used, c);
        cap = c;
    }
    Nodes view() {
        return Nodes{start.ptr, count.ptr, parent.ptr, level.ptr, first_child.ptr, nchild.ptr, size.ptr, pre.ptr,
                     lo.ptr, hi.ptr, et.ptr, pn.ptr, nn.ptr};
    }
};

}  // namespace

void build_octree_device(int n, const float *P, const float *N, const float *E, const float *A, const float bmin[3],
                         const float bmax[3], DeviceOctree &t) {
    if (n <= 0) throw Error(-1, "build_octree: no irradiance points");
    if (n >= (1 << 28)) throw Error(-1, "build_octree: more than 2^28 irradiance points");
    int pos_bits = 1;
    while ((1 << pos_bits) < n) ++pos_bits;
    const int key_bits = pos_bits + 3;

    DevBuf<int> orig[2], nid[2], head, idx;
    DevBuf<uint32_t> key[2];
    for (int b = 0; b < 2; ++b) {
        orig[b].alloc(n);
        nid[b].alloc(n);
        key[b].alloc(n);
    }
    head.alloc(n);
    idx.alloc(n);
    {  // orig = 0..n-1, every point in the root
        std::vector<int> iota(n);
        for (int i = 0; i < n; ++i) iota[i] = i;
        MPSS_HIP(hipMemcpy(orig[0].ptr, iota.data(), sizeof(int) * n, hipMemcpyHostToDevice));
        MPSS_HIP(hipMemset(nid[0].ptr, 0, sizeof(int) * n));
    }
    NodeStore ns;
    ns.reserve(0, (size_t)n / 2 + 64);
    {
        const int zero = 0, none = -1;
        const float4 lo = make_float4(bmin[0], bmin[1], bmin[2], 0.f), hi = make_float4(bmax[0], bmax[1], bmax[2], 0.f);
        MPSS_HIP(hipMemcpy(ns.start.ptr, &zero, sizeof(int), hipMemcpyHostToDevice));
        MPSS_HIP(hipMemcpy(ns.count.ptr, &n, sizeof(int), hipMemcpyHostToDevice));
        MPSS_HIP(hipMemcpy(ns.parent.ptr, &none, sizeof(int), hipMemcpyHostToDevice));
        MPSS_HIP(hipMemcpy(ns.level.ptr, &zero, sizeof(int), hipMemcpyHostToDevice));
        MPSS_HIP(hipMemcpy(ns.first_child.ptr, &none, sizeof(int), hipMemcpyHostToDevice));
        MPSS_HIP(hipMemcpy(ns.nchild.ptr, &zero, sizeof(int), hipMemcpyHostToDevice));
        MPSS_HIP(hipMemcpy(ns.lo.ptr, &lo, sizeof(float4), hipMemcpyHostToDevice));
        MPSS_HIP(hipMemcpy(ns.hi.ptr, &hi, sizeof(float4), hipMemcpyHostToDevice));
    }
    size_t sort_bytes = 0, scan_bytes = 0;
    MPSS_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, key[0].ptr, key[1].ptr, orig[0].ptr, orig[1].ptr,
                                                n, 0, key_bits));
    MPSS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, head.ptr, idx.ptr, n));
    DevBuf<unsigned char> tmp;
    tmp.alloc(std::max(sort_bytes, scan_bytes));

    std::vector<int> level_off = {0, 1};  // nodes of level d: [level_off[d], level_off[d + 1])
    int cur = 0;                          // ping-pong index of the live orig / nid arrays
    for (int lvl = 0;; ++lvl) {
        if (lvl > 96) throw Error(-2, "octree depth > 96: more than 8 coincident irradiance points");
        const int base = level_off.back();
        Nodes nd = ns.view();
        hipLaunchKernelGGL(level_keys_kernel, dim3(grid_of(n)), dim3(256), 0, 0, n, P, orig[cur].ptr, nid[cur].ptr, nd,
                           key[0].ptr);
        size_t sb = sort_bytes;
        MPSS_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.ptr, sb, key[0].ptr, key[1].ptr, orig[cur].ptr,
                                                    orig[1 - cur].ptr, n, 0, key_bits));
        hipLaunchKernelGGL(level_heads_kernel, dim3(grid_of(n)), dim3(256), 0, 0, n, nid[cur].ptr, nd, key[1].ptr,
                           head.ptr);
        size_t cb = scan_bytes;
        MPSS_HIP(hipcub::DeviceScan::ExclusiveSum(tmp.ptr, cb, head.ptr, idx.ptr, n));
        int last[2];
        MPSS_HIP(hipMemcpy(&last[0], idx.ptr + (n - 1), sizeof(int), hipMemcpyDeviceToHost));
        MPSS_HIP(hipMemcpy(&last[1], head.ptr + (n - 1), sizeof(int), hipMemcpyDeviceToHost));
        const int added = last[0] + last[1];
        if (added == 0) break;  // no node of this level splits: orig[cur] is final (nothing moved)
        ns.reserve((size_t)base, (size_t)base + added);
        nd = ns.view();
        hipLaunchKernelGGL(level_nodes_kernel, dim3(grid_of(n)), dim3(256), 0, 0, n, base, lvl + 1, nid[cur].ptr,
                           key[1].ptr, head.ptr, idx.ptr, nd);
        hipLaunchKernelGGL(level_assign_kernel, dim3(grid_of(n)), dim3(256), 0, 0, n, base, nid[cur].ptr, head.ptr,
                           idx.ptr, nd, nid[1 - cur].ptr);
        MPSS_HIP(hipGetLastError());
        cur = 1 - cur;
        level_off.push_back(base + added);
    }
    const int n_nodes = level_off.back(), depth_max = (int)level_off.size() - 2;
    ns.size.alloc(n_nodes);
    ns.pre.alloc(n_nodes);
    ns.pn.alloc(n_nodes);
    ns.nn.alloc(n_nodes);
    ns.et.alloc((size_t)n_nodes * NB);
    Nodes nd = ns.view();
    for (int d = depth_max; d >= 0; --d) {
        const int lo = level_off[d], hi = level_off[d + 1];
        hipLaunchKernelGGL(init_level_kernel, dim3(grid_of(hi - lo)), dim3(256), 0, 0, lo, hi, nd, orig[cur].ptr, P, N,
                           E, A);
    }
    MPSS_HIP(hipMemset(ns.pre.ptr, 0, sizeof(int)));
    for (int d = 0; d < depth_max; ++d) {
        const int lo = level_off[d], hi = level_off[d + 1];
        hipLaunchKernelGGL(preorder_level_kernel, dim3(grid_of(hi - lo)), dim3(256), 0, 0, lo, hi, nd);
    }
    t.layouts.clear();
    t.leaf_r2_error = -1.f;
    t.nodes.alloc(n_nodes);
    t.node_et.alloc((size_t)n_nodes * ROW);
    t.pt_hdr.alloc(n);
    t.pt_e.alloc((size_t)n * ROW);
    t.pt_index.alloc(n);
    hipLaunchKernelGGL(emit_kernel, dim3(grid_of(n_nodes)), dim3(256), 0, 0, n_nodes, nd, orig[cur].ptr, P, E, A,
                       t.nodes.ptr, t.node_et.ptr, t.pt_hdr.ptr, t.pt_e.ptr, t.pt_index.ptr);
    MPSS_HIP(hipGetLastError());
    MPSS_HIP(hipDeviceSynchronize());
    t.n_nodes = n_nodes;
    t.n_points = n;
    t.max_depth = depth_max;
    for (int k = 0; k < 3; ++k) {
        t.bmin[k] = bmin[k];
        t.bmax[k] = bmax[k];
    }
}

}  // namespace mpss
