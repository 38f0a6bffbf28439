// octree.cpp -- host octree build and flattening (see octree.h).
#include "octree.h"

#include <cmath>
#include <cstring>

#include "spectral.h"

namespace mpss {

namespace {

struct BuildNode {
    bool leaf = true;
    int32_t slot[8];  // point index (leaf) or child node index (interior); -1 = empty
    float p[3] = {0, 0, 0}, n[3] = {0, 0, 0}, et[NB] = {}, sum_area = 0.f;
    BuildNode() {
        for (int i = 0; i < 8; ++i) slot[i] = -1;
    }
};

struct Builder {
    const float *P, *N, *E, *A;
    std::vector<BuildNode> nodes;

    static void child_bounds(int c, const float *lo, const float *hi, const float *mid, float *clo, float *chi) {
        // octreeChildBound, core/octree.h:87-97
        for (int k = 0; k < 3; ++k) {
            const bool upper = (c >> (2 - k)) & 1;
            clo[k] = upper ? mid[k] : lo[k];
            chi[k] = upper ? hi[k] : mid[k];
        }
    }
    static int octant(const float *pt, const float *mid) {
        return (pt[0] > mid[0] ? 4 : 0) + (pt[1] > mid[1] ? 2 : 0) + (pt[2] > mid[2] ? 1 : 0);
    }

    void place(int node, const float *lo, const float *hi, const float *mid, int ip, int depth) {
        const int c = octant(P + 3 * (size_t)ip, mid);
        if (nodes[node].slot[c] < 0) {
            nodes[node].slot[c] = (int32_t)nodes.size();
            nodes.emplace_back();
        }
        float clo[3], chi[3];
        child_bounds(c, lo, hi, mid, clo, chi);
        insert(nodes[node].slot[c], clo, chi, ip, depth + 1);
    }

    // SubsurfaceOctreeNode::Insert, diffusionutil.h:94-132
    void insert(int node, const float *lo, const float *hi, int ip, int depth) {
        if (depth > 96) throw Error(-2, "octree depth > 96: more than 8 coincident irradiance points");
        float mid[3];
        for (int k = 0; k < 3; ++k) mid[k] = .5f * lo[k] + .5f * hi[k];
        if (nodes[node].leaf) {
            for (int i = 0; i < 8; ++i)
                if (nodes[node].slot[i] < 0) {
                    nodes[node].slot[i] = ip;
                    return;
                }
            nodes[node].leaf = false;
            int32_t local[8];
            memcpy(local, nodes[node].slot, sizeof(local));
            for (int i = 0; i < 8; ++i) nodes[node].slot[i] = -1;
            for (int i = 0; i < 8; ++i) place(node, lo, hi, mid, local[i], depth);
        }
        place(node, lo, hi, mid, ip, depth);
    }

    // SubsurfaceOctreeNode::InitHierarchy, diffusionutil.h:133-173
    void init(int node) {
        float sum_wt = 0.f;
        BuildNode &nd = nodes[node];
        for (int i = 0; i < 8; ++i) {
            const int s = nodes[node].slot[i];
            if (s < 0) {
                if (nodes[node].leaf) break;
                continue;
            }
            float et[NB], pp[3], nn[3], area;
            if (nodes[node].leaf) {
                area = A[s];
                for (int c = 0; c < NB; ++c) et[c] = E[(size_t)s * NB + c] * area;
                for (int k = 0; k < 3; ++k) {
                    pp[k] = P[3 * (size_t)s + k];
                    nn[k] = N[3 * (size_t)s + k];
                }
            } else {
                init(s);
                const BuildNode &ch = nodes[s];
                memcpy(et, ch.et, sizeof(et));
                memcpy(pp, ch.p, sizeof(pp));
                memcpy(nn, ch.n, sizeof(nn));
                area = ch.sum_area;
            }
            BuildNode &me = nodes[node];  // (vector may not grow during init, reference stays valid)
            const float wt = spectrum_y(et);
            for (int c = 0; c < NB; ++c) me.et[c] += et[c];
            for (int k = 0; k < 3; ++k) {
                me.p[k] += pp[k] * wt;
                me.n[k] += nn[k] * wt;
            }
            sum_wt += wt;
            me.sum_area += area;
        }
        (void)nd;
        if (sum_wt > 0.f) {
            const float inv = 1.f / sum_wt;
            for (int k = 0; k < 3; ++k) {
                nodes[node].p[k] *= inv;
                nodes[node].n[k] *= inv;
            }
        }
    }
};

bool black(const float *s) {
    for (int c = 0; c < NB; ++c)
        if (s[c] != 0.f) return false;
    return true;
}

struct Flattener {
    const Builder &b;
    FlatOctree &out;
    void emit(int node, const float *lo, const float *hi, int depth) {
        const BuildNode &nd = b.nodes[node];
        const int me = (int)out.hdr.size();
        out.hdr.emplace_back();
        out.node_et.resize(out.node_et.size() + ROW, 0.f);
        NodeHdr h{};
        h.px = nd.p[0]; h.py = nd.p[1]; h.pz = nd.p[2];
        h.sum_area = nd.sum_area;
        h.bminx = lo[0]; h.bminy = lo[1]; h.bminz = lo[2];
        h.bmaxx = hi[0]; h.bmaxy = hi[1]; h.bmaxz = hi[2];
        h.depth = depth;
        h.flags = black(nd.et) ? NODE_BLACK : 0u;
        memcpy(&out.node_et[(size_t)me * ROW], nd.et, sizeof(float) * NB);
        if (depth > out.max_depth) out.max_depth = depth;
        if (nd.leaf) {
            h.leaf_first = (int32_t)out.pt_index.size();
            int cnt = 0;
            for (int i = 0; i < 8 && nd.slot[i] >= 0; ++i, ++cnt) {
                const int ip = nd.slot[i];
                out.pt_index.push_back(ip);
                const float *e = b.E + (size_t)ip * NB;
                const float a = b.A[ip];
                out.pt_hdr.insert(out.pt_hdr.end(),
                                  {b.P[3 * (size_t)ip], b.P[3 * (size_t)ip + 1], b.P[3 * (size_t)ip + 2],
                                   black(e) ? copysignf(a, -1.f) : a});
                const size_t o = out.pt_e.size();
                out.pt_e.resize(o + ROW, 0.f);
                memcpy(&out.pt_e[o], e, sizeof(float) * NB);
            }
            h.leaf_count = cnt;
        } else {
            h.leaf_first = -1;
            h.leaf_count = 0;
            float mid[3];
            for (int k = 0; k < 3; ++k) mid[k] = .5f * lo[k] + .5f * hi[k];
            for (int c = 0; c < 8; ++c) {
                if (nd.slot[c] < 0) continue;
                float clo[3], chi[3];
                Builder::child_bounds(c, lo, hi, mid, clo, chi);
                emit(nd.slot[c], clo, chi, depth + 1);
            }
        }
        h.skip = (int32_t)out.hdr.size();
        out.hdr[me] = h;
    }
};

}  // namespace

void build_octree(int npts, const float *p, const float *n, const float *E, const float *area, FlatOctree &out) {
    out = FlatOctree();
    if (npts <= 0) throw Error(-1, "build_octree: no irradiance points");
    Builder b{p, n, E, area, {}};
    b.nodes.reserve((size_t)npts / 2 + 16);
    for (int k = 0; k < 3; ++k) {
        out.bmin[k] = INFINITY;
        out.bmax[k] = -INFINITY;
    }
    for (int i = 0; i < npts; ++i)  // Union(BBox, Point), core/geometry.cpp:38-47
        for (int k = 0; k < 3; ++k) {
            const float v = p[3 * (size_t)i + k];
            out.bmin[k] = (v < out.bmin[k]) ? v : out.bmin[k];
            out.bmax[k] = (out.bmax[k] < v) ? v : out.bmax[k];
        }
    b.nodes.emplace_back();
    for (int i = 0; i < npts; ++i) b.insert(0, out.bmin, out.bmax, i, 0);
    b.init(0);
    out.hdr.reserve(b.nodes.size());
    out.node_et.reserve(b.nodes.size() * ROW);
    out.pt_hdr.reserve((size_t)npts * 4);
    out.pt_e.reserve((size_t)npts * ROW);
    out.pt_index.reserve(npts);
    Flattener f{b, out};
    f.emit(0, out.bmin, out.bmax, 0);
}

}  // namespace mpss
