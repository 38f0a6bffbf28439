// scene.cpp -- BVH build (binned SAH, 4 prims per leaf like pbrt's default maxnodeprims,
// accelerators/bvh.cpp:547-550) and TessellateSurfacePoints (see scene.h).
#include "scene.h"

#include "geom.h"
#include "texture.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>

namespace mpss {

// ------------------------------------------------------------------------------- BVH
namespace {

struct PrimInfo {
    float lo[3], hi[3], c[3];
    int tri;
};

struct BuildCtx {
    std::vector<PrimInfo> prims;
    std::vector<BvhNode> nodes;
    std::vector<int> order;
};

void bounds_of(const std::vector<PrimInfo> &p, int b, int e, float *lo, float *hi, bool centroid) {
    for (int k = 0; k < 3; ++k) {
        lo[k] = INFINITY;
        hi[k] = -INFINITY;
    }
    for (int i = b; i < e; ++i)
        for (int k = 0; k < 3; ++k) {
            const float a = centroid ? p[i].c[k] : p[i].lo[k], z = centroid ? p[i].c[k] : p[i].hi[k];
            lo[k] = std::min(lo[k], a);
            hi[k] = std::max(hi[k], z);
        }
}

float area_of(const float *lo, const float *hi) {
    const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    if (dx < 0 || dy < 0 || dz < 0) return 0.f;
    return 2.f * (dx * dy + dy * dz + dz * dx);
}

int build_rec(BuildCtx &c, int b, int e) {
    const int me = (int)c.nodes.size();
    c.nodes.emplace_back();
    float lo[3], hi[3];
    bounds_of(c.prims, b, e, lo, hi, false);
    const int n = e - b;
    auto make_leaf = [&] {
        BvhNode &nd = c.nodes[me];
        memcpy(nd.bmin, lo, sizeof(lo));
        memcpy(nd.bmax, hi, sizeof(hi));
        nd.offset = (int32_t)c.order.size();
        nd.nprims = (uint16_t)n;
        nd.axis = 0;
        for (int i = b; i < e; ++i) c.order.push_back(c.prims[i].tri);
        return me;
    };
    if (n <= 4) return make_leaf();
    float clo[3], chi[3];
    bounds_of(c.prims, b, e, clo, chi, true);
    int axis = 0;
    for (int k = 1; k < 3; ++k)
        if (chi[k] - clo[k] > chi[axis] - clo[axis]) axis = k;
    if (chi[axis] <= clo[axis]) return make_leaf();
    // 16-bin SAH
    constexpr int NBIN = 16;
    int cnt[NBIN] = {};
    float blo[NBIN][3], bhi[NBIN][3];
    for (int i = 0; i < NBIN; ++i)
        for (int k = 0; k < 3; ++k) {
            blo[i][k] = INFINITY;
            bhi[i][k] = -INFINITY;
        }
    const float scale = NBIN / (chi[axis] - clo[axis]);
    auto bin_of = [&](const PrimInfo &p) {
        return std::min(NBIN - 1, std::max(0, (int)((p.c[axis] - clo[axis]) * scale)));
    };
    for (int i = b; i < e; ++i) {
        const int bi = bin_of(c.prims[i]);
        cnt[bi]++;
        for (int k = 0; k < 3; ++k) {
            blo[bi][k] = std::min(blo[bi][k], c.prims[i].lo[k]);
            bhi[bi][k] = std::max(bhi[bi][k], c.prims[i].hi[k]);
        }
    }
    float best = INFINITY;
    int best_split = -1;
    for (int s = 1; s < NBIN; ++s) {
        float llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        float rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        int nl = 0, nr = 0;
        for (int i = 0; i < NBIN; ++i) {
            float *L = i < s ? llo : rlo, *H = i < s ? lhi : rhi;
            (i < s ? nl : nr) += cnt[i];
            for (int k = 0; k < 3; ++k) {
                L[k] = std::min(L[k], blo[i][k]);
                H[k] = std::max(H[k], bhi[i][k]);
            }
        }
        if (!nl || !nr) continue;
        const float cost = nl * area_of(llo, lhi) + nr * area_of(rlo, rhi);
        if (cost < best) {
            best = cost;
            best_split = s;
        }
    }
    int mid;
    if (best_split < 0) {
        mid = (b + e) / 2;
        std::nth_element(c.prims.begin() + b, c.prims.begin() + mid, c.prims.begin() + e,
                         [&](const PrimInfo &x, const PrimInfo &y) { return x.c[axis] < y.c[axis]; });
    } else {
        mid = (int)(std::partition(c.prims.begin() + b, c.prims.begin() + e,
                                   [&](const PrimInfo &p) { return bin_of(p) < best_split; }) -
                    c.prims.begin());
        if (mid == b || mid == e) mid = (b + e) / 2;
    }
    build_rec(c, b, mid);
    const int second = build_rec(c, mid, e);
    BvhNode &nd = c.nodes[me];
    memcpy(nd.bmin, lo, sizeof(lo));
    memcpy(nd.bmax, hi, sizeof(hi));
    nd.offset = second;
    nd.nprims = 0;
    nd.axis = (uint16_t)axis;
    return me;
}

}  // namespace

void build_bvh(SceneData &s) {
    BuildCtx c;
    s.tri_mesh.clear();
    s.tri_local.clear();
    for (size_t m = 0; m < s.meshes.size(); ++m) {
        const Mesh &mesh = s.meshes[m];
        const int nt = (int)mesh.idx.size() / 3;
        for (int t = 0; t < nt; ++t) {
            PrimInfo p;
            for (int k = 0; k < 3; ++k) {
                p.lo[k] = INFINITY;
                p.hi[k] = -INFINITY;
            }
            for (int v = 0; v < 3; ++v) {
                const float *q = &mesh.P[3 * (size_t)mesh.idx[3 * t + v]];
                for (int k = 0; k < 3; ++k) {
                    p.lo[k] = std::min(p.lo[k], q[k]);
                    p.hi[k] = std::max(p.hi[k], q[k]);
                }
            }
            for (int k = 0; k < 3; ++k) p.c[k] = .5f * p.lo[k] + .5f * p.hi[k];
            p.tri = (int)s.tri_mesh.size();
            s.tri_mesh.push_back((int32_t)m);
            s.tri_local.push_back(t);
            c.prims.push_back(p);
        }
    }
    if (c.prims.empty()) throw Error(-1, "scene has no triangles");
    c.nodes.reserve(2 * c.prims.size());
    build_rec(c, 0, (int)c.prims.size());
    s.bvh = std::move(c.nodes);
    s.tris.resize(c.order.size());
    for (size_t i = 0; i < c.order.size(); ++i) {
        const int g = c.order[i];
        const Mesh &mesh = s.meshes[s.tri_mesh[g]];
        const int t = s.tri_local[g];
        const float *p1 = &mesh.P[3 * (size_t)mesh.idx[3 * t]];
        const float *p2 = &mesh.P[3 * (size_t)mesh.idx[3 * t + 1]];
        const float *p3 = &mesh.P[3 * (size_t)mesh.idx[3 * t + 2]];
        TriRec &r = s.tris[i];
        for (int k = 0; k < 3; ++k) {
            r.p1[k] = p1[k];
            r.e1[k] = p2[k] - p1[k];
            r.e2[k] = p3[k] - p1[k];
        }
        r.tri = g;
        r.mesh = s.tri_mesh[g];
        r.pad = 0;
    }
}

// ------------------------------------------------------------------------------- tessellation
namespace {

struct BC {
    float b0, b1, b2;
};
const BC kCentroid = {1.f / 3.f, 1.f / 3.f, 1.f / 3.f};  // trianglemesh.cpp:185

inline BC bc_lerp(float t, BC a, BC b) {  // BarycentricCoordinate::Lerp
    return BC{lerpf_t(t, a.b0, b.b0), lerpf_t(t, a.b1, b.b1), lerpf_t(t, a.b2, b.b2)};
}
inline BC bc_eval(BC s, BC a, BC b, BC c) {  // BarycentricCoordinate::Evaluate(BC, BC, BC)
    return BC{s.b0 * a.b0 + s.b1 * b.b0 + s.b2 * c.b0, s.b0 * a.b1 + s.b1 * b.b1 + s.b2 * c.b1,
              s.b0 * a.b2 + s.b1 * b.b2 + s.b2 * c.b2};
}
inline V3 bc_point(BC s, V3 a, V3 b, V3 c) {  // BarycentricCoordinate::Evaluate(Point x3)
    return (a * s.b0 + b * s.b1) + c * s.b2;
}

template <class Shader>
void matching(BC b0I, BC b1I, int segsI, BC b0O, BC b1O, int segsO, Shader &shader) {  // :321-351
    int ip = 0, op = 0;
    while (ip < segsI || op < segsO) {
        const BC bIn = segsI ? bc_lerp((float)ip / segsI, b0I, b1I) : b0I;
        const BC bOut = bc_lerp((float)op / segsO, b0O, b1O);
        const float sIn = (ip < segsI) ? fabsf((float)(ip + 1) + 1.f - (float)op / segsO * (segsI + 2)) : INFINITY;
        const float sOut = (op < segsO) ? fabsf((float)ip + 1.f - (float)(op + 1) / segsO * (segsI + 2)) : INFINITY;
        if (sIn < sOut) {
            shader(bc_lerp((float)(ip + 1) / segsI, b0I, b1I), bIn, bOut);
            ip++;
        } else {
            shader(bIn, bOut, bc_lerp((float)(op + 1) / segsO, b0O, b1O));
            op++;
        }
    }
}

template <class Shader>
void tessellator(float tfe0, float tfe1, float tfe2, float tfc, Shader &shader) {  // :265-318
    const int e0 = std::max((int)ceilf(tfe0), 1), e1 = std::max((int)ceilf(tfe1), 1),
              e2 = std::max((int)ceilf(tfe2), 1);
    int ic = std::max((int)ceilf(tfc), 1);
    if (e0 > 1 || e1 > 1 || e2 > 1) ic = std::max(ic, 2);
    const BC b0{1.f, 0.f, 0.f}, b1{0.f, 1.f, 0.f}, b2{0.f, 0.f, 1.f}, bc = kCentroid;
    const int rings = (ic + 1) / 2;
    for (int r = 0; r < rings - 1; ++r) {
        const int edgeInner = ic - (rings - r) * 2;
        const BC o0 = bc_lerp((float)(r + 1) / rings, bc, b0), o1 = bc_lerp((float)(r + 1) / rings, bc, b1),
                 o2 = bc_lerp((float)(r + 1) / rings, bc, b2);
        if (edgeInner >= 0) {
            const int edgeOuter = edgeInner + 2;
            const BC i0 = bc_lerp((float)r / rings, bc, b0), i1 = bc_lerp((float)r / rings, bc, b1),
                     i2 = bc_lerp((float)r / rings, bc, b2);
            matching(i0, i1, edgeInner, o0, o1, edgeOuter, shader);
            matching(i1, i2, edgeInner, o1, o2, edgeOuter, shader);
            matching(i2, i0, edgeInner, o2, o0, edgeOuter, shader);
        } else {
            shader(o0, o1, o2);
        }
    }
    const int edgeInner = ic - 2;
    if (edgeInner >= 0) {
        const float t = (float)(rings - 1) / rings;
        const BC i0 = bc_lerp(t, bc, b0), i1 = bc_lerp(t, bc, b1), i2 = bc_lerp(t, bc, b2);
        matching(i0, i1, edgeInner, b0, b1, e2, shader);
        matching(i1, i2, edgeInner, b1, b2, e0, shader);
        matching(i2, i0, edgeInner, b2, b0, e1, shader);
    } else {
        shader(b0, b1, b2);
    }
}

inline V3 ld3(const std::vector<float> &a, int i) { return V3{a[3 * (size_t)i], a[3 * (size_t)i + 1], a[3 * (size_t)i + 2]}; }

}  // namespace

MeshView mesh_view(const Mesh &m) {
    return MeshView{m.P.data(), m.N.empty() ? nullptr : m.N.data(), m.S.empty() ? nullptr : m.S.data(),
                    m.uv.empty() ? nullptr : m.uv.data(), m.idx.data(), m.o2w, m.w2o,
                    (int)(m.reverse_orientation ^ m.swaps_handedness)};
}

void tessellate_surface_points(const SceneData &s, float min_dist, bool incenter, std::vector<SurfacePoint> &out,
                               int nthreads, const TexView *const *bump) {
    out.clear();
    struct Job {
        int mesh, t0, t1;
        std::vector<SurfacePoint> pts;
    };
    std::vector<Job> jobs;
    for (size_t m = 0; m < s.meshes.size(); ++m) {
        const int nt = (int)s.meshes[m].idx.size() / 3;
        for (int t0 = 0; t0 < nt; t0 += 512) jobs.push_back(Job{(int)m, t0, std::min(nt, t0 + 512), {}});
    }
    if (nthreads <= 0) nthreads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::atomic<int> next{0};
    auto work = [&] {
        for (int j; (j = next.fetch_add(1)) < (int)jobs.size();) {
            Job &job = jobs[j];
            const Mesh &m = s.meshes[job.mesh];
            const MeshView mv = mesh_view(m);
            for (int t = job.t0; t < job.t1; ++t) {
                const V3 v0 = ld3(m.P, m.idx[3 * t]), v1 = ld3(m.P, m.idx[3 * t + 1]), v2 = ld3(m.P, m.idx[3 * t + 2]);
                const float le0 = length(v1 - v2), le1 = length(v2 - v0), le2 = length(v0 - v1);
                float tfe0 = le0 / min_dist * 0.8f, tfe1 = le1 / min_dist * 0.8f, tfe2 = le2 / min_dist * 0.8f;
                const float tfc = floorf((tfe0 + tfe1 + tfe2) / 3.f + .5f);
                tfe0 = floorf(tfe0 + .5f);
                tfe1 = floorf(tfe1 + .5f);
                tfe2 = floorf(tfe2 + .5f);
                auto shader = [&](BC a, BC b, BC c) {
                    const V3 s0 = bc_point(a, v0, v1, v2), s1 = bc_point(b, v0, v1, v2), s2 = bc_point(c, v0, v1, v2);
                    BC bc;
                    if (!incenter) {
                        bc = bc_eval(kCentroid, a, b, c);
                    } else {
                        const float l0 = length(s1 - s2), l1 = length(s2 - s0), l2 = length(s0 - s1);
                        const BC bic{l0 / (l0 + l1 + l2), l1 / (l0 + l1 + l2), l2 / (l0 + l1 + l2)};
                        bc = bc_eval(bic, a, b, c);
                    }
                    SurfacePoint sp;
                    const V3 p = bc_point(bc, v0, v1, v2);
                    sp.p[0] = p.x; sp.p[1] = p.y; sp.p[2] = p.z;
                    // GetDifferentialGeometries(bc) -> dgGeom, dgShading (no differentials); Bump with
                    // no map copies dgShading (material.cpp:107-114)
                    const ShadingFrame fr = tri_shading(mv, t, p, bc.b0, bc.b1, bc.b2);
                    sp.u = fr.u;
                    sp.v = fr.v;
                    V3 n = fr.nn;
                    const TexView *bt = bump ? bump[m.material] : nullptr;
                    if (bt) {
                        const UVDiff g{fr.u, fr.v, 0.f, 0.f, 0.f, 0.f};
                        V3 dpdu_b;
                        bump_frame(*bt, g, fr.ss, fr.ts, fr.dndu, fr.dndv, fr.nn, fr.ng, mv.flip, dpdu_b, n);
                    }
                    sp.n[0] = n.x; sp.n[1] = n.y; sp.n[2] = n.z;
                    sp.material = m.material;
                    sp.area = .5f * length(cross(s1 - s0, s2 - s0));
                    sp.ray_eps = min_dist / 10.f;
                    job.pts.push_back(sp);
                };
                tessellator(tfe0, tfe1, tfe2, tfc, shader);
            }
        }
    };
    std::vector<std::thread> th;
    for (int i = 0; i < nthreads; ++i) th.emplace_back(work);
    for (auto &x : th) x.join();
    size_t total = 0;
    for (auto &j : jobs) total += j.pts.size();
    out.reserve(total);
    for (auto &j : jobs) out.insert(out.end(), j.pts.begin(), j.pts.end());
}

}  // namespace mpss
