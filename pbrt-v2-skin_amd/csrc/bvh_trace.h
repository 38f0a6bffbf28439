// bvh_trace.h -- per-lane BVH traversal shared by the render kernels (render.hip) and the
// reference-sampler replay generator (replay_gen.hip): the node-bounds test and Scene::IntersectP.
#pragma once
#include "geom.h"
#include "mo_band.h"
#include "render.h"

#include <climits>

namespace mpss {

constexpr int kTraceStack = 48;  // BVH traversal stack depth (host checks the tree depth)

__device__ __forceinline__ bool bbox_hit(const BvhNode &n, V3 o, V3 inv, const int neg[3], float mint, float maxt) {
    // bvh.cpp:126-148 (IntersectP of a node's bounds)
    const float *lo = n.bmin, *hi = n.bmax;
    float tmin = ((neg[0] ? hi[0] : lo[0]) - o.x) * inv.x;
    float tmax = ((neg[0] ? lo[0] : hi[0]) - o.x) * inv.x;
    const float tymin = ((neg[1] ? hi[1] : lo[1]) - o.y) * inv.y;
    const float tymax = ((neg[1] ? lo[1] : hi[1]) - o.y) * inv.y;
    if ((tmin > tymax) || (tymin > tmax)) return false;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    const float tzmin = ((neg[2] ? hi[2] : lo[2]) - o.z) * inv.z;
    const float tzmax = ((neg[2] ? lo[2] : hi[2]) - o.z) * inv.z;
    if ((tmin > tzmax) || (tzmin > tmax)) return false;
    if (tzmin > tmin) tmin = tzmin;
    if (tzmax < tmax) tmax = tzmax;
    return (tmin < maxt) && (tmax > mint);
}

// Scene::IntersectP (bvh.cpp:442-488 + Sphere::IntersectP)
__device__ inline bool trace_any(const RenderScene &sc, V3 o, V3 d, float mint, float maxt, int *stk, int sstride) {
    for (int l = 0; l < sc.nlights; ++l) {
        float t;
        if (!sc.lights[l].kind && sphere_intersect(sc.lights[l].s, o, d, mint, maxt, t, nullptr)) return true;
    }
    const V3 inv = V3{1.f / d.x, 1.f / d.y, 1.f / d.z};
    const int neg[3] = {inv.x < 0.f, inv.y < 0.f, inv.z < 0.f};
    int todo = 0, node = 0;
    for (;;) {
        const BvhNode n = sc.bvh[node];
        if (bbox_hit(n, o, inv, neg, mint, maxt)) {
            if (n.nprims > 0) {
                for (int i = 0; i < n.nprims; ++i) {
                    const TriRec tr = sc.tris[n.offset + i];
                    float t, b1, b2;
                    if (tri_intersect(o, d, mint, maxt, V3{tr.p1[0], tr.p1[1], tr.p1[2]},
                                      V3{tr.e1[0], tr.e1[1], tr.e1[2]}, V3{tr.e2[0], tr.e2[1], tr.e2[2]}, t, b1, b2))
                        return true;
                }
                if (todo == 0) break;
                node = stk[--todo * sstride];
            } else if (neg[n.axis]) {
                stk[todo++ * sstride] = node + 1;
                node = n.offset;
            } else {
                stk[todo++ * sstride] = n.offset;
                node = node + 1;
            }
        } else {
            if (todo == 0) break;
            node = stk[--todo * sstride];
        }
    }
    return false;
}

namespace {
// Sphere::Intersect out of line: its double-precision atan2 (the phi test) would otherwise set the
// register budget of every kernel that inlines a light loop.
__device__ __noinline__ bool sphere_hit_ool(const SphereView &s, V3 o, V3 d, float mint, float maxt, float &thit,
                                            V3 *nn) {
    return sphere_intersect(s, o, d, mint, maxt, thit, nn);
}

// Scene::IntersectP (bvh.cpp:442-488 + Sphere::IntersectP) for every active lane, as trace_any,
// by a stackless walk of the threaded BVH: pre-order, so after an interior node the walk goes on at
// node + 1 when some lane hit its box and at its subtree's end (the threaded offset) otherwise. A
// lane evaluates a node when node >= its resume index; missing a box sets resume to the subtree's
// end, a hit ends the lane. Each lane tests exactly the nodes and triangles its own traversal
// reaches with the fixed maxt (any-hit prunes only by the box test, so the order does not change
// the answer). strict: a triangle counts only when t < maxt (the BSDF ray toward an area light,
// whose own surface is at maxt). spheres: test the area-light spheres first, as trace_any does.
__device__ bool trace_any_wave(const RenderScene &sc, V3 o, V3 d, float mint, float maxt, bool active, bool strict,
                               bool spheres) {
    bool hit = false;
    if (active && spheres)
        for (int l = 0; l < sc.nlights; ++l) {
            float t;
            if (!sc.lights[l].kind && sphere_hit_ool(sc.lights[l].s, o, d, mint, maxt, t, nullptr)) {
                hit = true;
                break;
            }
        }
    const V3 inv = V3{1.f / d.x, 1.f / d.y, 1.f / d.z};
    const int neg[3] = {inv.x < 0.f, inv.y < 0.f, inv.z < 0.f};
    int resume = (active && !hit) ? 0 : INT_MAX;
    const cptr<BvhNode> nodes = as_const(sc.bvh_thread);
    const cptr<TriRec> tris = as_const(sc.tris);
    int node = 0;
    while (node < sc.nbvh) {
        node = __builtin_amdgcn_readfirstlane(node);
        const BvhNode n = nodes[node];
        const bool act = node >= resume;
        const bool in = act && bbox_hit(n, o, inv, neg, mint, maxt);
        if (act && !in) resume = n.nprims > 0 ? node + 1 : n.offset;
        if (n.nprims > 0) {
            if (__builtin_amdgcn_ballot_w64(in) != 0) {
                bool found = false;
                for (int i = 0; i < (int)n.nprims; ++i) {
                    const TriRec tr = tris[n.offset + i];
                    float t, b1, b2;
                    if (in && !found &&
                        tri_intersect(o, d, mint, maxt, V3{tr.p1[0], tr.p1[1], tr.p1[2]},
                                      V3{tr.e1[0], tr.e1[1], tr.e1[2]}, V3{tr.e2[0], tr.e2[1], tr.e2[2]}, t, b1, b2))
                        found = !strict || t < maxt;
                }
                if (found) {
                    hit = true;
                    resume = INT_MAX;
                }
                if (__builtin_amdgcn_ballot_w64(resume != INT_MAX) == 0) break;  // every lane is done
            }
            node = node + 1;
        } else {
            node = __builtin_amdgcn_ballot_w64(in) != 0 ? node + 1 : n.offset;
        }
    }
    return hit;
}
}  // namespace

}  // namespace mpss
