// tessellate.h -- TriangleMesh::TessellateSurfacePoints for one triangle (reference
// src/shapes/trianglemesh.cpp:187-257; tessellator :265-318, matching :321-351), host and device.
//
// The same source runs in the host build (scene.cpp, threaded over triangles) and in the GPU
// build (render.hip tess_kernel, one thread per triangle): the same IEEE float operations in the
// same order (-ffp-contract=off on both sides), so the two give the same points bit for bit.
#pragma once
#include "geom.h"
#include "scene.h"
#include "texture.h"

namespace mpss {

struct BC {  // BarycentricCoordinate
    float b0, b1, b2;
};

MPSS_HD BC bc_lerp(float t, BC a, BC b) {  // BarycentricCoordinate::Lerp
    return BC{lerpf_t(t, a.b0, b.b0), lerpf_t(t, a.b1, b.b1), lerpf_t(t, a.b2, b.b2)};
}
MPSS_HD BC bc_eval(BC s, BC a, BC b, BC c) {  // BarycentricCoordinate::Evaluate(BC, BC, BC)
    return BC{s.b0 * a.b0 + s.b1 * b.b0 + s.b2 * c.b0, s.b0 * a.b1 + s.b1 * b.b1 + s.b2 * c.b1,
              s.b0 * a.b2 + s.b1 * b.b2 + s.b2 * c.b2};
}
MPSS_HD V3 bc_point(BC s, V3 a, V3 b, V3 c) {  // BarycentricCoordinate::Evaluate(Point x3)
    return (a * s.b0 + b * s.b1) + c * s.b2;
}
MPSS_HD BC bc_centroid() { return BC{1.f / 3.f, 1.f / 3.f, 1.f / 3.f}; }  // trianglemesh.cpp:185

template <class Shader>
MPSS_HD void tess_matching(BC b0I, BC b1I, int segsI, BC b0O, BC b1O, int segsO, Shader &shader) {  // :321-351
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
MPSS_HD void tessellator(float tfe0, float tfe1, float tfe2, float tfc, Shader &shader) {  // :265-318
    const int c0 = (int)ceilf(tfe0), c1 = (int)ceilf(tfe1), c2 = (int)ceilf(tfe2), cc = (int)ceilf(tfc);
    const int e0 = c0 > 1 ? c0 : 1, e1 = c1 > 1 ? c1 : 1, e2 = c2 > 1 ? c2 : 1;
    int ic = cc > 1 ? cc : 1;
    if ((e0 > 1 || e1 > 1 || e2 > 1) && ic < 2) ic = 2;
    const BC b0{1.f, 0.f, 0.f}, b1{0.f, 1.f, 0.f}, b2{0.f, 0.f, 1.f}, bc = bc_centroid();
    const int rings = (ic + 1) / 2;
    for (int r = 0; r < rings - 1; ++r) {
        const int edgeInner = ic - (rings - r) * 2;
        const BC o0 = bc_lerp((float)(r + 1) / rings, bc, b0), o1 = bc_lerp((float)(r + 1) / rings, bc, b1),
                 o2 = bc_lerp((float)(r + 1) / rings, bc, b2);
        if (edgeInner >= 0) {
            const int edgeOuter = edgeInner + 2;
            const BC i0 = bc_lerp((float)r / rings, bc, b0), i1 = bc_lerp((float)r / rings, bc, b1),
                     i2 = bc_lerp((float)r / rings, bc, b2);
            tess_matching(i0, i1, edgeInner, o0, o1, edgeOuter, shader);
            tess_matching(i1, i2, edgeInner, o1, o2, edgeOuter, shader);
            tess_matching(i2, i0, edgeInner, o2, o0, edgeOuter, shader);
        } else {
            shader(o0, o1, o2);
        }
    }
    const int edgeInner = ic - 2;
    if (edgeInner >= 0) {
        const float t = (float)(rings - 1) / rings;
        const BC i0 = bc_lerp(t, bc, b0), i1 = bc_lerp(t, bc, b1), i2 = bc_lerp(t, bc, b2);
        tess_matching(i0, i1, edgeInner, b0, b1, e2, shader);
        tess_matching(i1, i2, edgeInner, b1, b2, e0, shader);
        tess_matching(i2, i0, edgeInner, b2, b0, e1, shader);
    } else {
        shader(b0, b1, b2);
    }
}

// The triangle's corners (world space) and tessellation factors: per edge round(len / minDist *
// 0.8), centre the rounded mean of the unrounded edge factors (trianglemesh.cpp:195-205).
struct TessTri {
    V3 v0, v1, v2;
    float tfe0, tfe1, tfe2, tfc;
};
MPSS_HD TessTri tess_tri(const MeshView &m, int t, float min_dist) {
    TessTri r;
    r.v0 = ldv3(m.P, m.idx[3 * t]);
    r.v1 = ldv3(m.P, m.idx[3 * t + 1]);
    r.v2 = ldv3(m.P, m.idx[3 * t + 2]);
    const float le0 = length(r.v1 - r.v2), le1 = length(r.v2 - r.v0), le2 = length(r.v0 - r.v1);
    const float f0 = le0 / min_dist * 0.8f, f1 = le1 / min_dist * 0.8f, f2 = le2 / min_dist * 0.8f;
    r.tfc = floorf((f0 + f1 + f2) / 3.f + .5f);
    r.tfe0 = floorf(f0 + .5f);
    r.tfe1 = floorf(f1 + .5f);
    r.tfe2 = floorf(f2 + .5f);
    return r;
}

// One sub-triangle's SurfacePoint (the reference's SurfacePointShader, trianglemesh.cpp:210-256):
// the barycentre (or incentre) mapped through the sub-triangle, the shading geometry there
// (GetDifferentialGeometries, no differentials), the bump-mapped normal when the material has a
// bump map (Bump with no map copies dgShading, material.cpp:107-114), area = |cross| / 2.
MPSS_HD SurfacePoint tess_point(const MeshView &mv, int t, const TessTri &tr, BC a, BC b, BC c, bool incenter,
                                const TexView *bump, uint32_t material, float min_dist) {
    const V3 s0 = bc_point(a, tr.v0, tr.v1, tr.v2), s1 = bc_point(b, tr.v0, tr.v1, tr.v2),
             s2 = bc_point(c, tr.v0, tr.v1, tr.v2);
    BC bc;
    if (!incenter) {
        bc = bc_eval(bc_centroid(), a, b, c);
    } else {
        const float l0 = length(s1 - s2), l1 = length(s2 - s0), l2 = length(s0 - s1);
        const BC bic{l0 / (l0 + l1 + l2), l1 / (l0 + l1 + l2), l2 / (l0 + l1 + l2)};
        bc = bc_eval(bic, a, b, c);
    }
    SurfacePoint sp;
    const V3 p = bc_point(bc, tr.v0, tr.v1, tr.v2);
    sp.p[0] = p.x;
    sp.p[1] = p.y;
    sp.p[2] = p.z;
    const ShadingFrame fr = tri_shading(mv, t, p, bc.b0, bc.b1, bc.b2);
    sp.u = fr.u;
    sp.v = fr.v;
    V3 n = fr.nn;
    if (bump) {
        const UVDiff g{fr.u, fr.v, 0.f, 0.f, 0.f, 0.f};
        V3 dpdu_b;
        bump_frame(*bump, g, fr.ss, fr.ts, fr.dndu, fr.dndv, fr.nn, fr.ng, mv.flip, dpdu_b, n);
    }
    sp.n[0] = n.x;
    sp.n[1] = n.y;
    sp.n[2] = n.z;
    sp.material = material;
    sp.area = .5f * length(cross(s1 - s0, s2 - s0));
    sp.ray_eps = min_dist / 10.f;
    return sp;
}

}  // namespace mpss
