// geom.h -- host/device shape, BSDF and light routines of the multipole render path.
// Every routine cites the pbrt-v2-skin function it restates; float operation order follows
// the reference (see pbrt_math.h for the conventions).
#pragma once
#include "common.h"
#include "pbrt_math.h"

namespace mpss {

MPSS_HD float lerpf_t(float t, float a, float b) { return (1.f - t) * a + t * b; }  // pbrt.h:250

// Pixel range [lo, hi] one image-sample coordinate reaches through the 0.5-wide box filter
// (ImageFilm::AddSample, film/image.cpp:77-96: dImage = X - 0.5; [Ceil(d - .5), Floor(d + .5)],
// clamped to the film).
MPSS_HD void film_extent(float X, int res, int &lo, int &hi) {
    const float d = X - 0.5f;
    lo = (int)ceilf(d - 0.5f);
    hi = (int)floorf(d + 0.5f);
    lo = lo < 0 ? 0 : lo;
    hi = hi > res - 1 ? res - 1 : hi;
}

// Raw (device-friendly) view of one triangle mesh.
struct MeshView {
    const float *P, *N, *S, *uv;  // N, S, uv may be null
    const int32_t *idx;
    const float *o2w, *w2o;
    int flip;  // ReverseOrientation ^ TransformSwapsHandedness
    float o2w_store[16], w2o_store[16];  // device copies (o2w/w2o point here on the GPU)
};

MPSS_HD V3 ldv3(const float *a, int i) { return V3{a[3 * i], a[3 * i + 1], a[3 * i + 2]}; }

// TriangleBase::GetUVs, shapes/trianglemesh.h:109-122
MPSS_HD void tri_uvs(const MeshView &m, int t, float uv[3][2]) {
    if (m.uv) {
        for (int k = 0; k < 3; ++k) {
            uv[k][0] = m.uv[2 * m.idx[3 * t + k]];
            uv[k][1] = m.uv[2 * m.idx[3 * t + k] + 1];
        }
    } else {
        uv[0][0] = 0.f; uv[0][1] = 0.f;
        uv[1][0] = 1.f; uv[1][1] = 0.f;
        uv[2][0] = 1.f; uv[2][1] = 1.f;
    }
}

struct ShadingFrame {
    V3 p, ng, nn, sn, tn;  // geometric normal, shading normal, BSDF tangent frame (reflection.cpp:754-762)
    float u, v;
    V3 dpdu, dpdv;         // dgGeom's partial derivatives (ComputeDifferentials)
    V3 ss, ts, dndu, dndv; // dgShading's dpdu, dpdv, dndu, dndv (world space; Bump)
};

// Geometry + shading geometry at barycentrics (b0, b1, b2) with point p:
// TriangleBase::Intersect's dg part (trianglemesh.inl:85-130) / GetDifferentialGeometries
// (:303-346), then GetShadingGeometry (:224-300), then BSDF::BSDF (reflection.cpp:754-762).
MPSS_HD ShadingFrame tri_shading(const MeshView &m, int t, V3 p, float b0, float b1, float b2) {
    const V3 p1 = ldv3(m.P, m.idx[3 * t]), p2 = ldv3(m.P, m.idx[3 * t + 1]), p3 = ldv3(m.P, m.idx[3 * t + 2]);
    const V3 e1 = p2 - p1, e2 = p3 - p1;
    float uv[3][2];
    tri_uvs(m, t, uv);
    const float du1 = uv[0][0] - uv[2][0], du2 = uv[1][0] - uv[2][0];
    const float dv1 = uv[0][1] - uv[2][1], dv2 = uv[1][1] - uv[2][1];
    const V3 dp1 = p1 - p3, dp2 = p2 - p3;
    const float det = du1 * dv2 - dv1 * du2;
    V3 dpdu, dpdv;
    if (det == 0.f) {
        coordinate_system(normalize(cross(e2, e1)), dpdu, dpdv);
    } else {
        const float inv = 1.f / det;
        dpdu = (dp1 * dv2 - dp2 * dv1) * inv;
        dpdv = (dp1 * -du2 + dp2 * du1) * inv;
    }
    ShadingFrame f;
    f.p = p;
    f.u = b0 * uv[0][0] + b1 * uv[1][0] + b2 * uv[2][0];
    f.v = b0 * uv[0][1] + b1 * uv[1][1] + b2 * uv[2][1];
    V3 ng = normalize(cross(dpdu, dpdv));  // DifferentialGeometry ctor (core/diffgeom.cpp)
    if (m.flip) ng = ng * -1.f;
    f.ng = ng;
    V3 ss, ts;
    f.dpdu = dpdu;
    f.dpdv = dpdv;
    f.dndu = f.dndv = V3{0.f, 0.f, 0.f};
    if (!m.N && !m.S) {
        f.nn = ng;
        ss = dpdu;
        f.ss = dpdu;
        f.ts = dpdv;
    } else {
        float bb[3];
        const float A00 = uv[1][0] - uv[0][0], A01 = uv[2][0] - uv[0][0];
        const float A10 = uv[1][1] - uv[0][1], A11 = uv[2][1] - uv[0][1];
        const float C0 = f.u - uv[0][0], C1 = f.v - uv[0][1];
        const float d = A00 * A11 - A01 * A10;  // SolveLinearSystem2x2 (core/transform.cpp:39-49)
        bool ok = !(fabsf(d) < 1e-10f);
        if (ok) {
            bb[1] = (A11 * C0 - A01 * C1) / d;
            bb[2] = (A00 * C1 - A10 * C0) / d;
            if (bb[1] != bb[1] || bb[2] != bb[2]) ok = false;
        }
        if (!ok)
            bb[0] = bb[1] = bb[2] = 1.f / 3.f;
        else
            bb[0] = 1.f - bb[1] - bb[2];
        V3 ns;
        if (m.N) {
            const V3 n0 = ldv3(m.N, m.idx[3 * t]), n1 = ldv3(m.N, m.idx[3 * t + 1]), n2 = ldv3(m.N, m.idx[3 * t + 2]);
            ns = normalize(xform_normal(m.w2o, (n0 * bb[0] + n1 * bb[1]) + n2 * bb[2]));
        } else {
            ns = ng;
        }
        if (m.S) {
            const V3 s0 = ldv3(m.S, m.idx[3 * t]), s1 = ldv3(m.S, m.idx[3 * t + 1]), s2 = ldv3(m.S, m.idx[3 * t + 2]);
            ss = normalize(xform_vector(m.o2w, (s0 * bb[0] + s1 * bb[1]) + s2 * bb[2]));
        } else {
            ss = normalize(dpdu);
        }
        ts = cross(ss, ns);
        if (len2(ts) > 0.f) {
            ts = normalize(ts);
            ss = cross(ts, ns);
        } else {
            coordinate_system(ns, ss, ts);
        }
        V3 nn = normalize(cross(ss, ts));
        if (m.flip) nn = nn * -1.f;
        f.nn = nn;
        f.ss = ss;
        f.ts = ts;
        if (m.N && det != 0.f) {  // dndu, dndv from the vertex normals (trianglemesh.inl:269-295)
            const V3 n0 = ldv3(m.N, m.idx[3 * t]), n1 = ldv3(m.N, m.idx[3 * t + 1]), n2 = ldv3(m.N, m.idx[3 * t + 2]);
            const V3 dn1 = n0 - n2, dn2 = n1 - n2;
            const float invdet = 1.f / det;
            f.dndu = xform_normal(m.w2o, (dn1 * dv2 - dn2 * dv1) * invdet);
            f.dndv = xform_normal(m.w2o, (dn1 * -du2 + dn2 * du1) * invdet);
        }
    }
    f.sn = normalize(ss);        // BSDF: sn = Normalize(dgShading.dpdu)
    f.tn = cross(f.nn, f.sn);    //       tn = Cross(nn, sn)
    return f;
}

// Triangle ray test (trianglemesh.inl:47-84); returns t or -1, with barycentrics b1, b2.
MPSS_HD bool tri_intersect(V3 o, V3 d, float mint, float maxt, V3 p1, V3 e1, V3 e2, float &t_out, float &b1_out,
                           float &b2_out) {
    const V3 s1 = cross(d, e2);
    const float divisor = dot(s1, e1);
    if (divisor == 0.f) return false;
    const float inv = 1.f / divisor;
    const V3 dd = o - p1;
    const float b1 = dot(dd, s1) * inv;
    if (b1 < 0.f || b1 > 1.f) return false;
    const V3 s2 = cross(dd, e1);
    const float b2 = dot(d, s2) * inv;
    if (b2 < 0.f || b1 + b2 > 1.f) return false;
    const float t = dot(e2, s2) * inv;
    if (t < mint || t > maxt) return false;
    t_out = t;
    b1_out = b1;
    b2_out = b2;
    return true;
}

// ---------------------------------------------------------------- sphere (shapes/sphere.cpp)
struct SphereView {
    V3 c;
    float r, phi_max, area;  // full sphere: zmin=-r, zmax=r, thetaMin=pi, thetaMax=0
    float theta_min, theta_max;
};

// Quadratic, core/pbrt.h:354-368
MPSS_HD bool quadratic(float A, float B, float C, float &t0, float &t1) {
    const float disc = B * B - 4.f * A * C;
    if (disc < 0.f) return false;
    const float rd = sqrtf(disc);
    const float q = (B < 0.f) ? -.5f * (B - rd) : -.5f * (B + rd);
    t0 = q / A;
    t1 = C / q;
    if (t0 > t1) {
        const float x = t0;
        t0 = t1;
        t1 = x;
    }
    return true;
}

// Sphere::Intersect (sphere.cpp) for a full translated sphere; ray in world space, object
// space = world - centre. Outputs thit and (optionally) the world-space dg.nn.
MPSS_HD bool sphere_intersect(const SphereView &s, V3 o, V3 d, float mint, float maxt, float &thit, V3 *nn) {
    const V3 ro = o - s.c;  // WorldToObject: translation by -c
    const float A = d.x * d.x + d.y * d.y + d.z * d.z;
    const float B = 2 * (d.x * ro.x + d.y * ro.y + d.z * ro.z);
    const float C = ro.x * ro.x + ro.y * ro.y + ro.z * ro.z - s.r * s.r;
    float t0, t1;
    if (!quadratic(A, B, C, t0, t1)) return false;
    if (t0 > maxt || t1 < mint) return false;
    float th = t0;
    if (t0 < mint) {
        th = t1;
        if (th > maxt) return false;
    }
    V3 ph = ro + d * th;
    if (ph.x == 0.f && ph.y == 0.f) ph.x = 1e-5f * s.r;
    // The phi test can only reject below phiMax = Radians(360) = 2.f * kPiF exactly (the float
    // expression (kPiF / 180.f) * 360.f rounds to it), and phi never exceeds 2.f * kPiF: atan2 lies in
    // [-pi, pi], and a negative phi plus 2.f * kPiF rounds to at most 2.f * kPiF. A full sphere
    // therefore skips the (double-evaluated) atan2 with the same outcome.
    float phi = 0.f;
    if (s.phi_max < 2.f * kPiF) {
        phi = m_atan2(ph.y, ph.x);
        if (phi < 0.f) phi += 2.f * kPiF;
    }
    if (phi > s.phi_max) {  // zmin/zmax never clip a full sphere
        if (th == t1) return false;
        if (t1 > maxt) return false;
        th = t1;
        ph = ro + d * th;
        if (ph.x == 0.f && ph.y == 0.f) ph.x = 1e-5f * s.r;
        phi = m_atan2(ph.y, ph.x);
        if (phi < 0.f) phi += 2.f * kPiF;
        if (phi > s.phi_max) return false;
    }
    if (nn) {
        const float cz = ph.z / s.r;
        const float theta = m_acos(cz < -1.f ? -1.f : (cz > 1.f ? 1.f : cz));
        const float zr = sqrtf(ph.x * ph.x + ph.y * ph.y);
        const float izr = 1.f / zr;
        const float cphi = ph.x * izr, sphi = ph.y * izr;
        const V3 dpdu = V3{-s.phi_max * ph.y, s.phi_max * ph.x, 0.f};
        const V3 dpdv = V3{ph.z * cphi, ph.z * sphi, -s.r * m_sin(theta)} * (s.theta_max - s.theta_min);
        *nn = normalize(cross(dpdu, dpdv));  // o2w is a translation: vectors unchanged
    }
    thit = th;
    return true;
}

// UniformSampleCone with frame (montecarlo.cpp:413-420)
MPSS_HD V3 uniform_sample_cone(float u1, float u2, float ctmax, V3 x, V3 y, V3 z) {
    const float ct = lerpf_t(u1, ctmax, 1.f);
    const float st = sqrtf(1.f - ct * ct);
    const float phi = u2 * 2.f * kPiF;
    return (x * (m_cos(phi) * st) + y * (m_sin(phi) * st)) + z * ct;
}

// UniformSampleSphere (montecarlo.cpp:283-291)
MPSS_HD V3 uniform_sample_sphere(float u1, float u2) {
    const float z = 1.f - 2.f * u1;
    const float r = sqrtf(fmaxf(0.f, 1.f - z * z));
    const float phi = 2.f * kPiF * u2;
    return V3{r * m_cos(phi), r * m_sin(phi), z};
}

// Sphere::Sample(p, u1, u2, &ns) (sphere.cpp) followed by ShapeSet::Sample's re-intersection
// (core/light.cpp:145-158) for a one-shape set. Returns the sampled point and its normal.
MPSS_HD V3 sphere_sample_from(const SphereView &s, V3 p, float u1, float u2, V3 &ns) {
    const V3 pc = s.c;
    const V3 wc = normalize(pc - p);
    V3 wcx, wcy;
    coordinate_system(wc, wcx, wcy);
    V3 ps;
    if (dist2(p, pc) - s.r * s.r < 1e-4f) {  // Sphere::Sample(u1, u2, ns)
        const V3 q = uniform_sample_sphere(u1, u2) * s.r;
        ns = normalize(q);  // o2w(Normal): translation leaves normals unchanged
        ps = q + pc;
    } else {
        const float st2 = s.r * s.r / dist2(p, pc);
        const float ctmax = sqrtf(fmaxf(0.f, 1.f - st2));
        const V3 rd = uniform_sample_cone(u1, u2, ctmax, wcx, wcy, wc);
        float th;
        if (!sphere_intersect(s, p, rd, 1e-3f, INFINITY, th, nullptr)) th = dot(pc - p, normalize(rd));
        ps = p + rd * th;
        ns = normalize(ps - pc);
    }
    // ShapeSet::Sample: re-intersect r(p, pt - p) with every shape, thit starts at 1
    const V3 rd2 = ps - p;
    float th2 = 1.f;
    V3 nn2;
    if (sphere_intersect(s, p, rd2, 1e-3f, INFINITY, th2, &nn2)) ns = nn2;
    return p + rd2 * th2;
}

// Sphere::Pdf(p, wi) (sphere.cpp) inside ShapeSet::Pdf (core/light.cpp:167-172)
MPSS_HD float sphere_pdf(const SphereView &s, V3 p, V3 wi) {
    float pdf;
    if (dist2(p, s.c) - s.r * s.r < 1e-4f) {  // Shape::Pdf (core/shape.cpp:96-109)
        float th;
        V3 nn;
        if (!sphere_intersect(s, p, wi, 1e-3f, INFINITY, th, &nn))
            pdf = 0.f;
        else {
            pdf = dist2(p, p + wi * th) / (absdot(nn, -wi) * s.area);
            if (__builtin_isinf(pdf)) pdf = 0.f;
        }
    } else {
        const float st2 = s.r * s.r / dist2(p, s.c);
        const float ctmax = sqrtf(fmaxf(0.f, 1.f - st2));
        pdf = 1.f / (2.f * kPiF * (1.f - ctmax));  // UniformConePdf
    }
    return (0.f + s.area * pdf) / s.area;
}

// ---------------------------------------------------------------- microfacet BSDF
// Microfacet(R, FresnelDielectric(1, eta) [or Fixed], Beckmann(rough)) as LayeredSkin::GetBSDF
// builds it (materials/layeredskin.cpp:139-167); reflection.{h,cpp}.
struct Microfacet {
    float rms2, rcp_rms2, eta;
    int fixed_fresnel;
};

MPSS_HD float beckmann_D(const Microfacet &m, V3 wh) {  // reflection.h:514-521
    const float ct = fabsf(wh.z), c2 = ct * ct, d = c2 * c2 * kPiF;
    if (d == 0.f) return 0.f;
    const float e = (c2 - 1) * m.rcp_rms2 / c2;
    return m.rcp_rms2 * m_exp(e) / d;
}

MPSS_HD float fresnel_dielectric(float cosi, float eta_i, float eta_t, int fixed) {  // reflection.cpp:132-153
    cosi = cosi < -1.f ? -1.f : (cosi > 1.f ? 1.f : cosi);
    float ei = eta_i, et = eta_t;
    if (!(cosi > 0.f)) {
        ei = eta_t;
        et = eta_i;
    }
    const float x = 1.f - cosi * cosi;
    const float sint = ei / et * sqrtf(x > 0.f ? x : 0.f);
    float F;
    if (sint >= 1.f)
        F = 1.f;
    else {
        const float y = 1.f - sint * sint;
        const float cost = sqrtf(y > 0.f ? y : 0.f);
        const float ci = fabsf(cosi);
        const float par = ((et * ci) - (ei * cost)) / ((et * ci) + (ei * cost));
        const float per = ((ei * ci) - (et * cost)) / ((ei * ci) + (et * cost));
        F = (par * par + per * per) / 2.f;
    }
    if (fixed) F = F + F * (1.f - F) * (1.f - F);  // FixedFresnelDielectric, reflection.h:315-324
    return F;
}

MPSS_HD float microfacet_G(V3 wo, V3 wi, V3 wh) {  // reflection.h:430-437
    const float a = fabsf(wh.z), wowh = absdot(wo, wh);
    const float g1 = 2.f * a * fabsf(wo.z) / wowh, g2 = 2.f * a * fabsf(wi.z) / wowh;
    const float m = g2 < g1 ? g2 : g1;  // std::min(g1, g2): (b < a) ? b : a
    return m < 1.f ? m : 1.f;            // std::min(1.f, m)
}

// Microfacet::f with R factored out: returns (D, G, F, denominator) so that per band
// f[c] = R[c] * D * G * F / den exactly as reflection.cpp:228-240 evaluates it.
struct MfTerms {
    float D, G, F, den;
    bool zero;
};
MPSS_HD MfTerms microfacet_terms(const Microfacet &m, V3 wo, V3 wi) {
    MfTerms r{0.f, 0.f, 0.f, 1.f, true};
    const float co = fabsf(wo.z), ci = fabsf(wi.z);
    if (ci == 0.f || co == 0.f) return r;
    V3 wh = wi + wo;
    if (wh.x == 0.f && wh.y == 0.f && wh.z == 0.f) return r;
    wh = normalize(wh);
    r.F = fresnel_dielectric(dot(wi, wh), 1.f, m.eta, m.fixed_fresnel);
    r.D = beckmann_D(m, wh);
    r.G = microfacet_G(wo, wi, wh);
    r.den = 4.f * ci * co;
    r.zero = false;
    return r;
}

// Beckmann::Pdf (reflection.cpp:572-580) wrapped by Microfacet::Pdf (:399-403)
MPSS_HD float microfacet_pdf(const Microfacet &m, V3 wo, V3 wi) {
    if (!(wo.z * wi.z > 0.f)) return 0.f;
    const V3 wh = normalize(wo + wi);
    const float ct = fabsf(wh.z);
    float p = beckmann_D(m, wh) * ct / (4.f * dot(wo, wh));
    if (dot(wo, wh) <= 0.f || p < 1e-20f) p = 0.f;
    return p;
}

// Beckmann::Sample_f (reflection.cpp:548-570): wi and pdf
MPSS_HD void beckmann_sample(const Microfacet &m, V3 wo, float u1, float u2, V3 &wi, float &pdf) {
    const float theta = m_atan(sqrtf(-m.rms2 * m_log(1.f - u1)));
    const float ct = m_cos(theta), st = m_sin(theta);
    const float phi = u2 * 2.f * kPiF;
    V3 wh = V3{st * m_cos(phi), st * m_sin(phi), ct};  // SphericalDirection
    if (!(wo.z * wh.z > 0.f)) wh = -wh;
    const float dw = dot(wo, wh);
    wi = -wo + wh * (2.f * dw);
    float p = beckmann_D(m, wh) * ct / (4.f * dot(wo, wh));
    if (dot(wo, wh) <= 0.f || p < 1e-20f) p = 0.f;
    pdf = p;
}

// ---------------------------------------------------------------- MicrofacetTransmission
// reflection.cpp:242-281, 405-459 with the Beckmann distribution and the layer's (Fixed)
// FresnelDielectric(1, ior). Its f is T * s * (1 - F) with a scalar s (factored like MfTerms).
struct MtTerms {
    float s, F;
    bool zero;
};

MPSS_HD float beckmann_pdf(const Microfacet &m, V3 wo, V3 wi) {  // Beckmann::Pdf (no hemisphere test)
    const V3 wh = normalize(wo + wi);
    const float ct = fabsf(wh.z);
    float p = beckmann_D(m, wh) * ct / (4.f * dot(wo, wh));
    if (dot(wo, wh) <= 0.f || p < 1e-20f) p = 0.f;
    return p;
}

MPSS_HD float mt_G(V3 wo, V3 wi, V3 wh) {  // MicrofacetTransmission::G (reflection.cpp:273-281)
    const float nwh = fabsf(wh.z), nwo = fabsf(wo.z), nwi = fabsf(wi.z);
    const float owh = absdot(wo, wh), iwh = absdot(wi, wh);
    const float a = 2.f * nwh * nwo / owh, b = 2.f * nwh * nwi / iwh;
    const float m = b < a ? b : a;  // std::min semantics, as microfacet_G
    return m < 1.f ? m : 1.f;
}

MPSS_HD MtTerms mt_terms(const Microfacet &m, V3 wo, V3 wi) {  // MicrofacetTransmission::f (:251-270)
    MtTerms r{0.f, 0.f, true};
    const float ci = fabsf(wi.z), co = fabsf(wo.z);
    if (ci == 0.f || co == 0.f) return r;
    const bool entering = wo.z > 0.f;
    const float et = entering ? m.eta : 1.f / m.eta;
    V3 wh = -(wo + wi * et);
    const float den = len2(wh);
    if (den == 0.f) return r;
    wh = normalize(wh);
    const float chi = dot(wi, wh), cho = dot(wo, wh);
    if (chi == 0.f || cho == 0.f) return r;
    r.F = fresnel_dielectric(entering ? fabsf(cho) : -fabsf(cho), 1.f, m.eta, m.fixed_fresnel);
    r.s = fabsf(chi * cho) * et * et * beckmann_D(m, wh) * mt_G(wo, wi, wh) / (ci * co * den);
    r.zero = false;
    return r;
}

MPSS_HD float mt_pdf(const Microfacet &m, V3 wo, V3 wi) {  // MicrofacetTransmission::Pdf (:444-459)
    if (wo.z * wi.z > 0.f) return 0.f;  // SameHemisphere
    const bool entering = wo.z > 0.f;
    const float et = entering ? m.eta : 1.f / m.eta;
    V3 wh = -(wo + wi * et);
    if (wh.x == 0.f && wh.y == 0.f && wh.z == 0.f) return 0.f;
    const float den = len2(wh);
    wh = normalize(wh);
    const V3 wir = -wo + wh * (2.f * dot(wo, wh));
    float pdf = beckmann_pdf(m, wo, wir);
    const float cosi = dot(wo, wh);
    pdf *= 4 * cosi * cosi * et * et / den;
    return pdf;
}

// MicrofacetTransmission::Sample_f (:405-441): wi and pdf (pdf stays the distribution's when the
// half vector degenerates or wi lands in wo's hemisphere, as in the reference)
MPSS_HD void mt_sample(const Microfacet &m, V3 wo, float u1, float u2, V3 &wi, float &pdf) {
    beckmann_sample(m, wo, u1, u2, wi, pdf);
    const bool entering = wo.z > 0.f;
    const float et = entering ? m.eta : 1.f / m.eta;
    V3 wh = wo + wi;
    if (wh.x == 0.f && wh.y == 0.f && wh.z == 0.f) return;
    wh = normalize(wh);
    const float cosi = dot(wo, wh);
    const float x = 1.f - cosi * cosi;
    const float sini2 = x > 0.f ? x : 0.f;
    const float eta = 1.f / et;
    const float sint2 = eta * eta * sini2;
    if (sint2 >= 1.f) {
        pdf = 0.f;
        return;
    }
    const float y = 1.f - sint2;
    const float cost = sqrtf(y > 0.f ? y : 0.f);
    const float so = eta;
    wi = wo * -so + wh * (so * cosi - cost);
    const float den = len2(wo + wi * et);
    if (den == 0.f) {
        pdf = 0.f;
        return;
    }
    pdf *= 4 * cosi * cosi * et * et / den;
}

MPSS_HD V3 to_local(const ShadingFrame &f, V3 v) { return V3{dot(v, f.sn), dot(v, f.tn), dot(v, f.nn)}; }
MPSS_HD V3 to_world(const ShadingFrame &f, V3 v) {
    return V3{f.sn.x * v.x + f.tn.x * v.y + f.nn.x * v.z, f.sn.y * v.x + f.tn.y * v.y + f.nn.y * v.z,
              f.sn.z * v.x + f.tn.z * v.y + f.nn.z * v.z};
}

MPSS_HD float power_heuristic(float fpdf, float gpdf) {  // montecarlo.h:270-273 (nf = ng = 1)
    const float f = 1 * fpdf, g = 1 * gpdf;
    return (f * f) / (f * f + g * g);
}

// ---------------------------------------------------------------- the light sphere's own surface
// An area light's sphere carries pbrt's default material, "matte" (api.cpp:241,1085): Kd =
// Spectrum(0.5f), sigma 0 -> one Lambertian BRDF (matte.cpp:49-71). f = R * INV_PI.
constexpr float kMatteF = 0.5f * 0.31830988618379067154f;

// ConcentricSampleDisk (montecarlo.cpp:306-348); `theta *= M_PI / 4.f` is a double product
MPSS_HD void concentric_disk(float u1, float u2, float &dx, float &dy) {
    float r, theta;
    const float sx = 2 * u1 - 1, sy = 2 * u2 - 1;
    if (sx == 0.f && sy == 0.f) {
        dx = dy = 0.f;
        return;
    }
    if (sx >= -sy) {
        if (sx > sy) {
            r = sx;
            theta = sy > 0.f ? sy / r : 8.0f + sy / r;
        } else {
            r = sy;
            theta = 2.0f - sx / r;
        }
    } else if (sx <= sy) {
        r = -sx;
        theta = 4.0f - sy / r;
    } else {
        r = -sy;
        theta = 6.0f + sx / r;
    }
    theta = (float)((double)theta * (3.14159265358979323846 / 4.0));
    dx = r * m_cos(theta);
    dy = r * m_sin(theta);
}

// BxDF::Pdf / Sample_f defaults for the Lambertian (reflection.cpp): SameHemisphere ? |cos wi| / pi : 0;
// wi = CosineSampleHemisphere(u1, u2) (montecarlo.h:128-133), z turned to wo's side
MPSS_HD float lambert_pdf(V3 wo, V3 wi) { return wo.z * wi.z > 0.f ? fabsf(wi.z) * 0.31830988618379067154f : 0.f; }
MPSS_HD void lambert_sample(V3 wo, float u1, float u2, V3 &wi, float &pdf) {
    float x, y;
    concentric_disk(u1, u2, x, y);
    wi = V3{x, y, sqrtf(fmaxf(0.f, 1.f - x * x - y * y))};
    if (wo.z < 0.f) wi.z *= -1.f;
    pdf = lambert_pdf(wo, wi);
}

// Sphere::Intersect's DifferentialGeometry at a camera ray's thit (sphere.cpp:114-152; object space =
// world - centre) and the BSDF frame on it (reflection.cpp:754-762): nn = Normalize(Cross(dpdu, dpdv))
// = ng (no shading normals), sn = Normalize(dpdu), tn = Cross(nn, sn).
MPSS_HD ShadingFrame sphere_frame(const SphereView &s, V3 o, V3 d, float t) {
    ShadingFrame fr{};
    V3 ph = (o - s.c) + d * t;
    if (ph.x == 0.f && ph.y == 0.f) ph.x = 1e-5f * s.r;
    const float cz = ph.z / s.r;
    const float theta = m_acos(cz < -1.f ? -1.f : (cz > 1.f ? 1.f : cz));
    const float zr = sqrtf(ph.x * ph.x + ph.y * ph.y);
    const float izr = 1.f / zr;
    const float cphi = ph.x * izr, sphi = ph.y * izr;
    const V3 dpdu = V3{-s.phi_max * ph.y, s.phi_max * ph.x, 0.f};
    const V3 dpdv = V3{ph.z * cphi, ph.z * sphi, -s.r * m_sin(theta)} * (s.theta_max - s.theta_min);
    fr.p = ph + s.c;
    fr.nn = normalize(cross(dpdu, dpdv));
    fr.ng = fr.nn;
    fr.sn = normalize(dpdu);
    fr.tn = cross(fr.nn, fr.sn);
    return fr;
}

}  // namespace mpss
