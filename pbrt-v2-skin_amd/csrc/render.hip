// render.hip -- the per-pixel path of MultipoleSubsurfaceIntegrator on CDNA4:
//   irradiance_kernel   IrradianceTask::Run         (integrators/multipolesubsurface.cpp:156-236 [file])
//   camera_direct_kernel SamplerRendererTask::Run -> Camera::GenerateRay -> Scene::Intersect ->
//                        MultipoleSubsurfaceIntegrator::Li up to UniformSampleAllLights
//                        (renderers/samplerrenderer.cpp:60-167, cameras/perspective.cpp,
//                         accelerators/bvh.cpp:388-488, core/integrator.cpp:45-174)
//                        and compacts the samples that need Mo() into a dense query list
//   (mo_band_kernel)     the Mo() gather, spectrally sharded across XCDs (mo_band.h, mo_kernel.hip)
//   film_kernel          Li assembly (multipolesubsurface.cpp:253-303: L = Le + SSS + Ld), the
//                        NaN/negative/inf sample filter (samplerrenderer.cpp:119-133), ToXYZ, and
//                        ImageFilm::AddSample with the 0.5-wide box filter (film/image.cpp:77-137)
// Sample values come from counter-based scrambled (0,2)-sequences (pbrt_math.h), identical
// in the CPU oracle ("replay mode").
#include "render.h"

#include <climits>

#include "../../data/spectral_bands.h"
#include "geom.h"

namespace mpss {

__constant__ float kCieX[NB] = MPSS_BAND_CIE_X_INIT;
__constant__ float kCieY[NB] = MPSS_BAND_CIE_Y_INIT;
__constant__ float kCieZ[NB] = MPSS_BAND_CIE_Z_INIT;

namespace {

constexpr int kStack = 48;  // BVH traversal stack depth (host checks the tree depth)

// ------------------------------------------------------------------ BVH traversal (per lane)
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

struct Hit {
    float t, b1, b2;
    int tri;    // global triangle id (>= 0) or -1 - light index, or INT_MIN for a miss
    V3 lnn;     // light-sphere dg.nn when a light is hit
};

// Scene::Intersect: BVH triangles + every sphere light (closest hit, bvh.cpp:388-439).
__device__ Hit trace_closest(const RenderScene &sc, V3 o, V3 d, float mint, float maxt, int *stk, int sstride) {
    Hit h;
    h.tri = INT_MIN;
    h.t = maxt;
    const V3 inv = V3{1.f / d.x, 1.f / d.y, 1.f / d.z};
    const int neg[3] = {inv.x < 0.f, inv.y < 0.f, inv.z < 0.f};
    int todo = 0, node = 0;
    for (;;) {
        const BvhNode n = sc.bvh[node];
        if (bbox_hit(n, o, inv, neg, mint, h.t)) {
            if (n.nprims > 0) {
                for (int i = 0; i < n.nprims; ++i) {
                    const TriRec tr = sc.tris[n.offset + i];
                    float t, b1, b2;
                    if (tri_intersect(o, d, mint, h.t, V3{tr.p1[0], tr.p1[1], tr.p1[2]},
                                      V3{tr.e1[0], tr.e1[1], tr.e1[2]}, V3{tr.e2[0], tr.e2[1], tr.e2[2]}, t, b1, b2)) {
                        h.t = t;
                        h.b1 = b1;
                        h.b2 = b2;
                        h.tri = tr.tri;
                    }
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
    for (int l = 0; l < sc.nlights; ++l) {
        float t;
        V3 nn;
        if (sphere_intersect(sc.lights[l].s, o, d, mint, h.t, t, &nn)) {
            h.t = t;
            h.tri = -1 - l;
            h.lnn = nn;
        }
    }
    return h;
}

// Scene::IntersectP (bvh.cpp:442-488 + Sphere::IntersectP)
__device__ bool trace_any(const RenderScene &sc, V3 o, V3 d, float mint, float maxt, int *stk, int sstride) {
    for (int l = 0; l < sc.nlights; ++l) {
        float t;
        if (sphere_intersect(sc.lights[l].s, o, d, mint, maxt, t, nullptr)) return true;
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

// DiffuseAreaLight::Sample_L (lights/diffuse.cpp:75-87) + VisibilityTester::SetSegment (light.h:87-92)
struct LightSampleOut {
    V3 wi;
    float pdf;
    bool nonblack;    // Ls = L(ps, ns, -wi) = Dot(ns, -wi) > 0 ? Lemit : 0
    V3 so, sd;        // shadow segment ray
    float smint, smaxt;
};
__device__ __forceinline__ LightSampleOut sample_light(const RenderLight &L, V3 p, float peps, float u0, float u1) {
    LightSampleOut r;
    V3 ns;
    const V3 ps = sphere_sample_from(L.s, p, u0, u1, ns);
    r.wi = normalize(ps - p);
    r.pdf = sphere_pdf(L.s, p, r.wi);
    const float dist = length(p - ps);  // Distance(p1, p2)
    r.so = p;
    r.sd = div(ps - p, dist);
    r.smint = peps;
    r.smaxt = dist * (1.f - 1e-3f);
    r.nonblack = dot(ns, -r.wi) > 0.f;
    return r;
}

__device__ __forceinline__ float rho_lookup(const float *hd, int n, float ct) {  // multipole.cpp:458-463
    const float fid = ct * (float)(n - 1);
    int id = (int)fid;
    id = id < 0 ? 0 : (id > n - 2 ? n - 2 : id);
    const float t = fid - (float)id;
    return (1.f - t) * hd[id] + t * hd[id + 1];
}

}  // namespace

// ------------------------------------------------------------------ irradiance (Preprocess)
__global__ __launch_bounds__(256) void irradiance_kernel(RenderScene sc, const float *__restrict__ sp_p,
                                                         const float *__restrict__ sp_n,
                                                         const float *__restrict__ sp_eps,
                                                         const uint32_t *__restrict__ sp_mat, int n, uint32_t seed,
                                                         float *__restrict__ E_out) {
    __shared__ int stk_all[kStack * 256];
    int *stk = stk_all + threadIdx.x;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const V3 p = V3{sp_p[3 * i], sp_p[3 * i + 1], sp_p[3 * i + 2]};
    const V3 nrm = V3{sp_n[3 * i], sp_n[3 * i + 1], sp_n[3 * i + 2]};
    const float eps = sp_eps[i];
    const uint32_t mid = sp_mat[i];
    const bool has_mat = mid < (uint32_t)sc.nmaterials;
    const RenderMaterial *mat = has_mat ? &sc.materials[mid] : nullptr;
    const bool bss = has_mat && mat->has_bssrdf;
    float E[NB];
    for (int c = 0; c < NB; ++c) E[c] = 0.f;
    for (int l = 0; l < sc.nlights; ++l) {
        const RenderLight &L = sc.lights[l];
        float El[NB];
        for (int c = 0; c < NB; ++c) El[c] = 0.f;
        const int ns = L.nsamples_pow2;
        const uint32_t scr0 = hash3(seed, (uint32_t)i, 16u * l + DIM_IRR_POS);
        const uint32_t scr1 = hash3(seed, (uint32_t)i, 16u * l + DIM_IRR_POS + 8u);
        for (int s = 0; s < ns; ++s) {
            const float u0 = van_der_corput((uint32_t)s, scr0), u1 = sobol2((uint32_t)s, scr1);  // Sample02
            const LightSampleOut ls = sample_light(L, p, eps, u0, u1);
            if (dot(ls.wi, nrm) <= 0.f) continue;
            if (!ls.nonblack || ls.pdf == 0.f) continue;
            if (!trace_any(sc, ls.so, ls.sd, ls.smint, ls.smaxt, stk, 256)) {
                float ct = absdot(ls.wi, nrm);
                ct = ct < 1.f ? ct : 1.f;
                const float Ft = bss ? 1.f - rho_lookup(mat->rho, mat->n_rho, ct) : 1.f;
                for (int c = 0; c < NB; ++c) El[c] += Ft * L.Lemit[c] * ct / ls.pdf;
            }
        }
        for (int c = 0; c < NB; ++c) E[c] += El[c] / (float)ns;
    }
    if (bss)
        for (int c = 0; c < NB; ++c) E[c] *= mat->alb_mix[c];
    for (int c = 0; c < NB; ++c) E_out[(size_t)i * NB + c] = E[c];
}

// ------------------------------------------------------------------ camera + direct lighting
__global__ __launch_bounds__(256) void camera_direct_kernel(RenderScene sc, TileBatch tb, SampleRecs rec) {
    __shared__ int stk_all[kStack * 256];
    int *stk = stk_all + threadIdx.x;
    const int64_t sid0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool in_range = sid0 < tb.nsamples;
    const int64_t sid = in_range ? sid0 : tb.nsamples - 1;
    const int s = (int)(sid % tb.spp);
    const int li = (int)(sid / tb.spp);
    const int px = tb.ex0 + li % tb.ew, py = tb.ey0 + li / tb.ew;
    const uint32_t pix = (uint32_t)py * (uint32_t)sc.xres + (uint32_t)px;
    // image sample (LDPixelSample's imageSamples, montecarlo.cpp:200-250): imageX = x + u in float
    const float X = (float)px + van_der_corput((uint32_t)s, hash3(tb.seed, pix, DIM_IMAGE));
    const float Y = (float)py + sobol2((uint32_t)s, hash3(tb.seed, pix, DIM_IMAGE + 1));
    // border samples matter only when the box filter carries them into the tile (film_kernel)
    int lx, hx, ly, hy;
    film_extent(X, sc.xres, lx, hx);
    film_extent(Y, sc.yres, ly, hy);
    const bool live = in_range && lx < tb.x1 && hx >= tb.x0 && ly < tb.y1 && hy >= tb.y0;
    uint32_t flags = 0;
    float4 pq = make_float4(0.f, 0.f, 0.f, 0.f);
    float ld[NB];
    for (int c = 0; c < NB; ++c) ld[c] = 0.f;
    if (live) {
        flags |= REC_LIVE;
        // PerspectiveCamera::GenerateRay (cameras/perspective.cpp)
        const V3 pras = V3{X, Y, 0.f};
        const V3 pcam = xform_point(sc.raster_to_camera, pras);
        const V3 dcam = normalize(pcam);
        const V3 o = xform_point(sc.camera_to_world, V3{0.f, 0.f, 0.f});
        const V3 d = xform_vector(sc.camera_to_world, dcam);
        const Hit h = trace_closest(sc, o, d, 0.f, INFINITY, stk, 256);
        if (h.tri != INT_MIN && h.tri < 0) {  // an area light's own surface: Le only
            const int l = -1 - h.tri;
            if (dot(h.lnn, -d) > 0.f) flags |= REC_LE | ((uint32_t)l << REC_LIGHT_SHIFT);
        } else if (h.tri != INT_MIN) {
            const int mi = sc.tri_mesh[h.tri], lt = sc.tri_local[h.tri];
            const RenderMesh &mesh = sc.meshes[mi];
            const V3 p = o + d * h.t;  // Ray::operator()
            const float reps = 1e-3f * h.t;
            const ShadingFrame fr = tri_shading(mesh.view, lt, p, 1.f - h.b1 - h.b2, h.b1, h.b2);
            const V3 wo = -d;
            const RenderMaterial &mat = sc.materials[mesh.material];
            if (mat.has_bssrdf && sc.have_octree) {
                float ct = absdot(wo, fr.nn);
                ct = ct < 1.f ? ct : 1.f;
                flags |= REC_SSS | (mesh.material << REC_MAT_SHIFT);
                pq = make_float4(fr.p.x, fr.p.y, fr.p.z, ct);
            }
            flags |= REC_SURF;
            // UniformSampleAllLights (integrator.cpp:45-77) with EstimateDirect (:117-174)
            const V3 wo_l = to_local(fr, wo);
            const float ng_wo = dot(wo, fr.ng);
            for (int l = 0; l < sc.nlights; ++l) {
                const RenderLight &L = sc.lights[l];
                const int ns = L.nsamples_round;
                float Ld[NB];
                for (int c = 0; c < NB; ++c) Ld[c] = 0.f;
                const uint32_t xr = (tb.spp & (tb.spp - 1)) == 0 ? (hash3(tb.seed, pix, 16u * l + 9u) & (tb.spp - 1)) : 0u;
                const uint32_t base = (uint32_t)(s ^ xr) * (uint32_t)ns;
                const uint32_t sl0 = hash3(tb.seed, pix, 16u * l + DIM_LIGHT_POS),
                               sl1 = hash3(tb.seed, pix, 16u * l + DIM_LIGHT_POS + 8u),
                               sb0 = hash3(tb.seed, pix, 16u * l + DIM_BSDF_DIR),
                               sb1 = hash3(tb.seed, pix, 16u * l + DIM_BSDF_DIR + 8u);
                for (int j = 0; j < ns; ++j) {
                    const uint32_t nidx = base + (uint32_t)j;
                    float ed[NB];
                    for (int c = 0; c < NB; ++c) ed[c] = 0.f;
                    // --- light sampling
                    const LightSampleOut ls = sample_light(L, fr.p, reps, van_der_corput(nidx, sl0), sobol2(nidx, sl1));
                    float lightPdf = ls.pdf;
                    if (lightPdf > 0.f && ls.nonblack && mat.has_refl) {
                        const V3 wi_l = to_local(fr, ls.wi);
                        const bool refl = dot(ls.wi, fr.ng) * ng_wo > 0.f;  // BSDF::f ng test
                        const MfTerms mt = microfacet_terms(mat.mf, wo_l, wi_l);
                        bool fblack = true;
                        float f[NB];
                        for (int c = 0; c < NB; ++c) {
                            f[c] = (refl && !mt.zero) ? mat.R[c] * mt.D * mt.G * mt.F / mt.den : 0.f;
                            fblack = fblack && f[c] == 0.f;
                        }
                        if (!fblack && !trace_any(sc, ls.so, ls.sd, ls.smint, ls.smaxt, stk, 256)) {
                            const float bsdfPdf = microfacet_pdf(mat.mf, wo_l, wi_l);
                            const float w = power_heuristic(lightPdf, bsdfPdf);
                            const float sc1 = absdot(ls.wi, fr.nn) * w / lightPdf;
                            for (int c = 0; c < NB; ++c) ed[c] += f[c] * L.Lemit[c] * sc1;
                        }
                    }
                    // --- BSDF sampling (BSDF::Sample_f, reflection.cpp:675-733)
                    if (mat.has_refl) {
                        V3 wi_l;
                        float bsdfPdf;
                        beckmann_sample(mat.mf, wo_l, van_der_corput(nidx, sb0), sobol2(nidx, sb1), wi_l, bsdfPdf);
                        if (bsdfPdf != 0.f) {
                            const V3 wi = to_world(fr, wi_l);
                            const bool refl = dot(wi, fr.ng) * ng_wo > 0.f;
                            const MfTerms mt = microfacet_terms(mat.mf, wo_l, wi_l);
                            bool fblack = true;
                            float f[NB];
                            for (int c = 0; c < NB; ++c) {
                                f[c] = (refl && !mt.zero) ? mat.R[c] * mt.D * mt.G * mt.F / mt.den : 0.f;
                                fblack = fblack && f[c] == 0.f;
                            }
                            if (!fblack && bsdfPdf > 0.f) {
                                lightPdf = sphere_pdf(L.s, fr.p, wi);
                                if (lightPdf != 0.f) {
                                    const float w = power_heuristic(bsdfPdf, lightPdf);
                                    const Hit hl = trace_closest(sc, fr.p, wi, reps, INFINITY, stk, 256);
                                    // Li = lightIsect.Le(-wi) when the hit primitive is this light
                                    if (hl.tri == -1 - l && dot(hl.lnn, -wi) > 0.f) {
                                        const float adn = absdot(wi, fr.nn);
                                        for (int c = 0; c < NB; ++c) ed[c] += f[c] * L.Lemit[c] * adn * w / bsdfPdf;
                                    }
                                }
                            }
                        }
                    }
                    for (int c = 0; c < NB; ++c) Ld[c] += ed[c];
                }
                for (int c = 0; c < NB; ++c) ld[c] += Ld[c] / (float)ns;
            }
        }
    }
    // compact the surface hits: one atomic per wave, sample order kept inside the wave
    const bool surf = (flags & REC_SURF) != 0;
    const uint64_t m = __builtin_amdgcn_ballot_w64(surf);
    const int lane = (int)(threadIdx.x & 63);
    int base = 0;
    if (lane == 0 && m) base = atomicAdd(rec.hit_count, (int)__builtin_popcountll(m));
    base = __shfl(base, 0);
    const int slot = base + (int)__builtin_popcountll(m & ((1ull << lane) - 1ull));
    if (!in_range) return;
    rec.flags[sid] = flags;
    rec.slot[sid] = surf ? slot : -1;
    if (surf) {
        rec.hit_q[slot] = (flags & REC_SSS) ? pq : make_float4(pq.x, pq.y, pq.z, -1.f);
        float4 *row = reinterpret_cast<float4 *>(rec.ld + (size_t)slot * ROW);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int c = 4 * k;
            row[k] = make_float4(ld[c], ld[c + 1], c + 2 < NB ? ld[c + 2] : 0.f, c + 3 < NB ? ld[c + 3] : 0.f);
        }
    }
}

// ------------------------------------------------------------------ film
// Li of one camera sample (MultipoleSubsurfaceIntegrator::Li, multipolesubsurface.cpp:253-303):
// L = 0 + Le; L += ((INV_PI * Ft) * Mo * Pow(albedo, 1 - mix)).Clamp(0); L += Ld -- then the
// SamplerRenderer sample filter (NaN / y < -1e-5 / inf -> 0) and Spectrum::ToXYZ, band order.
__device__ __forceinline__ void sample_xyz(const RenderScene &sc, const SampleRecs &rec, const BandPos &bp,
                                           int64_t sid, float &X, float &Y, float &Z) {
    const uint32_t flags = rec.flags[sid];
    X = Y = Z = 0.f;
    if (!(flags & (REC_SURF | REC_LE))) return;
    const float *le = (flags & REC_LE) ? sc.lights[(flags >> REC_LIGHT_SHIFT) & 0xff].Lemit : nullptr;
    const float *mo = nullptr;
    const RenderMaterial *mat = nullptr;
    float kss = 0.f;
    const int slot = (flags & REC_SURF) ? rec.slot[sid] : -1;
    if (flags & REC_SSS) {
        const float4 q = rec.hit_q[slot];
        mat = &sc.materials[(flags >> REC_MAT_SHIFT) & 0xff];
        const float Ft = mat->is_mc ? 1.f : 1.f - rho_lookup(mat->rho, mat->n_rho, q.w);
        kss = kInvPiF * Ft;
        mo = reinterpret_cast<const float *>(rec.mo4 + (size_t)slot * kGroups);
    }
    const float *ld = (flags & REC_SURF) ? rec.ld + (size_t)slot * ROW : nullptr;
    bool nan = false;
    for (int c = 0; c < NB; ++c) {
        float L = 0.f;
        if (le) L += le[c];
        if (mo) {
            float t = (kss * mo[bp.pos[c]]) * mat->alb_1mmix[c];
            t = t < 0.f ? 0.f : t;  // Spectrum::Clamp(0, INFINITY)
            L += t;
        }
        if (ld) L += ld[c];
        nan = nan || (L != L);
        X += kCieX[c] * L;
        Y += kCieY[c] * L;
        Z += kCieZ[c] * L;
    }
    const float scale = (float)(700 - 400) / (float)(MPSS_CIE_Y_INTEGRAL * NB);
    const float y = Y * (float)(700 - 400) / (float)(MPSS_CIE_Y_INTEGRAL * NB);
    X *= scale;
    Y *= scale;
    Z *= scale;
    if (nan || y < -1e-5f || __builtin_isinf(y)) X = Y = Z = 0.f;  // samplerrenderer.cpp:119-133
}

__global__ __launch_bounds__(256) void film_kernel(RenderScene sc, TileBatch tb, SampleRecs rec, BandPos bp,
                                                   float *__restrict__ out, int out_stride_px) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int tw = tb.x1 - tb.x0, th = tb.y1 - tb.y0;
    if (i >= tw * th) return;
    const int xres = sc.xres, yres = sc.yres;
    const int px = tb.x0 + i % tw, py = tb.y0 + i / tw;
    float X = 0.f, Y = 0.f, Z = 0.f, W = 0.f;
    // own samples (always inside this pixel's filter support), then the 8 neighbours' samples
    // in row-major order whose float image position rounds onto the shared edge
    // (ImageFilm::AddSample with the 0.5-wide box filter, image.cpp:77-137)
    for (int q = 0; q < 9; ++q) {
        const int dx = q == 0 ? 0 : ((q - 1 + (q > 4)) % 3) - 1;
        const int dy = q == 0 ? 0 : ((q - 1 + (q > 4)) / 3) - 1;
        const int qx = px + dx, qy = py + dy;
        if (qx < tb.ex0 || qy < tb.ey0 || qx >= tb.ex0 + tb.ew || qy >= tb.ey0 + tb.eh) continue;
        const int64_t li = (int64_t)(qy - tb.ey0) * tb.ew + (qx - tb.ex0);
        const uint32_t pix = (uint32_t)qy * (uint32_t)xres + (uint32_t)qx;
        const uint32_t su = hash3(tb.seed, pix, DIM_IMAGE), sv = hash3(tb.seed, pix, DIM_IMAGE + 1);
        for (int s = 0; s < tb.spp; ++s) {
            if (q > 0) {
                int lo, hi;
                if (dx != 0) {
                    film_extent((float)qx + van_der_corput((uint32_t)s, su), xres, lo, hi);
                    if (px < lo || px > hi) continue;
                }
                if (dy != 0) {
                    film_extent((float)qy + sobol2((uint32_t)s, sv), yres, lo, hi);
                    if (py < lo || py > hi) continue;
                }
            }
            float sx, sy, sz;
            sample_xyz(sc, rec, bp, li * tb.spp + s, sx, sy, sz);
            X += 1.f * sx;
            Y += 1.f * sy;
            Z += 1.f * sz;
            W += 1.f;
        }
    }
    float *o = out + ((size_t)(py - tb.y0) * out_stride_px + (px - tb.x0)) * 4;
    o[0] = X;
    o[1] = Y;
    o[2] = Z;
    o[3] = W;
}

}  // namespace mpss
