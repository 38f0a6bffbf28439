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
#include "bvh_trace.h"
#include "geom.h"
#include "tessellate.h"

namespace mpss {

__constant__ float kCieX[NB] = MPSS_BAND_CIE_X_INIT;
__constant__ float kCieY[NB] = MPSS_BAND_CIE_Y_INIT;
__constant__ float kCieZ[NB] = MPSS_BAND_CIE_Z_INIT;
// rgbIllum2Spect{White, Cyan, Magenta, Yellow, Red, Green, Blue} (spectrum.cpp:316-370)
__constant__ float kIllum[7][NB] = {MPSS_BAND_RGBILLUM2SPECTWHITE_INIT,  MPSS_BAND_RGBILLUM2SPECTCYAN_INIT,
                                    MPSS_BAND_RGBILLUM2SPECTMAGENTA_INIT, MPSS_BAND_RGBILLUM2SPECTYELLOW_INIT,
                                    MPSS_BAND_RGBILLUM2SPECTRED_INIT,     MPSS_BAND_RGBILLUM2SPECTGREEN_INIT,
                                    MPSS_BAND_RGBILLUM2SPECTBLUE_INIT};

// rgbRefl2Spect{White, Cyan, Magenta, Yellow, Red, Green, Blue} (spectrum.cpp:316-370)
__constant__ float kRefl[7][NB] = {MPSS_BAND_RGBREFL2SPECTWHITE_INIT,  MPSS_BAND_RGBREFL2SPECTCYAN_INIT,
                                   MPSS_BAND_RGBREFL2SPECTMAGENTA_INIT, MPSS_BAND_RGBREFL2SPECTYELLOW_INIT,
                                   MPSS_BAND_RGBREFL2SPECTRED_INIT,     MPSS_BAND_RGBREFL2SPECTGREEN_INIT,
                                   MPSS_BAND_RGBREFL2SPECTBLUE_INIT};

namespace {

constexpr int kStack = kTraceStack;

// ------------------------------------------------------------------ BVH traversal (per lane)
// (bbox_hit, trace_any: bvh_trace.h)
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
        if (sc.lights[l].kind) continue;  // an infinite light has no shape
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

// (sphere_hit_ool: bvh_trace.h)

// ------------------------------------------------------------------ BVH traversal (per wave)
// The hot kernels trace with the whole wave walking one node sequence: the node index is
// wave-uniform, so node and triangle records are scalar loads, and no lane carries a stack.

// (trace_any_wave: bvh_trace.h)

// Scene::Intersect's BVH part (bvh.cpp:388-439) for the active lanes whose rays share the direction
// signs (dirIsNeg) of `pat`: with the signs shared, every lane's ordered traversal (near child first)
// visits its nodes in one common order, so the wave walks the union with one stack of (node, lane
// mask) entries in LDS; a lane enters a node only if it is in the entry's mask and hits the box with
// its own current t. Each lane therefore tests exactly the nodes and triangles, in exactly the
// order, of its own traversal, and ends with the same hit.
__device__ void trace_closest_packet(const RenderScene &sc, V3 o, V3 inv, const int neg[3], V3 d, float mint, Hit &h,
                                     uint64_t grp, int pat, int *snode, uint64_t *smask) {
    const int lane = (int)(threadIdx.x & 63);
    const bool mine = (grp >> lane) & 1ull;
    const cptr<BvhNode> nodes = as_const(sc.bvh);
    const cptr<TriRec> tris = as_const(sc.tris);
    int node = 0, sp = 0;
    uint64_t mask = grp;
    for (;;) {
        node = __builtin_amdgcn_readfirstlane(node);
        const BvhNode n = nodes[node];
        const bool in = mine && ((mask >> lane) & 1ull) && bbox_hit(n, o, inv, neg, mint, h.t);
        const uint64_t m = __builtin_amdgcn_ballot_w64(in);
        if (m != 0 && n.nprims == 0) {  // interior: near child now, far child on the stack
            const int a = (int)n.axis;
            const bool far_first = ((pat >> a) & 1) != 0;  // dirIsNeg[axis]: the second child is near
            snode[sp] = far_first ? node + 1 : n.offset;
            smask[sp] = m;
            ++sp;
            node = far_first ? n.offset : node + 1;
            mask = m;
            continue;
        }
        if (m != 0) {  // leaf
            for (int i = 0; i < (int)n.nprims; ++i) {
                const TriRec tr = tris[n.offset + i];
                float t, b1, b2;
                if (in && tri_intersect(o, d, mint, h.t, V3{tr.p1[0], tr.p1[1], tr.p1[2]},
                                        V3{tr.e1[0], tr.e1[1], tr.e1[2]}, V3{tr.e2[0], tr.e2[1], tr.e2[2]}, t, b1, b2)) {
                    h.t = t;
                    h.b1 = b1;
                    h.b2 = b2;
                    h.tri = tr.tri;
                }
            }
        }
        if (sp == 0) break;
        --sp;
        node = snode[sp];
        mask = __builtin_amdgcn_readfirstlane((uint32_t)smask[sp]) |
               ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(smask[sp] >> 32)) << 32);
    }
}

// trace_closest for every active lane, by sign packets: the lanes are grouped by their rays'
// direction signs and each group is traced as one packet (camera rays of one pixel share them).
// snode / smask: this wave's kStack-entry stack in LDS.
__device__ Hit trace_closest_wave(const RenderScene &sc, V3 o, V3 d, float mint, float maxt, bool active, int *snode,
                                  uint64_t *smask) {
    Hit h;
    h.tri = INT_MIN;
    h.t = maxt;
    const V3 inv = V3{1.f / d.x, 1.f / d.y, 1.f / d.z};
    const int neg[3] = {inv.x < 0.f, inv.y < 0.f, inv.z < 0.f};
    const int sgn = neg[0] | (neg[1] << 1) | (neg[2] << 2);
    uint64_t todo = __builtin_amdgcn_ballot_w64(active);
    while (todo != 0) {
        const int lead = __builtin_ctzll(todo);
        const int pat = __builtin_amdgcn_readlane(sgn, lead);
        const uint64_t grp = __builtin_amdgcn_ballot_w64(active && sgn == pat) & todo;
        todo &= ~grp;
        trace_closest_packet(sc, o, inv, neg, d, mint, h, grp, pat, snode, smask);
    }
    if (active)
        for (int l = 0; l < sc.nlights; ++l) {
            if (sc.lights[l].kind) continue;  // an infinite light has no shape
            float t;
            V3 nn;
            if (sphere_hit_ool(sc.lights[l].s, o, d, mint, h.t, t, &nn)) {
                h.t = t;
                h.tri = -1 - l;
                h.lnn = nn;
            }
        }
    return h;
}

// DiffuseAreaLight::Sample_L (lights/diffuse.cpp:75-87) + VisibilityTester::SetSegment (light.h:87-92)
struct LightSampleOut {
    V3 wi;
    float pdf;
    bool nonblack;    // Ls = L(ps, ns, -wi) = Dot(ns, -wi) > 0 ? Lemit : 0
    V3 so, sd;        // shadow segment ray
    float smint, smaxt;
    float ms, mt;     // infinite light: radiance-map coordinates of the sample
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
    r.ms = r.mt = 0.f;
    return r;
}

// ---- InfiniteAreaLight with the 1x1 radiance map of a light without "mapname"
__device__ __forceinline__ V3 xform3(const float *m, V3 v) {  // Transform::operator()(Vector)
    return V3{(m[0] * v.x + m[1] * v.y) + m[2] * v.z, (m[3] * v.x + m[4] * v.y) + m[5] * v.z,
              (m[6] * v.x + m[7] * v.y) + m[8] * v.z};
}

__device__ __forceinline__ int mod_pbrt(int a, int b) {  // Mod (pbrt.h:282-287)
    const int n = a / b;
    a -= n * b;
    return a < 0 ? a + b : a;
}

// MIPMap<RGBSpectrum>::Lookup(s, t) = triangle(0, s, t) (mipmap.h:239-269) on level 0 with
// TEXTURE_REPEAT: four texels weighted (1-ds)(1-dt), (1-ds)dt, ds(1-dt), ds dt, summed in order
__device__ __forceinline__ void inf_lookup(const RenderLight &L, float s, float t, float rgb[3]) {
    s = s * (float)L.tw - 0.5f;
    t = t * (float)L.th - 0.5f;
    const int s0 = (int)floorf(s), t0 = (int)floorf(t);
    const float ds = s - (float)s0, dt = t - (float)t0;
    const float w0 = (1.f - ds) * (1.f - dt), w1 = (1.f - ds) * dt, w2 = ds * (1.f - dt), w3 = ds * dt;
    const int sa = mod_pbrt(s0, L.tw), sb = mod_pbrt(s0 + 1, L.tw);
    const int ta = mod_pbrt(t0, L.th) * L.tw, tb = mod_pbrt(t0 + 1, L.th) * L.tw;
    const float *a = L.tex + 3 * (ta + sa), *b = L.tex + 3 * (tb + sa), *c = L.tex + 3 * (ta + sb),
                *d = L.tex + 3 * (tb + sb);
    for (int k = 0; k < 3; ++k) rgb[k] = ((a[k] * w0 + b[k] * w1) + c[k] * w2) + d[k] * w3;
}

// Distribution1D::SampleContinuous (montecarlo.h:81-98): std::upper_bound over cdf[0..count]
__device__ __forceinline__ float d1_sample(const float *func, const float *cdf, float fint, int count, float u,
                                           float &pdf, int &off) {
    int lo = 0, len = count + 1;
    while (len > 0) {
        const int half = len >> 1;
        if (!(u < cdf[lo + half])) {
            lo += half + 1;
            len -= half + 1;
        } else {
            len = half;
        }
    }
    int offset = lo - 1;
    offset = offset < 0 ? 0 : (offset > count - 1 ? count - 1 : offset);
    off = offset;
    const float du = (u - cdf[offset]) / (cdf[offset + 1] - cdf[offset]);
    pdf = func[offset] / fint;
    return ((float)offset + du) / (float)count;
}

// band c of Spectrum(rgb, SPECTRUM_ILLUMINANT) = SampledSpectrum::FromRGB (spectrum.cpp:103-187)
__device__ __forceinline__ float illum_band(const float rgb[3], int c) {
    const float R = rgb[0], G = rgb[1], B = rgb[2];
    float r = 0.f;
    if (R <= G && R <= B) {
        r += kIllum[0][c] * R;
        if (G <= B) {
            r += kIllum[1][c] * (G - R);
            r += kIllum[6][c] * (B - G);
        } else {
            r += kIllum[1][c] * (B - R);
            r += kIllum[5][c] * (G - B);
        }
    } else if (G <= R && G <= B) {
        r += kIllum[0][c] * G;
        if (R <= B) {
            r += kIllum[2][c] * (R - G);
            r += kIllum[6][c] * (B - R);
        } else {
            r += kIllum[2][c] * (B - G);
            r += kIllum[4][c] * (R - B);
        }
    } else {
        r += kIllum[0][c] * B;
        if (R <= G) {
            r += kIllum[3][c] * (R - B);
            r += kIllum[5][c] * (G - R);
        } else {
            r += kIllum[3][c] * (G - B);
            r += kIllum[4][c] * (R - G);
        }
    }
    const float v = r * .86445f;
    return v < 0.f ? 0.f : v;  // Clamp(0, INFINITY)
}

// band c of Spectrum::FromRGB(rgb) (reflectance; spectrum.cpp:103-187): ImageTexture's convertOut
__device__ __forceinline__ float refl_band(const float rgb[3], int c) {
    const float R = rgb[0], G = rgb[1], B = rgb[2];
    float r = 0.f;
    if (R <= G && R <= B) {
        r += kRefl[0][c] * R;
        if (G <= B) {
            r += kRefl[1][c] * (G - R);
            r += kRefl[6][c] * (B - G);
        } else {
            r += kRefl[1][c] * (B - R);
            r += kRefl[5][c] * (G - B);
        }
    } else if (G <= R && G <= B) {
        r += kRefl[0][c] * G;
        if (R <= B) {
            r += kRefl[2][c] * (R - G);
            r += kRefl[6][c] * (B - R);
        } else {
            r += kRefl[2][c] * (B - G);
            r += kRefl[4][c] * (R - B);
        }
    } else {
        r += kRefl[0][c] * B;
        if (R <= G) {
            r += kRefl[3][c] * (R - B);
            r += kRefl[5][c] * (G - R);
        } else {
            r += kRefl[3][c] * (G - B);
            r += kRefl[4][c] * (R - G);
        }
    }
    const float v = r * .94f;
    return v < 0.f ? 0.f : v;
}

// Pow(albedo, e) band c for a textured albedo: the ImageTexture value at the point, FromRGB. The
// exponent is mix or 1 - mix, 0.5 at the default mix: then pow(x, 0.5) = sqrt(x) for every x >= +0
// (refl_band clamps at 0) -- the correctly rounded sqrtf, where the double pow rounded to float costs
// a software log and exp per band per hit (3.3 ms of a textured C2 frame's 3.4 M SSS hits x 30 bands)
__device__ __noinline__ float tex_pow_general(float x, float e) { return m_pow(x, e); }
__device__ __forceinline__ float tex_albedo_pow(const float rgb[3], int c, float e) {
    const float x = refl_band(rgb, c);
    return e == 0.5f ? __builtin_sqrtf(x) : tex_pow_general(x, e);
}

__device__ __noinline__ bool inf_nonblack(const RenderLight &L, float s, float t) {  // !Le.IsBlack()
    float rgb[3];
    inf_lookup(L, s, t, rgb);
    for (int c = 0; c < NB; ++c)
        if (illum_band(rgb, c) != 0.f) return true;
    return false;
}

// InfiniteAreaLight::Le (infinite.cpp:115-120): map coordinates of a world direction
__device__ __noinline__ void inf_coords(const RenderLight &L, V3 d, float &s, float &t) {
    const V3 wh = normalize(xform3(L.w2l, d));
    float ph = m_atan2(wh.y, wh.x);  // SphericalPhi
    ph = ph < 0.f ? ph + 2.f * kPiF : ph;
    s = ph * 0.15915494309189533577f;  // INV_TWOPI
    const float z = wh.z < -1.f ? -1.f : (wh.z > 1.f ? 1.f : wh.z);
    t = m_acos(z) * kInvPiF;  // SphericalTheta * INV_PI
}

// InfiniteAreaLight::Sample_L (infinite.cpp:195-218): Distribution2D::SampleContinuous
// (montecarlo.h:154-161) picks a row with the marginal, then a column in that row;
// VisibilityTester::SetRay (light.h:93-96). (ms, mt) = uv, where Ls is looked up.
__device__ __noinline__ LightSampleOut sample_infinite(const RenderLight &L, V3 p, float peps, float u0, float u1) {
    LightSampleOut r;
    float pdf0, pdf1;
    int v, col;
    const float uv1 = d1_sample(L.rint, L.mcdf, L.mint, L.nv, u1, pdf1, v);
    const float uv0 = d1_sample(L.func + (size_t)v * L.nu, L.cdf + (size_t)v * (L.nu + 1), L.rint[v], L.nu, u0, pdf0, col);
    const float mapPdf = pdf0 * pdf1;
    r.ms = uv0;
    r.mt = uv1;
    r.so = p;
    r.smint = peps;
    r.smaxt = INFINITY;
    if (mapPdf == 0.f) {  // "return 0.f": Ls black, nothing contributes
        r.wi = r.sd = V3{0.f, 0.f, 0.f};
        r.pdf = 0.f;
        r.nonblack = false;
        return r;
    }
    const float theta = uv1 * kPiF, phi = (uv0 * 2.f) * kPiF;
    const float costheta = m_cos(theta), sintheta = m_sin(theta);
    const float sinphi = m_sin(phi), cosphi = m_cos(phi);
    r.wi = xform3(L.l2w, V3{sintheta * cosphi, sintheta * sinphi, costheta});
    r.pdf = mapPdf / (((2.f * kPiF) * kPiF) * sintheta);
    if (sintheta == 0.f) r.pdf = 0.f;
    r.sd = r.wi;
    r.nonblack = inf_nonblack(L, uv0, uv1);
    return r;
}

// InfiniteAreaLight::Pdf (infinite.cpp:222-232) with Distribution2D::Pdf (montecarlo.h:162-170)
__device__ __noinline__ float infinite_pdf(const RenderLight &L, V3 w) {
    const V3 wi = xform3(L.w2l, w);
    const float z = wi.z < -1.f ? -1.f : (wi.z > 1.f ? 1.f : wi.z);
    const float theta = m_acos(z);
    float phi = m_atan2(wi.y, wi.x);
    phi = phi < 0.f ? phi + 2.f * kPiF : phi;
    const float sintheta = m_sin(theta);
    if (sintheta == 0.f) return 0.f;
    int iu = (int)(phi * kInvTwoPiF * (float)L.nu), iv = (int)(theta * kInvPiF * (float)L.nv);
    iu = iu < 0 ? 0 : (iu > L.nu - 1 ? L.nu - 1 : iu);
    iv = iv < 0 ? 0 : (iv > L.nv - 1 ? L.nv - 1 : iv);
    const float ri = L.rint[iv];
    const float dp = ri * L.mint == 0.f ? 0.f : (L.func[(size_t)iv * L.nu + iu] * ri) / (ri * L.mint);
    return dp / (((2.f * kPiF) * kPiF) * sintheta);
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
                                                         const uint32_t *__restrict__ sp_mat,
                                                         const float *__restrict__ sp_uv, int n, uint32_t seed,
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
        uint32_t scr0, scr1;
        if (sc.irr_scr) {  // the reference's RNG(47 k) stream (replay_irradiance_kernel)
            scr0 = sc.irr_scr[((size_t)i * sc.nlights + l) * 2];
            scr1 = sc.irr_scr[((size_t)i * sc.nlights + l) * 2 + 1];
        } else {
            scr0 = hash3(seed, (uint32_t)i, 16u * l + DIM_IRR_POS);
            scr1 = hash3(seed, (uint32_t)i, 16u * l + DIM_IRR_POS + 8u);
        }
        for (int s = 0; s < ns; ++s) {
            const float u0 = van_der_corput((uint32_t)s, scr0), u1 = sobol2((uint32_t)s, scr1);  // Sample02
            const LightSampleOut ls = L.kind ? sample_infinite(L, p, eps, u0, u1) : sample_light(L, p, eps, u0, u1);
            if (dot(ls.wi, nrm) <= 0.f) continue;
            if (!ls.nonblack || ls.pdf == 0.f) continue;
            if (!trace_any(sc, ls.so, ls.sd, ls.smint, ls.smaxt, stk, 256)) {
                float ct = absdot(ls.wi, nrm);
                ct = ct < 1.f ? ct : 1.f;
                const float Ft = bss ? 1.f - rho_lookup(mat->rho, mat->n_rho, ct) : 1.f;
                if (L.kind) {  // Li = Spectrum(map lookup at the sampled uv, SPECTRUM_ILLUMINANT)
                    float rgb[3];
                    inf_lookup(L, ls.ms, ls.mt, rgb);
                    for (int c = 0; c < NB; ++c) El[c] += Ft * illum_band(rgb, c) * ct / ls.pdf;
                } else {
                    for (int c = 0; c < NB; ++c) El[c] += Ft * L.Lemit[c] * ct / ls.pdf;
                }
            }
        }
        for (int c = 0; c < NB; ++c) E[c] += El[c] / (float)ns;
    }
    if (bss && mat->has_alb_tex) {  // albedo->Evaluate(dgs): dgs has no differentials -> triangle(0, s, t)
        const UVDiff g{sp_uv[2 * i], sp_uv[2 * i + 1], 0.f, 0.f, 0.f, 0.f};
        float rgb[3];
        tex_eval(mat->alb_tex, g, rgb);
        for (int c = 0; c < NB; ++c) E[c] *= tex_albedo_pow(rgb, c, mat->mix);
    } else if (bss) {
        for (int c = 0; c < NB; ++c) E[c] *= mat->alb_mix[c];
    }
    for (int c = 0; c < NB; ++c) E_out[(size_t)i * NB + c] = E[c];
}

// ------------------------------------------------------------------ Poisson point finder
// SurfacePointTask::Run's paths (renderers/surfacepoints.cpp:181-215): from pCamera in a
// uniformly random direction, up to 30 rays; a ray that leaves the scene bounces off the inside
// of the bounding sphere; hits of rays of depth >= 3 on a surface whose material has a BSSRDF
// become candidate SurfacePoints (p, shading normal, u, v, material, area, rayEpsilon); each
// next direction is a uniform sphere sample turned to the faceforwarded normal. Random numbers
// are counter-based per (seed, path, draw) -- replay mode, like the render sampler.
__device__ __forceinline__ float poisson_u01(uint32_t seed, uint32_t path, uint32_t k) {
    return (float)(hash3(seed, path, k) >> 8) * 0x1p-24f;
}
__device__ __forceinline__ V3 sphere_hit_point(const SphereView &s, V3 o, V3 d, float t) {
    V3 ph = (o - s.c) + d * t;  // object-space Ray::operator() of the translated sphere
    if (ph.x == 0.f && ph.y == 0.f) ph.x = 1e-5f * s.r;
    return ph + s.c;
}
__device__ __forceinline__ V3 faceforward(V3 n, V3 v) { return dot(n, v) < 0.f ? -n : n; }

__global__ __launch_bounds__(256) void poisson_walk_kernel(RenderScene sc, PoissonWalk w, SurfacePoint *out,
                                                           int *count) {
    __shared__ int stk_all[kStack * 256];
    int *stk = stk_all + threadIdx.x;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= w.npaths) return;
    const uint32_t path = w.path0 + (uint32_t)i;
    uint32_t k = 0;
    float u1 = poisson_u01(w.seed, path, k++), u2 = poisson_u01(w.seed, path, k++);
    V3 o = w.origin, d = uniform_sample_sphere(u1, u2);
    float mint = 0.f;
    int n = 0;
    SurfacePoint *mine = out + (size_t)i * kPoissonCand;
    for (int depth = 0; depth < kPoissonDepth; ++depth) {
        const Hit h = trace_closest(sc, o, d, mint, INFINITY, stk, 256);
        V3 p, nn;
        float eps;
        if (h.tri == INT_MIN) {  // sphere.Intersect(ray, &isect): the bounding sphere
            float t;
            V3 snn;
            if (!sphere_intersect(w.bound, o, d, mint, INFINITY, t, &snn)) break;
            p = sphere_hit_point(w.bound, o, d, t);
            nn = snn;
            eps = 5e-4f * t;
            nn = faceforward(nn, -d);
        } else if (h.tri < 0) {  // an area light's sphere (its material has no BSSRDF)
            p = sphere_hit_point(sc.lights[-1 - h.tri].s, o, d, h.t);
            nn = faceforward(h.lnn, -d);
            eps = 5e-4f * h.t;
        } else {
            const int mi = sc.tri_mesh[h.tri], lt = sc.tri_local[h.tri];
            const RenderMesh &mesh = sc.meshes[mi];
            p = o + d * h.t;
            const ShadingFrame fr = tri_shading(mesh.view, lt, p, 1.f - h.b1 - h.b2, h.b1, h.b2);
            nn = faceforward(fr.ng, -d);
            eps = 1e-3f * h.t;
            // every mesh material is a LayeredSkin, whose GetBSSRDF is never NULL (layeredskin.cpp:170-177;
            // surfacepoints.cpp:202) -- genprofile false included: its points are candidates too
            if (depth >= 3 && mesh.material < (uint32_t)sc.nmaterials) {
                // dgs = Bump(hitGeometry, dgShading); without N and S the shading geometry is dg itself
                // (its nn already faceforwarded); no ray differentials (GetBSSRDF(RayDifferential(ray)))
                V3 sn = (!mesh.view.N && !mesh.view.S) ? nn : fr.nn;
                const RenderMaterial &mt = sc.materials[mesh.material];
                if (mt.has_bump) {
                    const UVDiff g{fr.u, fr.v, 0.f, 0.f, 0.f, 0.f};
                    V3 dpdu_b;
                    bump_frame(mt.bump_tex, g, fr.ss, fr.ts, fr.dndu, fr.dndv, sn, nn, mesh.view.flip, dpdu_b, sn);
                }
                SurfacePoint sp;
                sp.p[0] = p.x;
                sp.p[1] = p.y;
                sp.p[2] = p.z;
                sp.n[0] = sn.x;
                sp.n[1] = sn.y;
                sp.n[2] = sn.z;
                sp.u = fr.u;
                sp.v = fr.v;
                sp.material = mesh.material;
                sp.area = 0.f;  // pi (minDist / 2)^2, set by the host
                sp.ray_eps = eps;
                mine[n++] = sp;
            }
        }
        u1 = poisson_u01(w.seed, path, k++);
        u2 = poisson_u01(w.seed, path, k++);
        d = faceforward(uniform_sample_sphere(u1, u2), nn);
        o = p;
        mint = eps;
    }
    count[i] = n;
}

// Value k of camera sample s of pixel (px, py) in the batch's replay window (RenderScene::replay)
__device__ __forceinline__ float replay_val(const RenderScene &sc, int px, int py, int s, int k) {
    const int64_t p = (int64_t)(py - sc.replay_y0) * sc.replay_w + (px - sc.replay_x0);
    return sc.replay[((int64_t)k * sc.replay_npix + p) * sc.replay_spp + s];
}

// The image sample of camera sample s of pixel (px, py): LDPixelSample's imageX = xPos + u
__device__ __forceinline__ void image_sample(const RenderScene &sc, uint32_t seed, int px, int py, int s, float &X,
                                             float &Y) {
    if (sc.replay) {
        X = (float)px + replay_val(sc, px, py, s, 0);
        Y = (float)py + replay_val(sc, px, py, s, 1);
        return;
    }
    const uint32_t pix = (uint32_t)py * (uint32_t)sc.xres + (uint32_t)px;
    X = (float)px + van_der_corput((uint32_t)s, hash3(seed, pix, DIM_IMAGE));
    Y = (float)py + sobol2((uint32_t)s, hash3(seed, pix, DIM_IMAGE + 1));
}

// ------------------------------------------------------------------ camera rays (primary)
// SamplerRendererTask::Run's per-sample head: image sample -> PerspectiveCamera::GenerateRay ->
// Scene::Intersect. Surface hits are compacted (one atomic per wave, sample order kept inside
// the wave) so the shading kernel runs on full waves; a miss or an area-light hit ends here.
__global__ __launch_bounds__(256) void primary_kernel(RenderScene sc, PieceList pl, SampleRecs rec) {
    __shared__ int snode_all[kStack * 4];  // one traversal stack per wave (trace_closest_wave)
    __shared__ uint64_t smask_all[kStack * 4];
    const int wv = (int)(threadIdx.x >> 6);
    const int k = piece_of(pl, (int)blockIdx.x);
    const TileBatch &tb = pl.tb[k];
    rec.flags += pl.off[k];
    rec.slot += pl.off[k];
    rec.spill += pl.off[k] / tb.spp;
    const int64_t sid0 = (int64_t)((int)blockIdx.x - pl.block0[k]) * blockDim.x + threadIdx.x;
    const bool in_range = sid0 < tb.nsamples;
    const int64_t sid = in_range ? sid0 : tb.nsamples - 1;
    const int s = (int)(sid % tb.spp);
    const int li = (int)(sid / tb.spp);
    const int px = tb.ex0 + li % tb.ew, py = tb.ey0 + li / tb.ew;
    const uint32_t pix = (uint32_t)py * (uint32_t)sc.xres + (uint32_t)px;
    // image sample (LDPixelSample's imageSamples, montecarlo.cpp:200-250): imageX = x + u in float
    float X, Y;
    image_sample(sc, tb.seed, px, py, s, X, Y);
    // border samples matter only when the box filter carries them into the tile (film_kernel)
    int lx, hx, ly, hy;
    film_extent(X, sc.xres, lx, hx);
    film_extent(Y, sc.yres, ly, hy);
    const bool live = in_range && lx < tb.x1 && hx >= tb.x0 && ly < tb.y1 && hy >= tb.y0;
    uint32_t flags = 0;
    V3 d = V3{1.f, 1.f, 1.f};
    const V3 o = xform_point(sc.camera_to_world, V3{0.f, 0.f, 0.f});
    if (live) {
        flags |= REC_LIVE;
        const uint32_t edge = (lx < px ? REC_XLO : 0u) | (hx > px ? REC_XHI : 0u) | (ly < py ? REC_YLO : 0u) |
                              (hy > py ? REC_YHI : 0u);
        if (edge) {
            flags |= edge;
            atomicOr(&rec.spill[li], edge);
        }
        // PerspectiveCamera::GenerateRay (cameras/perspective.cpp)
        const V3 pcam = xform_point(sc.raster_to_camera, V3{X, Y, 0.f});
        d = xform_vector(sc.camera_to_world, normalize(pcam));
    }
    // Scene::Intersect, the wave's rays as sign packets (one pixel's samples share one packet)
    const Hit h = trace_closest_wave(sc, o, d, 0.f, INFINITY, live, snode_all + kStack * wv, smask_all + kStack * wv);
    if (live) {
        if (h.tri == INT_MIN) {  // SamplerRenderer::Li: Li += lights[i]->Le(ray) for every light
            if (sc.n_infinite > 0) flags |= REC_LE | (0xffu << REC_LIGHT_SHIFT);
        } else if (h.tri < 0) {  // an area light's own sphere: Le(wo) if it faces wo, then matte shading
            const int l = -1 - h.tri;
            flags |= REC_LSURF | ((uint32_t)l << REC_LIGHT_SHIFT);
            if (dot(h.lnn, -d) > 0.f) flags |= REC_LE;
        } else if (h.tri != INT_MIN) {
            const uint32_t mid = sc.meshes[sc.tri_mesh[h.tri]].material;
            flags |= REC_SURF | (mid << REC_MAT_SHIFT);
            if (sc.materials[mid].has_bssrdf && sc.have_octree) flags |= REC_SSS;
        }
    }
    // every sample with radiance (a surface hit, or an area light seen directly) gets a slot
    const bool surf = (flags & REC_SURF) != 0, has_l = surf || (flags & (REC_LE | REC_LSURF));
    const uint64_t m = __builtin_amdgcn_ballot_w64(has_l);
    const int lane = (int)(threadIdx.x & 63);
    int base = 0;
    if (lane == 0 && m) base = atomicAdd(rec.hit_count, (int)__builtin_popcountll(m));
    base = __shfl(base, 0);
    const int slot = base + (int)__builtin_popcountll(m & ((1ull << lane) - 1ull));
    if (!in_range) return;
    rec.flags[sid] = flags;
    rec.slot[sid] = has_l ? slot : -1;
    if (surf) {
        rec.hit_a[slot] = make_float4(h.t, h.b1, h.b2, __int_as_float(h.tri));
        rec.hit_b[slot] = make_float4(d.x, d.y, d.z, __uint_as_float(pix));
        // sample index (16 bits) | material (8 bits) | SSS bit 31
        rec.hit_s[slot] = (uint32_t)s | (flags & (0xffu << REC_MAT_SHIFT)) | ((flags & REC_SSS) ? HS_SSS : 0u);
    } else if (has_l) {
        // a light seen directly: light index (0xff = the infinite lights of a miss); a light sphere's
        // surface is also shaded (HS_LSURF), its Le counted when it faces the ray (HS_LE)
        rec.hit_s[slot] = (uint32_t)s | (((flags >> REC_LIGHT_SHIFT) & 0xffu) << REC_MAT_SHIFT) | HS_LIGHT |
                          ((flags & REC_LSURF) ? HS_LSURF : 0u) | ((flags & REC_LE) ? HS_LE : 0u);
        rec.hit_b[slot] = make_float4(d.x, d.y, d.z, __uint_as_float(pix));
        if (flags & REC_LSURF) rec.hit_a[slot] = make_float4(h.t, 0.f, 0.f, __int_as_float(h.tri));
    }
}

// ------------------------------------------------------------------ shading + direct light
// The rest of MultipoleSubsurfaceIntegrator::Li for the compacted surface hits, with one lane
// per (hit, light, light-sample j) of UniformSampleAllLights (integrator.cpp:47-77): each lane
// runs one EstimateDirect (:117-174) -- light sample + shadow ray, BSDF sample + ray -- and
// stores its scalars; direct_combine_kernel then forms the per-band sums in the reference's
// order (j ascending inside a light, lights ascending). A BSDF value is R[c] * D * G * F / den
// (Microfacet::f) with scalar D, G, F, den, so no lane carries a 30-band spectrum.
// One lobe value of the layer-0 BSDF for a direction pair (BSDF::f, reflection.cpp:765-779):
// kind 1 = Microfacet (R * D * G * F / den), kind 2 = MicrofacetTransmission (T * s * (1 - F)).
// The transmission lobe and the infinite light run only for the materials / scenes that have
// them; they are called out of line so the common path keeps its code small (I-cache).
__device__ __noinline__ MtTerms mt_terms_ool(const Microfacet &m, V3 wo, V3 wi) { return mt_terms(m, wo, wi); }
__device__ __noinline__ float mt_pdf_ool(const Microfacet &m, V3 wo, V3 wi) { return mt_pdf(m, wo, wi); }
__device__ __noinline__ void mt_sample_ool(const Microfacet &m, V3 wo, float u1, float u2, V3 &wi, float &pdf) {
    mt_sample(m, wo, u1, u2, wi, pdf);
}

struct Lobe {
    uint32_t kind;
    float a, b, c, d;
};

// The shading point's BSDF is a mesh material's (mat), or -- mat == nullptr -- the default matte of a
// light sphere seen directly (geom.h kMatteF): kind 3, f = 0 + R * INV_PI on the reflection side.
__device__ __forceinline__ Lobe bsdf_lobe(const RenderMaterial *mat, bool refl, V3 wo_l, V3 wi_l) {
    Lobe L{0u, 0.f, 0.f, 0.f, 1.f};
    if (!mat) {
        if (refl) L = Lobe{3u, 0.f + kMatteF, 0.f, 0.f, 1.f};
    } else if (refl) {  // the ng test keeps BRDFs only
        if (mat->has_refl) {
            const MfTerms t = microfacet_terms(mat->mf, wo_l, wi_l);
            if (!t.zero) L = Lobe{1u, t.D, t.G, t.F, t.den};
        }
    } else if (mat->has_trans) {  // ... or BTDFs only
        const MtTerms t = mt_terms_ool(mat->mf, wo_l, wi_l);
        if (!t.zero) L = Lobe{2u, t.s, t.F, 0.f, 1.f};
    }
    return L;
}

__device__ __forceinline__ float lobe_value(const RenderMaterial *mat, const Lobe &L, int c) {
    if (L.kind == 3u) return L.a;
    return L.kind == 1u ? mat->R[c] * L.a * L.b * L.c / L.d : (mat->T[c] * L.a) * (1.f - L.b);
}

// x / d (IEEE, correctly rounded) for many x over one d, from inv = x-independent RN(1 / d): with
// q = RN(x inv) and the exact residual r = x - d q (one FMA), RN(q + r inv) is RN(x / d) -- Markstein's
// correction, valid when nothing under- or overflows (it replaces the ~10-instruction IEEE division
// sequence by 3 instructions; tools/check_div.c runs it against x / d on 2e8 random operand pairs, 0
// differences). Outside the guarded range, and when d itself is out of range (dok false), it divides.
__device__ __forceinline__ float div_by(float x, float d, float inv, bool dok) {
    const float q = x * inv;
    const float r = __builtin_fmaf(-d, q, x);
    const float q1 = __builtin_fmaf(r, inv, q);
    const float ax = fabsf(x), aq = fabsf(q1);
    if (dok && ax >= 0x1p-100f && ax <= 0x1p100f && aq >= 0x1p-100f && aq <= 0x1p100f) return q1;
    return x / d;
}
struct Den {  // one denominator shared by the 30 bands
    float d, inv;
    bool ok;
};
__device__ __forceinline__ Den make_den(float d) {
    const float ad = fabsf(d);
    return Den{d, 1.f / d, ad >= 0x1p-60f && ad <= 0x1p60f};
}
// lobe_value with the reflection lobe's division by L.d done through den = make_den(L.d)
__device__ __forceinline__ float lobe_value_den(const RenderMaterial *mat, const Lobe &L, int c, const Den &den) {
    if (L.kind == 3u) return L.a;
    return L.kind == 1u ? div_by(mat->R[c] * L.a * L.b * L.c, den.d, den.inv, den.ok)
                        : (mat->T[c] * L.a) * (1.f - L.b);
}

__device__ __forceinline__ bool lobe_black(const RenderMaterial *mat, const Lobe &L) {
    if (L.kind == 0u) return true;
    if (L.kind == 3u) return false;
    for (int c = 0; c < NB; ++c)
        if (lobe_value(mat, L, c) != 0.f) return false;
    return true;
}

// BSDF::Pdf (reflection.cpp:736-751): mean of the matching lobes' pdfs, R then T
__device__ __forceinline__ float bsdf_pdf(const RenderMaterial *mat, V3 wo_l, V3 wi_l) {
    if (!mat) return lambert_pdf(wo_l, wi_l);  // (0 + pdf) / 1
    const int n = mat->has_refl + mat->has_trans;
    if (n == 0) return 0.f;
    float pdf = 0.f;
    if (mat->has_refl) pdf += microfacet_pdf(mat->mf, wo_l, wi_l);
    if (mat->has_trans) pdf += mt_pdf_ool(mat->mf, wo_l, wi_l);
    return pdf / (float)n;
}

// ------------------------------------------------------------------ shading + direct light
// The rest of MultipoleSubsurfaceIntegrator::Li for the compacted surface hits, with one lane
// per (hit, light, light-sample j) of UniformSampleAllLights (integrator.cpp:47-77): each lane
// runs one EstimateDirect (:117-174) -- light sample + shadow ray, BSDF sample + ray -- and
// stores its scalars; direct_combine_kernel then forms the per-band sums in the reference's
// order (j ascending inside a light, lights ascending). BSDF values are a 30-band factor times
// scalars (Lobe), so no lane carries a spectrum.
struct DirectTerms {       // 16 words: one EstimateDirect
    float k1, adn, w2, pdf2;   // light term f * Li * k1; BSDF term f * Li * adn * w2 / pdf2
    Lobe l1, l2;               // the BSDF lobe value of each term (kind 0: term absent)
    float pad[2];
};
static_assert(sizeof(DirectTerms) == 64, "one 64-B record per light sample");

__global__ __launch_bounds__(256) void shade_direct_kernel(RenderScene sc, SampleRecs rec, int spp, uint32_t seed,
                                                           int max_hits, int ns_max, DirectTerms *terms,
                                                           float4 *__restrict__ inf_st) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int per_hit = sc.nlights * ns_max;
    const int nhits = *rec.hit_count;
    if ((int64_t)blockIdx.x * blockDim.x >= (int64_t)nhits * per_hit) return;
    const int slot = (int)(gid / per_hit);
    if (slot >= nhits || slot >= max_hits) return;
    const int lj = (int)(gid % per_hit), l = lj / ns_max, j = lj % ns_max;
    const uint32_t hs = rec.hit_s[slot];
    const bool lsurf = (hs & HS_LSURF) != 0;  // a light sphere's own surface: matte, no Mo()
    if ((hs & HS_LIGHT) && !lsurf) {  // a miss with infinite lights: no shading point, no Mo()
        if (lj == 0) rec.hit_q[slot] = make_float4(0.f, 0.f, 0.f, -1.f);
        return;
    }
    const RenderLight &L = sc.lights[l];
    const int ns = L.nsamples_round;
    DirectTerms out{};
    if (j >= ns && lj != 0) return;
    const float4 ha = rec.hit_a[slot], hb = rec.hit_b[slot];
    const int s = (int)(hs & 0xffffu);
    const uint32_t mid = (hs >> REC_MAT_SHIFT) & 0xffu;
    const bool sss = (hs >> 31) != 0;
    const int tri = __float_as_int(ha.w);
    const uint32_t pix = __float_as_uint(hb.w);
    const V3 d = V3{hb.x, hb.y, hb.z};
    const V3 o = xform_point(sc.camera_to_world, V3{0.f, 0.f, 0.f});
    const V3 wo = -d;
    ShadingFrame fr;
    float reps;
    const RenderMaterial *mat = nullptr;
    if (lsurf) {  // Sphere::Intersect: rayEpsilon = 5e-4f * thit (sphere.cpp:155)
        fr = sphere_frame(sc.lights[-1 - tri].s, o, d, ha.x);
        reps = 5e-4f * ha.x;
    } else {
        const RenderMesh &mesh = sc.meshes[sc.tri_mesh[tri]];
        const V3 p = o + d * ha.x;  // Ray::operator()
        reps = 1e-3f * ha.x;
        fr = tri_shading(mesh.view, sc.tri_local[tri], p, 1.f - ha.y - ha.z, ha.y, ha.z);
        mat = &sc.materials[mid];
        if (mat->has_bump) {  // BSDF on the bumped dgs: nn, sn = Normalize(dpdu), tn = Cross(nn, sn)
            const float4 a = rec.hit_frame[2 * (size_t)slot], b = rec.hit_frame[2 * (size_t)slot + 1];
            fr.nn = V3{a.x, a.y, a.z};
            fr.sn = V3{b.x, b.y, b.z};
            fr.tn = cross(fr.nn, fr.sn);
        }
    }
    if (lj == 0) {
        float ct = absdot(wo, fr.nn);
        ct = ct < 1.f ? ct : 1.f;
        rec.hit_q[slot] = make_float4(fr.p.x, fr.p.y, fr.p.z, sss ? ct : -1.f);
        if (j >= ns) return;
    }
    const int ncomp = mat ? mat->has_refl + mat->has_trans : 1;
    const V3 wo_l = to_local(fr, wo);
    const float ng_wo = dot(wo, fr.ng);
    // LightSample(sample, offsets, j) / BSDFSample(sample, offsets, j) (light.cpp, reflection.cpp)
    float lu0, lu1, ubc, ub0, ub1;
    if (sc.replay) {
        const int px = (int)(pix % (uint32_t)sc.xres), py = (int)(pix / (uint32_t)sc.xres);
        const int k = L.replay_off + j * kReplayPerLightSample;
        lu0 = replay_val(sc, px, py, s, k);
        lu1 = replay_val(sc, px, py, s, k + 1);
        ubc = replay_val(sc, px, py, s, k + 2);
        ub0 = replay_val(sc, px, py, s, k + 3);
        ub1 = replay_val(sc, px, py, s, k + 4);
    } else {
        const uint32_t xr = (spp & (spp - 1)) == 0 ? (hash3(seed, pix, 16u * l + 9u) & (uint32_t)(spp - 1)) : 0u;
        const uint32_t nidx = (uint32_t)(s ^ (int)xr) * (uint32_t)ns + (uint32_t)j;
        lu0 = van_der_corput(nidx, hash3(seed, pix, 16u * l + DIM_LIGHT_POS));
        lu1 = sobol2(nidx, hash3(seed, pix, 16u * l + DIM_LIGHT_POS + 8u));
        ubc = van_der_corput(nidx, hash3(seed, pix, 16u * l + DIM_BSDF_COMP));
        ub0 = van_der_corput(nidx, hash3(seed, pix, 16u * l + DIM_BSDF_DIR));
        ub1 = sobol2(nidx, hash3(seed, pix, 16u * l + DIM_BSDF_DIR + 8u));
    }
    // --- light sampling: ed += f * Li * (|wi.n| * w / lightPdf)
    const LightSampleOut ls = L.kind ? sample_infinite(L, fr.p, reps, lu0, lu1) : sample_light(L, fr.p, reps, lu0, lu1);
    float lightPdf = ls.pdf;
    float4 st = make_float4(ls.ms, ls.mt, 0.f, 0.f);
    if (lightPdf > 0.f && ls.nonblack && ncomp > 0) {
        const V3 wi_l = to_local(fr, ls.wi);
        const Lobe f1 = bsdf_lobe(mat, dot(ls.wi, fr.ng) * ng_wo > 0.f, wo_l, wi_l);
        if (!lobe_black(mat, f1) && !trace_any_wave(sc, ls.so, ls.sd, ls.smint, ls.smaxt, true, false, true)) {
            const float bsdfPdf = bsdf_pdf(mat, wo_l, wi_l);
            const float w = power_heuristic(lightPdf, bsdfPdf);
            out.k1 = absdot(ls.wi, fr.nn) * w / lightPdf;
            out.l1 = f1;
        }
    }
    // --- BSDF sampling (BSDF::Sample_f, reflection.cpp:675-733): ed += f * Li * |wi.n| * w / pdf
    if (ncomp > 0) {
        int which = (int)floorf(ubc * (float)ncomp);
        which = which < ncomp - 1 ? which : ncomp - 1;
        const bool pick_t = mat && (!mat->has_refl || which == 1);
        V3 wi_l;
        float bsdfPdf;
        if (!mat)
            lambert_sample(wo_l, ub0, ub1, wi_l, bsdfPdf);
        else if (pick_t)
            mt_sample_ool(mat->mf, wo_l, ub0, ub1, wi_l, bsdfPdf);
        else
            beckmann_sample(mat->mf, wo_l, ub0, ub1, wi_l, bsdfPdf);
        if (bsdfPdf != 0.f) {
            const V3 wi = to_world(fr, wi_l);
            if (ncomp > 1) {
                bsdfPdf += pick_t ? microfacet_pdf(mat->mf, wo_l, wi_l) : mt_pdf_ool(mat->mf, wo_l, wi_l);
                bsdfPdf /= (float)ncomp;
            }
            const Lobe f2 = bsdf_lobe(mat, dot(wi, fr.ng) * ng_wo > 0.f, wo_l, wi_l);
            if (!lobe_black(mat, f2) && bsdfPdf > 0.f) {
                lightPdf = L.kind ? infinite_pdf(L, wi) : sphere_pdf(L.s, fr.p, wi);
                if (lightPdf != 0.f) {
                    const float w = power_heuristic(bsdfPdf, lightPdf);
                    // Li = lightIsect.Le(-wi) when Scene::Intersect's closest primitive is this light;
                    // light->Le(ray) when the ray escapes (0 for an area light). Both are answered by
                    // any-hit walks:
                    //  * infinite light: the ray escapes iff it hits no triangle and no light sphere;
                    //  * area light: the ray meets the light only if it meets its sphere at all (the
                    //    sphere test with maxt = inf accepts every hit the closest-hit search would), at
                    //    tl. The closest-hit search from maxt = tl ends on a triangle iff one lies at
                    //    t < tl (at t == tl the spheres, tested last, take over), and otherwise its
                    //    sphere loop alone decides -- so: no triangle before tl (strict any-hit), then
                    //    the sphere loop from tl, exactly as trace_closest runs it.
                    bool lit = false;
                    if (L.kind) {
                        lit = !trace_any_wave(sc, fr.p, wi, reps, INFINITY, true, false, true);
                        if (lit) {
                            inf_coords(L, wi, st.z, st.w);
                            lit = inf_nonblack(L, st.z, st.w);
                        }
                    } else {
                        float tl;
                        if (sphere_hit_ool(L.s, fr.p, wi, reps, INFINITY, tl, nullptr) &&
                            !trace_any_wave(sc, fr.p, wi, reps, tl, true, true, false)) {
                            float ht = tl;
                            int who = INT_MIN;
                            V3 lnn = V3{0.f, 0.f, 0.f};
                            for (int k = 0; k < sc.nlights; ++k) {
                                if (sc.lights[k].kind) continue;
                                float t;
                                V3 nn;
                                if (sphere_hit_ool(sc.lights[k].s, fr.p, wi, reps, ht, t, &nn)) {
                                    ht = t;
                                    who = -1 - k;
                                    lnn = nn;
                                }
                            }
                            lit = who == -1 - l && dot(lnn, -wi) > 0.f;
                        }
                    }
                    if (lit) {
                        out.adn = absdot(wi, fr.nn);
                        out.w2 = w;
                        out.pdf2 = bsdfPdf;
                        out.l2 = f2;
                    }
                }
            }
        }
    }
    terms[gid] = out;
    if (L.kind) inf_st[gid] = st;
}

// ------------------------------------------------------------------ textures
// Li's GetBSDF / GetMultipoleBSSRDF for materials with an albedo texture or a bump map: the
// camera RayDifferential (PerspectiveCamera::GenerateRayDifferential, perspective.cpp:81-113,
// ScaleDifferentials(1 / sqrtf(spp)), samplerrenderer.cpp:90-91), dg.ComputeDifferentials, then
// albedo->Evaluate(dgShading) (layeredskin.cpp:180-185) and Bump (layeredskin.cpp:143-146).
__global__ __launch_bounds__(256) void shade_tex_kernel(RenderScene sc, SampleRecs rec, int spp, uint32_t seed,
                                                        int max_hits) {
    const int slot = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    const int nhits = *rec.hit_count;
    if (slot >= nhits || slot >= max_hits) return;
    const uint32_t hs = rec.hit_s[slot];
    if (hs & HS_LIGHT) return;
    const RenderMaterial &mat = sc.materials[(hs >> REC_MAT_SHIFT) & 0xffu];
    const bool want_alb = (hs >> 31) && mat.has_alb_tex;
    if (!want_alb && !mat.has_bump) return;
    const float4 ha = rec.hit_a[slot], hb = rec.hit_b[slot];
    const int s = (int)(hs & 0xffffu), tri = __float_as_int(ha.w);
    const uint32_t pix = __float_as_uint(hb.w);
    const V3 d = V3{hb.x, hb.y, hb.z};
    const V3 o = xform_point(sc.camera_to_world, V3{0.f, 0.f, 0.f});
    const RenderMesh &mesh = sc.meshes[sc.tri_mesh[tri]];
    const V3 p = o + d * ha.x;
    const ShadingFrame fr = tri_shading(mesh.view, sc.tri_local[tri], p, 1.f - ha.y - ha.z, ha.y, ha.z);
    // the sample's image position (as primary_kernel) and its offset rays
    const int px = (int)(pix % (uint32_t)sc.xres), py = (int)(pix / (uint32_t)sc.xres);
    float X, Y;
    image_sample(sc, seed, px, py, s, X, Y);
    const V3 pcam = xform_point(sc.raster_to_camera, V3{X, Y, 0.f});
    const V3 dxc = V3{sc.dx_camera[0], sc.dx_camera[1], sc.dx_camera[2]};
    const V3 dyc = V3{sc.dy_camera[0], sc.dy_camera[1], sc.dy_camera[2]};
    const V3 rxw = xform_vector(sc.camera_to_world, normalize(pcam + dxc));
    const V3 ryw = xform_vector(sc.camera_to_world, normalize(pcam + dyc));
    const float k = 1.f / sqrtf((float)spp);
    const V3 rxd = d + (rxw - d) * k, ryd = d + (ryw - d) * k;
    UVDiff g;
    g.u = fr.u;
    g.v = fr.v;
    compute_differentials(p, fr.ng, fr.dpdu, fr.dpdv, o, rxd, ryd, g);
    if (want_alb) {
        float rgb[3];
        tex_eval(mat.alb_tex, g, rgb);
        rec.hit_alb[slot] = make_float4(rgb[0], rgb[1], rgb[2], 0.f);
    }
    if (mat.has_bump) {
        V3 dpdu_b, nn_b;
        bump_frame(mat.bump_tex, g, fr.ss, fr.ts, fr.dndu, fr.dndv, fr.nn, fr.ng, mesh.view.flip, dpdu_b, nn_b);
        const V3 sn = normalize(dpdu_b);  // BSDF: sn = Normalize(dgs.dpdu)
        rec.hit_frame[2 * (size_t)slot] = make_float4(nn_b.x, nn_b.y, nn_b.z, 0.f);
        rec.hit_frame[2 * (size_t)slot + 1] = make_float4(sn.x, sn.y, sn.z, 0.f);
    }
}

// A scene without lights: no direct light and (Preprocess returned early) no octree.
__global__ __launch_bounds__(256) void shade_nolight_kernel(RenderScene sc, SampleRecs rec, int max_hits) {
    const int slot = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    const int nhits = *rec.hit_count;
    if (slot >= nhits || slot >= max_hits) return;
    rec.hit_q[slot] = make_float4(0.f, 0.f, 0.f, -1.f);
    float4 *row = reinterpret_cast<float4 *>(rec.ld + (size_t)slot * ROW);
    for (int k = 0; k < 8; ++k) row[k] = make_float4(0.f, 0.f, 0.f, 0.f);
}

// One test per light sample for the Microfacet half: every band's dividend x = ((R[c] D) G) F and quotient
// x / den lie in div_by's guarded range [2^-100, 2^100] (or x = +0), so the 30 quotients take div_by's fast
// path (RN(x inv) and one Markstein correction) with no per-band range test: the same values. R, D, G, F
// >= 0, so x >= +0. r_lo / r_hi bound R's nonzero values; the factor-2 margins absorb the roundings of
// the bound's own products and of x's (a few ulps).
__device__ __forceinline__ bool refl_quotients_safe(const RenderMaterial &m, const Lobe &L, const Den &den) {
    if (!den.ok || !m.r_nonneg || !(L.a >= 0.f && L.b >= 0.f && L.c >= 0.f)) return false;
    if (L.a == 0.f || L.b == 0.f || L.c == 0.f || m.r_hi == 0.f) return true;  // every x = +0: q = +-0 exactly
    const float abc = (L.a * L.b) * L.c;
    const float lo = m.r_lo * abc, hi = m.r_hi * abc, ai = fabsf(den.inv);
    return lo >= 0x1p-99f && hi <= 0x1p99f && lo * ai >= 0x1p-99f && hi * ai <= 0x1p99f;
}

// ld[c] = sum over lights of (sum over j of (0 + light term + BSDF term)) / ns, band by band in
// the order UniformSampleAllLights accumulates (Ld += EstimateDirect; L += Ld / nSamples). Each
// light sample's record is read once and added to all 30 per-band accumulators (registers);
// every band sees exactly the reference's sequence of float operations. kInf: the scene has
// infinite lights, whose radiance depends on each term's direction (map coordinates in inf_st).
template <bool kInf>
__global__ __launch_bounds__(256) void direct_combine_kernel(RenderScene sc, SampleRecs rec, int max_hits, int ns_max,
                                                             const DirectTerms *__restrict__ terms,
                                                             const float4 *__restrict__ inf_st) {
    const int slot = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    const int nhits = *rec.hit_count;
    if (slot >= nhits || slot >= max_hits) return;
    const uint32_t hs = rec.hit_s[slot];
    if ((hs & HS_LIGHT) && !(hs & HS_LSURF)) return;
    // a light sphere's surface: the matte lobe (kind 3) needs no material
    const RenderMaterial *mat = (hs & HS_LIGHT) ? nullptr : &sc.materials[(hs >> REC_MAT_SHIFT) & 0xffu];
    const size_t base = (size_t)slot * sc.nlights * ns_max;
    float ld[NB];
#pragma unroll
    for (int c = 0; c < NB; ++c) ld[c] = 0.f;
    for (int l = 0; l < sc.nlights; ++l) {
        const RenderLight &L = sc.lights[l];
        const int ns = L.nsamples_round;
        float Ld[NB];
#pragma unroll
        for (int c = 0; c < NB; ++c) Ld[c] = 0.f;
        for (int j = 0; j < ns; ++j) {
            const DirectTerms e = terms[base + l * ns_max + j];
            if (!e.l1.kind && !e.l2.kind) continue;  // ed = 0 and Ld += 0 changes nothing (Ld is never -0)
            float rgb1[3], rgb2[3];
            const bool inf = kInf && L.kind;
            if (inf) {  // Spectrum(map lookup, SPECTRUM_ILLUMINANT) at each term's direction
                const float4 st = inf_st[base + l * ns_max + j];
                inf_lookup(L, st.x, st.y, rgb1);
                inf_lookup(L, st.z, st.w, rgb2);
            }
            const Den d1 = make_den(e.l1.d), d2 = make_den(e.l2.d), dp = make_den(e.pdf2);
            if (!e.l2.kind && e.l1.kind == 1u && refl_quotients_safe(*mat, e.l1, d1)) {
                // the common term: a Microfacet light-sample half alone, its quotients on the fast path
#pragma unroll
                for (int c = 0; c < NB; ++c) {
                    const float Li1 = inf ? illum_band(rgb1, c) : L.Lemit[c];
                    const float x = mat->R[c] * e.l1.a * e.l1.b * e.l1.c;
                    const float q = x * d1.inv;
                    const float f1 = __builtin_fmaf(__builtin_fmaf(-d1.d, q, x), d1.inv, q);
                    Ld[c] += 0.f + f1 * Li1 * e.k1;
                }
                continue;
            }
#pragma unroll
            for (int c = 0; c < NB; ++c) {
                const float Li1 = inf ? illum_band(rgb1, c) : L.Lemit[c];
                const float Li2 = inf ? illum_band(rgb2, c) : L.Lemit[c];
                float ed = 0.f;
                if (e.l1.kind) ed += lobe_value_den(mat, e.l1, c, d1) * Li1 * e.k1;
                if (e.l2.kind) ed += div_by(lobe_value_den(mat, e.l2, c, d2) * Li2 * e.adn * e.w2, dp.d, dp.inv, dp.ok);
                Ld[c] += ed;
            }
        }
        // L += Ld / nSamples. nsamples_round is a power of two (LDSampler::RoundSize), and x / 2^k and
        // x * 2^-k are the same exact real rounded once, for every x (subnormal results included)
        if ((ns & (ns - 1)) == 0) {
            const float inv_ns = 1.f / (float)ns;
#pragma unroll
            for (int c = 0; c < NB; ++c) ld[c] += Ld[c] * inv_ns;
        } else {
            const Den dn = make_den((float)ns);
#pragma unroll
            for (int c = 0; c < NB; ++c) ld[c] += div_by(Ld[c], dn.d, dn.inv, dn.ok);
        }
    }
    float4 *row = reinterpret_cast<float4 *>(rec.ld + (size_t)slot * ROW);
#pragma unroll
    for (int k = 0; k < 7; ++k) row[k] = make_float4(ld[4 * k], ld[4 * k + 1], ld[4 * k + 2], ld[4 * k + 3]);
    row[7] = make_float4(ld[28], ld[29], 0.f, 0.f);
}
template __global__ void direct_combine_kernel<false>(RenderScene, SampleRecs, int, int, const DirectTerms *,
                                                      const float4 *);
template __global__ void direct_combine_kernel<true>(RenderScene, SampleRecs, int, int, const DirectTerms *,
                                                     const float4 *);

// ------------------------------------------------------------------ film
// Li of one camera sample with radiance (MultipoleSubsurfaceIntegrator::Li,
// multipolesubsurface.cpp:253-303): L = 0 + Le; L += ((INV_PI * Ft) * Mo * Pow(albedo, 1 - mix))
// .Clamp(0); L += Ld -- then the SamplerRenderer sample filter (NaN / y < -1e-5 / inf -> 0,
// samplerrenderer.cpp:119-133) and Spectrum::ToXYZ in band order. One lane per slot.
// The common wave: every lane an SSS hit of one untextured material. The material is then
// wave-uniform (its tables are scalar loads), the lane's Ld row and the band-ordered Mo() values
// are all issued up front, and the 30-band loop is unrolled -- the same float operations, in the
// same order, as the general path below.
// Pow(FromRGB(rgb), e) for all 30 bands of a textured albedo, the branches of refl_band (FromRGB,
// spectrum.cpp:103-187) decided once per lane instead of per band: the minimum / middle / maximum
// components and the rows of their secondary (X: Cyan, Magenta, Yellow) and primary (Y: Red, Green,
// Blue) spectra; then per band the same products and sums in the same order. e = 0.5 (the default mix)
// as sqrtf (tex_albedo_pow).
__device__ __forceinline__ void tex_albedo_pow_all(const float4 rgb, float e, float out[NB]) {
    const float R = rgb.x, G = rgb.y, B = rgb.z;
    float mn, md, mx;
    int xi, yi;
    if (R <= G && R <= B) {
        mn = R;
        xi = 1;
        if (G <= B) { md = G; mx = B; yi = 6; } else { md = B; mx = G; yi = 5; }
    } else if (G <= R && G <= B) {
        mn = G;
        xi = 2;
        if (R <= B) { md = R; mx = B; yi = 6; } else { md = B; mx = R; yi = 4; }
    } else {
        mn = B;
        xi = 3;
        if (R <= G) { md = R; mx = G; yi = 5; } else { md = G; mx = R; yi = 4; }
    }
    const float d1 = md - mn, d2 = mx - md;
#pragma unroll
    for (int c = 0; c < NB; ++c) {
        const float X = xi == 1 ? kRefl[1][c] : (xi == 2 ? kRefl[2][c] : kRefl[3][c]);
        const float Y = yi == 4 ? kRefl[4][c] : (yi == 5 ? kRefl[5][c] : kRefl[6][c]);
        float r = 0.f;
        r += kRefl[0][c] * mn;
        r += X * d1;
        r += Y * d2;
        float v = r * .94f;
        v = v < 0.f ? 0.f : v;
        out[c] = e == 0.5f ? __builtin_sqrtf(v) : tex_pow_general(v, e);
    }
}

template <bool TEX>
__device__ __forceinline__ void assemble_uniform(const RenderScene &sc, const SampleRecs &rec, int slot, int mid) {
    const RenderMaterial &mat = sc.materials[mid];
    const float4 q = rec.hit_q[slot];
    const float Ft = mat.is_mc ? 1.f : 1.f - rho_lookup(mat.rho, mat.n_rho, q.w);
    const float kss = kInvPiF * Ft;
    const float *mo = reinterpret_cast<const float *>(rec.mo4 + (size_t)slot * kGroups);
    const float4 *ld4 = reinterpret_cast<const float4 *>(rec.ld + (size_t)slot * ROW);
    float ld[32], m[NB];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const float4 v = ld4[k];
        ld[4 * k] = v.x;
        ld[4 * k + 1] = v.y;
        ld[4 * k + 2] = v.z;
        ld[4 * k + 3] = v.w;
    }
#pragma unroll
    for (int c = 0; c < NB; ++c) m[c] = mo[mat.band_pos[c]];
    float ab[NB];
    if (TEX) {  // the hit's albedo texture value (shade_tex_kernel): Pow(albedo, 1 - mix) per lane
        tex_albedo_pow_all(rec.hit_alb[slot], 1.f - mat.mix, ab);
    } else {
#pragma unroll
        for (int c = 0; c < NB; ++c) ab[c] = mat.alb_1mmix[c];
    }
    float X = 0.f, Y = 0.f, Z = 0.f;
    bool nan = false;
#pragma unroll
    for (int c = 0; c < NB; ++c) {
        float L = 0.f;
        float t = (kss * m[c]) * ab[c];
        t = t < 0.f ? 0.f : t;  // Spectrum::Clamp(0, INFINITY)
        L += t;
        L += ld[c];
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
    if (nan || y < -1e-5f || __builtin_isinf(y)) X = Y = Z = 0.f;
    rec.xyz[slot] = make_float4(X, Y, Z, 0.f);
}

__global__ __launch_bounds__(256) void assemble_kernel(RenderScene sc, SampleRecs rec, int max_hits) {
    const int slot = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    const int nhits = *rec.hit_count;
    const bool in = slot < nhits && slot < max_hits;
    {
        const uint32_t hs0 = in ? rec.hit_s[slot] : 0u;
        const int mid = (int)((hs0 >> REC_MAT_SHIFT) & 0xffu);
        const int mid0 = __builtin_amdgcn_readfirstlane(mid);
        // SSS hit (bit 31, not a light) of material mid0 (with or without an albedo texture)
        const bool fast = in && (hs0 >> 31) && mid == mid0;
        if (__builtin_amdgcn_ballot_w64(in && !fast) == 0) {
            if (in) {
                if (sc.materials[mid0].has_alb_tex)
                    assemble_uniform<true>(sc, rec, slot, mid0);
                else
                    assemble_uniform<false>(sc, rec, slot, mid0);
            }
            return;
        }
    }
    if (!in) return;
    const uint32_t hs = rec.hit_s[slot];
    const float *le = nullptr, *mo = nullptr, *ld = nullptr;
    const RenderMaterial *mat = nullptr;
    float kss = 0.f, arg[3] = {0.f, 0.f, 0.f};
    bool alb = false;
    if ((hs & HS_LIGHT) && !(hs & HS_LSURF)) return;  // escaped: sky_kernel
    if (hs & HS_LIGHT) {  // a light sphere: L = 0 + Le(wo) (if it faces the ray) + Ld of its matte surface
        if (hs & HS_LE) le = sc.lights[(hs >> REC_MAT_SHIFT) & 0xffu].Lemit;
        ld = rec.ld + (size_t)slot * ROW;
    } else {
        ld = rec.ld + (size_t)slot * ROW;
        if (hs >> 31) {
            const float4 q = rec.hit_q[slot];
            mat = &sc.materials[(hs >> REC_MAT_SHIFT) & 0xffu];
            const float Ft = mat->is_mc ? 1.f : 1.f - rho_lookup(mat->rho, mat->n_rho, q.w);
            kss = kInvPiF * Ft;
            mo = reinterpret_cast<const float *>(rec.mo4 + (size_t)slot * kGroups);
            if (mat->has_alb_tex) {
                const float4 a = rec.hit_alb[slot];
                arg[0] = a.x;
                arg[1] = a.y;
                arg[2] = a.z;
                alb = true;
            }
        }
    }
    float X = 0.f, Y = 0.f, Z = 0.f;
    bool nan = false;
    for (int c = 0; c < NB; ++c) {
        float L = 0.f;
        if (le) L += le[c];
        if (mo) {
            const float ab = alb ? tex_albedo_pow(arg, c, 1.f - mat->mix) : mat->alb_1mmix[c];
            float t = (kss * mo[mat->band_pos[c]]) * ab;
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
    if (nan || y < -1e-5f || __builtin_isinf(y)) X = Y = Z = 0.f;
    rec.xyz[slot] = make_float4(X, Y, Z, 0.f);
}

// Camera rays that escaped with infinite lights in the scene (SamplerRenderer::Li,
// samplerrenderer.cpp:144-151): L = 0 + sum over lights of Le(ray), area lights adding 0; then
// the sample filter and ToXYZ as in assemble_kernel. A separate launch keeps assemble_kernel's
// registers (and occupancy) independent of the 30-band sky sum.
__global__ __launch_bounds__(256) void sky_kernel(RenderScene sc, SampleRecs rec, int max_hits) {
    const int slot = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    const int nhits = *rec.hit_count;
    if (slot >= nhits || slot >= max_hits) return;
    const uint32_t hs = rec.hit_s[slot];
    if (!((hs & HS_LIGHT) && !(hs & HS_LSURF))) return;
    const float4 hb = rec.hit_b[slot];
    float Ls[NB];
#pragma unroll
    for (int c = 0; c < NB; ++c) Ls[c] = 0.f;
    for (int l = 0; l < sc.nlights; ++l) {
        const RenderLight &Lt = sc.lights[l];
        if (!Lt.kind) continue;
        float s, t, rgb[3];
        inf_coords(Lt, V3{hb.x, hb.y, hb.z}, s, t);
        inf_lookup(Lt, s, t, rgb);
#pragma unroll
        for (int c = 0; c < NB; ++c) Ls[c] += illum_band(rgb, c);
    }
    float X = 0.f, Y = 0.f, Z = 0.f;
    bool nan = false;
#pragma unroll
    for (int c = 0; c < NB; ++c) {
        const float L = Ls[c];
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
    if (nan || y < -1e-5f || __builtin_isinf(y)) X = Y = Z = 0.f;
    rec.xyz[slot] = make_float4(X, Y, Z, 0.f);
}

__global__ __launch_bounds__(256) void film_kernel(RenderScene sc, PieceList pl, SampleRecs rec) {
    const int k = piece_of(pl, (int)blockIdx.x);
    const TileBatch &tb = pl.tb[k];
    rec.flags += pl.off[k];
    rec.slot += pl.off[k];
    rec.spill += pl.off[k] / tb.spp;
    float *__restrict__ out = pl.out[k];
    const int out_stride_px = pl.out_stride[k];
    const int i = ((int)blockIdx.x - pl.block0[k]) * blockDim.x + threadIdx.x;
    const int tw = tb.x1 - tb.x0, th = tb.y1 - tb.y0;
    if (i >= tw * th) return;
    const int px = tb.x0 + i % tw, py = tb.y0 + i / tw;
    float X = 0.f, Y = 0.f, Z = 0.f, W = 0.f;
    // own samples (always inside this pixel's filter support), then the 8 neighbours' samples
    // in row-major order whose float image position rounds onto the shared edge
    // (ImageFilm::AddSample with the 0.5-wide box filter, image.cpp:77-137). Samples that hit
    // nothing add exactly 0 to X, Y, Z (never -0), so only their weight is accumulated.
    for (int q = 0; q < 9; ++q) {
        const int dx = q == 0 ? 0 : ((q - 1 + (q > 4)) % 3) - 1;
        const int dy = q == 0 ? 0 : ((q - 1 + (q > 4)) / 3) - 1;
        const int qx = px + dx, qy = py + dy;
        if (qx < tb.ex0 || qy < tb.ey0 || qx >= tb.ex0 + tb.ew || qy >= tb.ey0 + tb.eh) continue;
        const int64_t li = (int64_t)(qy - tb.ey0) * tb.ew + (qx - tb.ex0);
        // bits the neighbour's samples need to reach this pixel
        const uint32_t need = (dx < 0 ? REC_XHI : dx > 0 ? REC_XLO : 0u) | (dy < 0 ? REC_YHI : dy > 0 ? REC_YLO : 0u);
        if (q == 0) {
            const int32_t *sl = rec.slot + li * tb.spp;
            if ((tb.spp & 7) == 0) {
                // 8 slots as two 16-byte loads: a lane's run of slots is contiguous, and the
                // vector-memory path pays per cache line an instruction touches, so one wide load
                // per line instead of four narrow ones (same slots, same order)
                const int4 *sl4 = reinterpret_cast<const int4 *>(sl);
                for (int s0 = 0; s0 < tb.spp; s0 += 8) {
                    const int4 a4 = sl4[s0 >> 2], b4 = sl4[(s0 >> 2) + 1];
                    const int32_t v[8] = {a4.x, a4.y, a4.z, a4.w, b4.x, b4.y, b4.z, b4.w};
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        if (v[k] >= 0) {
                            const float4 x = rec.xyz[v[k]];
                            X += 1.f * x.x;
                            Y += 1.f * x.y;
                            Z += 1.f * x.z;
                        }
                        W += 1.f;
                    }
                }
                continue;
            }
            for (int s0 = 0; s0 < tb.spp; s0 += 8) {
                int32_t v[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = s0 + k < tb.spp ? sl[s0 + k] : -2;
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    if (v[k] == -2) break;
                    if (v[k] >= 0) {
                        const float4 x = rec.xyz[v[k]];
                        X += 1.f * x.x;
                        Y += 1.f * x.y;
                        Z += 1.f * x.z;
                    }
                    W += 1.f;
                }
            }
            continue;
        }
        if ((rec.spill[li] & need) != need) continue;
        for (int s = 0; s < tb.spp; ++s) {
            const int64_t sid = li * tb.spp + s;
            if ((rec.flags[sid] & need) != need) continue;
            const int32_t v = rec.slot[sid];
            if (v >= 0) {
                const float4 x = rec.xyz[v];
                X += 1.f * x.x;
                Y += 1.f * x.y;
                Z += 1.f * x.z;
            }
            W += 1.f;
        }
    }
    float *o = out + ((size_t)(py - tb.y0) * out_stride_px + (px - tb.x0)) * 4;
    o[0] = X;
    o[1] = Y;
    o[2] = Z;
    o[3] = W;
}

// ------------------------------------------------------------------ Preprocess: tessellation
// TessellateSurfacePoints on the GPU (tessellate.h, the host build's code), one thread per triangle
// of one mesh: the counting pass writes each triangle's point count, the emitting pass its points
// from out[offs[base + t]] in the reference's shader order. Points therefore land in triangle order,
// as the host build and the reference (surfacepoints.cpp:328-332) emit them.
// INCENTER is a template parameter, not a kernel argument: with the centroid/incentre choice left to a
// run-time flag, this compiler (ROCm 7.2, gfx950) evaluated the incentre for the sub-triangles of one
// of tess_matching's two shader call sites (tests/test_tessellate_gpu.py caught it); with the choice
// fixed at compile time every point equals the host build's.
template <bool EMIT, bool INCENTER>
__global__ __launch_bounds__(64) void tess_kernel(RenderScene sc, int mesh, int ntri, int64_t base, float min_dist,
                                                  int64_t *counts, const int64_t *offs, SurfacePoint *out) {
    const int t = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (t >= ntri) return;
    const RenderMesh &m = sc.meshes[mesh];
    const TessTri tr = tess_tri(m.view, t, min_dist);
    if (!EMIT) {
        int64_t n = 0;
        auto shader = [&](BC, BC, BC) { ++n; };
        tessellator(tr.tfe0, tr.tfe1, tr.tfe2, tr.tfc, shader);
        counts[base + t] = n;
        return;
    }
    const RenderMaterial &mt = sc.materials[m.material];
    const TexView *bt = mt.has_bump ? &mt.bump_tex : nullptr;
    int64_t k = offs[base + t];
    auto shader = [&](BC a, BC b, BC c) {
        out[k++] = tess_point(m.view, t, tr, a, b, c, INCENTER, bt, m.material, min_dist);
    };
    tessellator(tr.tfe0, tr.tfe1, tr.tfe2, tr.tfc, shader);
}
template __global__ void tess_kernel<false, false>(RenderScene, int, int, int64_t, float, int64_t *, const int64_t *,
                                                   SurfacePoint *);
template __global__ void tess_kernel<true, false>(RenderScene, int, int, int64_t, float, int64_t *, const int64_t *,
                                                  SurfacePoint *);
template __global__ void tess_kernel<true, true>(RenderScene, int, int, int64_t, float, int64_t *, const int64_t *,
                                                 SurfacePoint *);

// ------------------------------------------------------------------ tile-cost probe
// PerspectiveCamera::GenerateRay through the pixel centre and Scene::Intersect, as primary_kernel.
__global__ __launch_bounds__(256) void probe_kernel(RenderScene sc, int x0, int x1, int y0, int y1, uint8_t *cls) {
    __shared__ int stk_all[kStack * 256];
    int *stk = stk_all + threadIdx.x;
    const int w = x1 - x0;
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= w * (y1 - y0)) return;
    const int px = x0 + i % w, py = y0 + i / w;
    const V3 pcam = xform_point(sc.raster_to_camera, V3{(float)px + 0.5f, (float)py + 0.5f, 0.f});
    const V3 o = xform_point(sc.camera_to_world, V3{0.f, 0.f, 0.f});
    const V3 d = xform_vector(sc.camera_to_world, normalize(pcam));
    const Hit h = trace_closest(sc, o, d, 0.f, INFINITY, stk, 256);
    uint8_t c = 0;
    if (h.tri >= 0) {
        const uint32_t mid = sc.meshes[sc.tri_mesh[h.tri]].material;
        c = (sc.materials[mid].has_bssrdf && sc.have_octree) ? 2 : 1;
    }
    cls[i] = c;
}

// ------------------------------------------------------------------ reference-sampler replay
// (the render tasks' streams: replay_gen.hip)

// IrradianceTask::Run's RNG(47 k) (multipolesubsurface.cpp:81, 110-112): per point of the task's
// slice and per light, scramble[0], scramble[1], compScramble
__global__ __launch_bounds__(64) void replay_irradiance_kernel(int n, int nlights, int ntasks, uint32_t *mt,
                                                               uint32_t *scr) {
    const int task = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (task >= ntasks) return;
    const int i0 = (int)((uint64_t)task * (uint64_t)n / (uint64_t)ntasks);
    const int i1 = (int)((uint64_t)(task + 1) * (uint64_t)n / (uint64_t)ntasks);
    if (i0 == i1) return;
    Mt19937 rng{mt + task, ntasks, 624};
    rng.seed((uint32_t)task * 47u);
    for (int i = i0; i < i1; ++i)
        for (int l = 0; l < nlights; ++l) {
            uint32_t *o = scr + ((size_t)i * nlights + l) * 2;
            o[0] = rng.next();
            o[1] = rng.next();
            rng.skip(1);  // compScramble (a LightSample's component: one shape per light here)
        }
}

}  // namespace mpss
