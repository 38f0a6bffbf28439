/*
 * render.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Scalar CPU restatement of the per-pixel path of MultipoleSubsurfaceIntegrator with
 * LayeredSkin: surface-point tessellation, irradiance Preprocess, camera rays, scene
 * intersection, direct lighting with MIS, the Mo() term and the box-filtered film.
 * Sample values come from the same counter-based scrambled (0,2)-sequences as the product
 * ("replay mode"), so both sides see identical sample values.
 *
 * Reference files (paths under /root/reference/src):
 *   shapes/trianglemesh.cpp:187-351   TessellateSurfacePoints / tessellator / matching
 *   shapes/trianglemesh.inl:54-135,224-346  Triangle::Intersect, GetShadingGeometry, ...
 *   shapes/sphere.cpp                 Sphere::Intersect / Sample / Pdf
 *   core/light.cpp:145-172            ShapeSet::Sample / Pdf
 *   lights/diffuse.cpp:45-87          DiffuseAreaLight::L / Sample_L / Pdf
 *   core/integrator.cpp:47-174        UniformSampleAllLights / EstimateDirect
 *   core/reflection.{h,cpp}           Microfacet, Beckmann, FresnelDielectric, BSDF::f/Sample_f/Pdf
 *   integrators/multipolesubsurface.cpp:72-152 (IrradianceTask), 253-303 (Li)
 *   renderers/samplerrenderer.cpp:100-140 (sample filter), film/image.cpp:77-137 (AddSample)
 *   cameras/perspective.cpp (GenerateRay)
 * Intersection uses its own median-split BVH: the closest hit does not depend on the tree
 * (only exact t ties between triangles could differ).
 */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "oracle.h"
#include "../data/spectral_bands.h"

#define PI_F 3.14159265358979323846f
#define INV_PI_F 0.31830988618379067154f

typedef struct { float x, y, z; } v3;

static inline v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }
static inline v3 mul(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
static inline float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline float absdot(v3 a, v3 b) { return fabsf(dot(a, b)); }
static inline float lensq(v3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
static inline float len(v3 a) { return sqrtf(lensq(a)); }
/* geometry.h: v / f multiplies by the reciprocal */
static inline v3 divf(v3 a, float f) { float inv = 1.f / f; return mk(a.x * inv, a.y * inv, a.z * inv); }
static inline v3 nrm(v3 a) { return divf(a, len(a)); }
/* geometry.h Cross: double intermediates */
static inline v3 crs(v3 a, v3 b) {
    double ax = a.x, ay = a.y, az = a.z, bx = b.x, by = b.y, bz = b.z;
    return mk((float)((ay * bz) - (az * by)), (float)((az * bx) - (ax * bz)), (float)((ax * by) - (ay * bx)));
}
static inline float dsq(v3 a, v3 b) { return lensq(sub(a, b)); }
static inline v3 ld(const float *a, int i) { return mk(a[3 * i], a[3 * i + 1], a[3 * i + 2]); }

/* transcendentals: evaluated in double, rounded once (DESIGN.md "float conventions") */
static inline float fsin(float x) { return (float)sin((double)x); }
static inline float fcos(float x) { return (float)cos((double)x); }
static inline float fexp(float x) { return (float)exp((double)x); }
static inline float flog(float x) { return (float)log((double)x); }
static inline float fatan(float x) { return (float)atan((double)x); }
static inline float fatan2(float y, float x) { return (float)atan2((double)y, (double)x); }
static inline float facos(float x) { return (float)acos((double)x); }
static inline float fpowf_(float x, float y) { return (float)pow((double)x, (double)y); }

static void coord_system(v3 v1, v3 *v2, v3 *v3o) { /* geometry.h CoordinateSystem */
    if (fabsf(v1.x) > fabsf(v1.y)) {
        float inv = 1.f / sqrtf(v1.x * v1.x + v1.z * v1.z);
        *v2 = mk(-v1.z * inv, 0.f, v1.x * inv);
    } else {
        float inv = 1.f / sqrtf(v1.y * v1.y + v1.z * v1.z);
        *v2 = mk(0.f, v1.z * inv, -v1.y * inv);
    }
    *v3o = crs(v1, *v2);
}

/* Transform::operator() on points / vectors / normals (transform.h:190-237) */
static v3 xpoint(const float *m, v3 p) {
    float xp = m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3];
    float yp = m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7];
    float zp = m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11];
    float wp = m[12] * p.x + m[13] * p.y + m[14] * p.z + m[15];
    if (wp == 1.f) return mk(xp, yp, zp);
    return divf(mk(xp, yp, zp), wp);
}
static v3 xvector(const float *m, v3 v) {
    return mk(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[4] * v.x + m[5] * v.y + m[6] * v.z,
              m[8] * v.x + m[9] * v.y + m[10] * v.z);
}
static v3 xnormal(const float *mi, v3 n) {
    return mk(mi[0] * n.x + mi[4] * n.y + mi[8] * n.z, mi[1] * n.x + mi[5] * n.y + mi[9] * n.z,
              mi[2] * n.x + mi[6] * n.y + mi[10] * n.z);
}

/* ------------------------------------------------------------------ replay-mode sampler */
static uint32_t mix32(uint32_t h) {
    h ^= h >> 16; h *= 0x7feb352du; h ^= h >> 15; h *= 0x846ca68bu; h ^= h >> 16;
    return h;
}
static uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) { return mix32(a ^ mix32(b ^ mix32(c + 0x9e3779b9u))); }
#define ONE_MINUS_EPS 0x1.fffffep-1f
static float vdc(uint32_t n, uint32_t scramble) { /* montecarlo.h VanDerCorput */
    n = (n << 16) | (n >> 16);
    n = ((n & 0x00ff00ffu) << 8) | ((n & 0xff00ff00u) >> 8);
    n = ((n & 0x0f0f0f0fu) << 4) | ((n & 0xf0f0f0f0u) >> 4);
    n = ((n & 0x33333333u) << 2) | ((n & 0xccccccccu) >> 2);
    n = ((n & 0x55555555u) << 1) | ((n & 0xaaaaaaaau) >> 1);
    n ^= scramble;
    float v = (float)((n >> 8) & 0xffffff) / (float)(1 << 24);
    return v < ONE_MINUS_EPS ? v : ONE_MINUS_EPS;
}
static float sobol(uint32_t n, uint32_t scramble) { /* montecarlo.h Sobol2 */
    for (uint32_t v = 1u << 31; n != 0; n >>= 1, v ^= v >> 1)
        if (n & 1u) scramble ^= v;
    float r = (float)((scramble >> 8) & 0xffffff) / (float)(1 << 24);
    return r < ONE_MINUS_EPS ? r : ONE_MINUS_EPS;
}
/* dimension ids of one camera sample (see DESIGN.md "replay mode") */
enum { D_IMAGE = 0, D_LIGHT_POS = 2, D_BSDF_DIR = 4, D_BSDF_COMP = 5, D_IRR_POS = 6, D_PERM = 9 };

/* ------------------------------------------------------------------ scene */
typedef struct {
    int nv, nt;
    float *P, *N, *S, *uv;
    int *idx;
    float o2w[16], w2o[16];
    int flip, material;
} o_mesh;

typedef struct {
    int kind; /* 0 sphere area light, 1 infinite light with a constant (1x1) map */
    v3 c;
    float r, phimax, thetamin, thetamax, area;
    float Le[O_NB];
    int ns_pow2;
    int replay_off;       /* first float of this light's values in a reference-sampler row */
    float l2w[9], w2l[9]; /* kind 1: LightToWorld, WorldToLight */
    o_envmap em;          /* kind 1: radiance map + Distribution2D */
} o_light;

typedef struct {
    float R[O_NB], T[O_NB], alb_mix[O_NB], alb_1mmix[O_NB];
    float mix;
    int has_alb, has_bump; /* ImageTexture "albedo" / "bumpmap" */
    o_tex alb, bump;
    float rough2, eta;
    int fixed_fresnel, is_mc, has_refl, has_trans;
    float *rho;
    int n_rho;
    float *rd;
    int L;
    float rcp[O_NB];
    int rgb; /* rgbprofile: rd rows 0..2 = R, G, B (multipole.cpp:85-107) */
    int lambert; /* the area-light sphere's default "matte" material: one Lambertian(R) BxDF */
    int no_bssrdf; /* LayeredSkin genprofile false: no MultipoleBSSRDF data (layeredskin.cpp:120-122) */
} o_mat;

typedef struct { float bmin[3], bmax[3]; int left, right, first, count; } o_bnode;

struct o_scene {
    int xres, yres;
    float r2c[16], c2w[16];
    o_mesh *meshes; int nmeshes;
    o_light *lights; int nlights;
    o_mat *mats; int nmats;
    /* flattened triangles for intersection */
    int ntris;
    int *tri_mesh, *tri_local;
    float *tp1, *te1, *te2; /* p1, e1 = p2 - p1, e2 = p3 - p1 */
    o_bnode *bvh; int nbvh;
    int *order;
    o_octree *octree;
    float max_error;
};

o_scene *o_scene_create(int xres, int yres, const float *r2c, const float *c2w) {
    o_scene *s = (o_scene *)calloc(1, sizeof(o_scene));
    s->xres = xres;
    s->yres = yres;
    memcpy(s->r2c, r2c, sizeof(s->r2c));
    memcpy(s->c2w, c2w, sizeof(s->c2w));
    return s;
}

static float *dupf(const float *a, size_t n) {
    if (!a) return NULL;
    float *r = (float *)malloc(n * sizeof(float));
    memcpy(r, a, n * sizeof(float));
    return r;
}

int o_scene_add_material(o_scene *s, const float *R, const float *T, const float *albedo, float mix,
                         float roughness, float eta, int fixed_fresnel, const float *rho, int n_rho, int is_mc,
                         const float *rd, int L, const float *rcp) {
    s->mats = (o_mat *)realloc(s->mats, (s->nmats + 1) * sizeof(o_mat));
    o_mat *m = &s->mats[s->nmats];
    memset(m, 0, sizeof(*m));
    m->has_refl = 0;
    m->has_trans = 0;
    for (int c = 0; c < O_NB; ++c) {
        m->R[c] = R[c];
        m->T[c] = T ? T[c] : 0.f;
        if (R[c] != 0.f) m->has_refl = 1;
        if (m->T[c] != 0.f) m->has_trans = 1;
        m->alb_mix[c] = fpowf_(albedo[c], mix);          /* Pow(albedo, mix): IrradianceTask */
        m->alb_1mmix[c] = fpowf_(albedo[c], 1.f - mix);  /* Pow(albedo, 1 - mix): Li */
        m->mix = mix;
        m->rcp[c] = rcp[c];
    }
    float r = roughness < 1e-3f ? 1e-3f : roughness;    /* Beckmann ctor clamps */
    m->rough2 = r * r;
    m->eta = eta;
    m->fixed_fresnel = fixed_fresnel;
    m->is_mc = is_mc;
    m->rho = dupf(rho, (size_t)n_rho);
    m->n_rho = n_rho;
    m->rd = dupf(rd, (size_t)O_NB * L);
    m->L = L;
    return s->nmats++;
}

int o_scene_set_material_rgb(o_scene *s, int material, int rgb) {
    if (material < 0 || material >= s->nmats) return -1;
    s->mats[material].rgb = rgb;
    return 0;
}

/* genprofile false (layeredskin.cpp:70,120-122): preparedBSSRDFData = NULL. Li adds no Mo() term and
 * IrradianceTask lights the material's points as points without a MultipoleBSSRDF
 * (multipolesubsurface.cpp:100-107: Ft = 1, no albedo^mix). */
int o_scene_set_material_no_bssrdf(o_scene *s, int material, int no_bssrdf) {
    if (material < 0 || material >= s->nmats) return -1;
    s->mats[material].no_bssrdf = no_bssrdf;
    return 0;
}

int o_scene_set_material_texture(o_scene *s, int material, int which, int W, int H, const float *texels,
                                 float shift, float scale, float gamma, int wrap, int trilinear, float max_aniso,
                                 float su, float sv, float du, float dv) {
    if (material < 0 || material >= s->nmats) return -1;
    o_mat *m = &s->mats[material];
    o_tex *t = which ? &m->bump : &m->alb;
    if (which ? m->has_bump : m->has_alb) o_tex_free(t);
    o_tex_build(t, W, H, texels, which, shift, scale, gamma, wrap, trilinear, max_aniso, su, sv, du, dv);
    if (which) m->has_bump = 1;
    else m->has_alb = 1;
    return 0;
}

int o_scene_add_mesh(o_scene *s, int nv, const float *P, const float *N, const float *S, const float *uv, int nt,
                     const int32_t *idx, const float *o2w, const float *w2o, int flip, int material) {
    s->meshes = (o_mesh *)realloc(s->meshes, (s->nmeshes + 1) * sizeof(o_mesh));
    o_mesh *m = &s->meshes[s->nmeshes];
    m->nv = nv;
    m->nt = nt;
    m->P = dupf(P, 3 * (size_t)nv);
    m->N = dupf(N, 3 * (size_t)nv);
    m->S = dupf(S, 3 * (size_t)nv);
    m->uv = dupf(uv, 2 * (size_t)nv);
    m->idx = (int *)malloc(3 * (size_t)nt * sizeof(int));
    memcpy(m->idx, idx, 3 * (size_t)nt * sizeof(int));
    memcpy(m->o2w, o2w, sizeof(m->o2w));
    memcpy(m->w2o, w2o, sizeof(m->w2o));
    m->flip = flip;
    m->material = material;
    return s->nmeshes++;
}

static int round_up_pow2(int v) { int r = 1; while (r < v) r <<= 1; return r; }

int o_scene_add_sphere_light(o_scene *s, const float *c, float r, const float *Le, int nsamples) {
    s->lights = (o_light *)realloc(s->lights, (s->nlights + 1) * sizeof(o_light));
    o_light *l = &s->lights[s->nlights];
    memset(l, 0, sizeof(*l));
    l->c = mk(c[0], c[1], c[2]);
    l->r = r;
    /* Sphere ctor (sphere.cpp): zmin = -r, zmax = r, phiMax = 360 degrees */
    l->phimax = (PI_F / 180.f) * 360.f;
    l->thetamin = facos(-1.f);
    l->thetamax = facos(1.f);
    l->area = l->phimax * r * (r - -r);
    memcpy(l->Le, Le, sizeof(l->Le));
    l->ns_pow2 = round_up_pow2(nsamples);
    return s->nlights++;
}

/* CreateInfiniteLight + InfiniteAreaLight ctor (lights/infinite.cpp:66-106, 180-188): L is the
 * 30-band L * scale; texels are multiplied by L.ToRGBSpectrum(), or the map is that one texel */
int o_scene_add_infinite_light(o_scene *s, const float *L, int nsamples, const float *l2w, const float *w2l, int W,
                               int H, const float *texels) {
    s->lights = (o_light *)realloc(s->lights, (s->nlights + 1) * sizeof(o_light));
    o_light *l = &s->lights[s->nlights];
    memset(l, 0, sizeof(*l));
    l->kind = 1;
    float rgb[3];
    o_to_rgb(L, rgb);
    float *t;
    if (texels) {
        t = (float *)malloc((size_t)W * H * 3 * sizeof(float));
        for (size_t i = 0; i < (size_t)W * H; ++i)
            for (int k = 0; k < 3; ++k) t[3 * i + k] = texels[3 * i + k] * rgb[k];
    } else {
        W = H = 1;
        t = (float *)malloc(3 * sizeof(float));
        memcpy(t, rgb, sizeof(rgb));
    }
    int rc = o_envmap_build(W, H, t, &l->em);
    free(t);
    if (rc) return -1;
    for (int r = 0; r < 3; ++r)
        for (int k = 0; k < 3; ++k) {
            l->l2w[3 * r + k] = l2w[4 * r + k];
            l->w2l[3 * r + k] = w2l[4 * r + k];
        }
    l->ns_pow2 = round_up_pow2(nsamples);
    return s->nlights++;
}

/* ------------------------------------------------------------------ triangle geometry */
typedef struct {
    v3 p, ng, nn, sn, tn;
    float u, v;
    v3 dpdu, dpdv;          /* dgGeom */
    v3 ss, ts, dndu, dndv;  /* dgShading's dpdu, dpdv, dndu, dndv */
} frame_t;

static void tri_uvs(const o_mesh *m, int t, float uv[3][2]) { /* TriangleBase::GetUVs */
    if (m->uv) {
        for (int k = 0; k < 3; ++k) {
            uv[k][0] = m->uv[2 * m->idx[3 * t + k]];
            uv[k][1] = m->uv[2 * m->idx[3 * t + k] + 1];
        }
    } else {
        uv[0][0] = 0.f; uv[0][1] = 0.f; uv[1][0] = 1.f; uv[1][1] = 0.f; uv[2][0] = 1.f; uv[2][1] = 1.f;
    }
}

/* dg (Intersect / GetDifferentialGeometries) + GetShadingGeometry + BSDF frame */
static frame_t tri_frame(const o_mesh *m, int t, v3 p, float b0, float b1, float b2) {
    v3 p1 = ld(m->P, m->idx[3 * t]), p2 = ld(m->P, m->idx[3 * t + 1]), p3 = ld(m->P, m->idx[3 * t + 2]);
    v3 e1 = sub(p2, p1), e2 = sub(p3, p1);
    float uv[3][2];
    tri_uvs(m, t, uv);
    float du1 = uv[0][0] - uv[2][0], du2 = uv[1][0] - uv[2][0];
    float dv1 = uv[0][1] - uv[2][1], dv2 = uv[1][1] - uv[2][1];
    v3 dp1 = sub(p1, p3), dp2 = sub(p2, p3);
    float det = du1 * dv2 - dv1 * du2;
    v3 dpdu, dpdv;
    if (det == 0.f) {
        coord_system(nrm(crs(e2, e1)), &dpdu, &dpdv);
    } else {
        float invdet = 1.f / det;
        dpdu = mul(sub(mul(dp1, dv2), mul(dp2, dv1)), invdet);
        dpdv = mul(add(mul(dp1, -du2), mul(dp2, du1)), invdet);
    }
    frame_t f;
    f.p = p;
    f.u = b0 * uv[0][0] + b1 * uv[1][0] + b2 * uv[2][0];
    f.v = b0 * uv[0][1] + b1 * uv[1][1] + b2 * uv[2][1];
    /* DifferentialGeometry ctor: nn = Normalize(Cross(dpdu, dpdv)), flipped on RO ^ SwapsHandedness */
    v3 ng = nrm(crs(dpdu, dpdv));
    if (m->flip) ng = mul(ng, -1.f);
    f.ng = ng;
    v3 ss, ts;
    f.dpdu = dpdu;
    f.dpdv = dpdv;
    f.dndu = f.dndv = mk(0.f, 0.f, 0.f);
    if (!m->N && !m->S) {
        f.nn = ng;
        ss = dpdu;
        f.ss = dpdu;
        f.ts = dpdv;
    } else {
        /* GetShadingGeometry: barycentrics of (u, v) via SolveLinearSystem2x2 */
        float b[3];
        float A[2][2] = {{uv[1][0] - uv[0][0], uv[2][0] - uv[0][0]}, {uv[1][1] - uv[0][1], uv[2][1] - uv[0][1]}};
        float C[2] = {f.u - uv[0][0], f.v - uv[0][1]};
        float d = A[0][0] * A[1][1] - A[0][1] * A[1][0];
        int ok = !(fabsf(d) < 1e-10f);
        if (ok) {
            b[1] = (A[1][1] * C[0] - A[0][1] * C[1]) / d;
            b[2] = (A[0][0] * C[1] - A[1][0] * C[0]) / d;
            if (isnan(b[1]) || isnan(b[2])) ok = 0;
        }
        if (!ok) b[0] = b[1] = b[2] = 1.f / 3.f;
        else b[0] = 1.f - b[1] - b[2];
        v3 ns;
        if (m->N) {
            v3 n0 = ld(m->N, m->idx[3 * t]), n1 = ld(m->N, m->idx[3 * t + 1]), n2 = ld(m->N, m->idx[3 * t + 2]);
            ns = nrm(xnormal(m->w2o, add(add(mul(n0, b[0]), mul(n1, b[1])), mul(n2, b[2]))));
        } else {
            ns = ng;
        }
        if (m->S) {
            v3 s0 = ld(m->S, m->idx[3 * t]), s1 = ld(m->S, m->idx[3 * t + 1]), s2 = ld(m->S, m->idx[3 * t + 2]);
            ss = nrm(xvector(m->o2w, add(add(mul(s0, b[0]), mul(s1, b[1])), mul(s2, b[2]))));
        } else {
            ss = nrm(dpdu);
        }
        ts = crs(ss, ns);
        if (lensq(ts) > 0.f) {
            ts = nrm(ts);
            ss = crs(ts, ns);
        } else {
            coord_system(ns, &ss, &ts);
        }
        v3 nn = nrm(crs(ss, ts));
        if (m->flip) nn = mul(nn, -1.f);
        f.nn = nn;
        f.ss = ss;
        f.ts = ts;
        if (m->N && det != 0.f) { /* trianglemesh.inl:269-295, then ObjectToWorld(Normal) */
            v3 n0 = ld(m->N, m->idx[3 * t]), n1 = ld(m->N, m->idx[3 * t + 1]), n2 = ld(m->N, m->idx[3 * t + 2]);
            v3 dn1 = sub(n0, n2), dn2 = sub(n1, n2);
            float invdet = 1.f / det;
            f.dndu = xnormal(m->w2o, mul(sub(mul(dn1, dv2), mul(dn2, dv1)), invdet));
            f.dndv = xnormal(m->w2o, mul(add(mul(dn1, -du2), mul(dn2, du1)), invdet));
        }
    }
    f.sn = nrm(ss);
    f.tn = crs(f.nn, f.sn);
    return f;
}

/* ------------------------------------------------------------------ textures on the surface */
/* DifferentialGeometry::ComputeDifferentials (diffgeom.cpp:58-111) for the offset rays
 * (rxOrigin = ryOrigin = o, directions rxd, ryd): dudx, dvdx, dudy, dvdy into g[2..5] */
static int solve22(const float A[2][2], const float B[2], float *x0, float *x1) { /* SolveLinearSystem2x2 */
    float det = A[0][0] * A[1][1] - A[0][1] * A[1][0];
    if (fabsf(det) < 1e-10f) return 0;
    *x0 = (A[1][1] * B[0] - A[0][1] * B[1]) / det;
    *x1 = (A[0][0] * B[1] - A[1][0] * B[0]) / det;
    if (isnan(*x0) || isnan(*x1)) return 0;
    return 1;
}
static float comp(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
static void differentials(v3 p, v3 nn, v3 dpdu, v3 dpdv, v3 o, v3 rxd, v3 ryd, float g[6]) {
    g[2] = g[3] = g[4] = g[5] = 0.f;
    float d = -dot(nn, p);
    float tx = -(dot(nn, o) + d) / dot(nn, rxd);
    if (isnan(tx)) return;
    v3 px = add(o, mul(rxd, tx));
    float ty = -(dot(nn, o) + d) / dot(nn, ryd);
    if (isnan(ty)) return;
    v3 py = add(o, mul(ryd, ty));
    int a0, a1;
    if (fabsf(nn.x) > fabsf(nn.y) && fabsf(nn.x) > fabsf(nn.z)) { a0 = 1; a1 = 2; }
    else if (fabsf(nn.y) > fabsf(nn.z)) { a0 = 0; a1 = 2; }
    else { a0 = 0; a1 = 1; }
    float A[2][2] = {{comp(dpdu, a0), comp(dpdv, a0)}, {comp(dpdu, a1), comp(dpdv, a1)}};
    float Bx[2] = {comp(px, a0) - comp(p, a0), comp(px, a1) - comp(p, a1)};
    float By[2] = {comp(py, a0) - comp(p, a0), comp(py, a1) - comp(p, a1)};
    if (!solve22(A, Bx, &g[2], &g[3])) g[2] = g[3] = 0.f;
    if (!solve22(A, By, &g[4], &g[5])) g[4] = g[5] = 0.f;
}

static float tex1(const o_tex *t, const float g[6]) {
    float x[3];
    o_tex_eval(t, g[0], g[1], g[2], g[3], g[4], g[5], x);
    return x[0];
}

/* Material::Bump (material.cpp:47-104, this fork's central differences); g = u, v, dudx, dvdx,
 * dudy, dvdy of dgs; returns the bumped dpdu and (faceforwarded to ng) nn */
static void bump(const o_tex *t, const float g[6], const frame_t *f, v3 nn_s, v3 ng, int flip, v3 *dpdu_b,
                 v3 *nn_b) {
    float e[6];
    memcpy(e, g, sizeof(e));
    float du = fabsf(g[2]) + fabsf(g[4]);
    if (du == 0.f) du = .01f;
    e[0] = g[0] + du;
    float upD = tex1(t, e);
    float dv = fabsf(g[3]) + fabsf(g[5]);
    if (dv == 0.f) dv = .01f;
    e[0] = g[0];
    e[1] = g[1] + dv;
    float vpD = tex1(t, e);
    float disp = tex1(t, g);
    du = -du;
    e[0] = g[0] + du; /* e[1] stays v + dv, as dgEval.v does */
    float unD = tex1(t, e);
    dv = -dv;
    e[0] = g[0];
    e[1] = g[1] + dv;
    float vnD = tex1(t, e);
    *dpdu_b = add(add(f->ss, mul(nn_s, (upD - unD) / (2 * du))), mul(f->dndu, disp));
    v3 dpdv_b = add(add(f->ts, mul(nn_s, (vpD - vnD) / (2 * dv))), mul(f->dndv, disp));
    v3 n = nrm(crs(*dpdu_b, dpdv_b));
    if (flip) n = mul(n, -1.f);
    *nn_b = dot(n, ng) < 0.f ? neg(n) : n;
}

/* Pow(FromRGB(albedo lookup), e) */
static void albedo_pow(const o_tex *t, const float g[6], float e, float out[O_NB]) {
    float rgb[3], spec[O_NB];
    o_tex_eval(t, g[0], g[1], g[2], g[3], g[4], g[5], rgb);
    o_from_rgb(rgb, 0, spec);
    for (int c = 0; c < O_NB; ++c) out[c] = fpowf_(spec[c], e);
}

/* Triangle::Intersect ray test */
static int tri_hit(v3 o, v3 d, float mint, float maxt, v3 p1, v3 e1, v3 e2, float *tt, float *bb1, float *bb2) {
    v3 s1 = crs(d, e2);
    float divisor = dot(s1, e1);
    if (divisor == 0.f) return 0;
    float inv = 1.f / divisor;
    v3 dd = sub(o, p1);
    float b1 = dot(dd, s1) * inv;
    if (b1 < 0.f || b1 > 1.f) return 0;
    v3 s2 = crs(dd, e1);
    float b2 = dot(d, s2) * inv;
    if (b2 < 0.f || b1 + b2 > 1.f) return 0;
    float t = dot(e2, s2) * inv;
    if (t < mint || t > maxt) return 0;
    *tt = t; *bb1 = b1; *bb2 = b2;
    return 1;
}

/* ------------------------------------------------------------------ sphere light */
static int quad(float A, float B, float C, float *t0, float *t1) { /* pbrt.h Quadratic */
    float disc = B * B - 4.f * A * C;
    if (disc < 0.f) return 0;
    float rd = sqrtf(disc);
    float q = (B < 0.f) ? -.5f * (B - rd) : -.5f * (B + rd);
    *t0 = q / A;
    *t1 = C / q;
    if (*t0 > *t1) { float x = *t0; *t0 = *t1; *t1 = x; }
    return 1;
}

static int sphere_hit(const o_light *s, v3 o, v3 d, float mint, float maxt, float *thit, v3 *nn) {
    v3 ro = sub(o, s->c); /* WorldToObject of a translation */
    float A = d.x * d.x + d.y * d.y + d.z * d.z;
    float B = 2 * (d.x * ro.x + d.y * ro.y + d.z * ro.z);
    float C = ro.x * ro.x + ro.y * ro.y + ro.z * ro.z - s->r * s->r;
    float t0, t1;
    if (!quad(A, B, C, &t0, &t1)) return 0;
    if (t0 > maxt || t1 < mint) return 0;
    float th = t0;
    if (t0 < mint) {
        th = t1;
        if (th > maxt) return 0;
    }
    v3 ph = add(ro, mul(d, th));
    if (ph.x == 0.f && ph.y == 0.f) ph.x = 1e-5f * s->r;
    float phi = fatan2(ph.y, ph.x);
    if (phi < 0.f) phi += 2.f * PI_F;
    if (phi > s->phimax) {
        if (th == t1) return 0;
        if (t1 > maxt) return 0;
        th = t1;
        ph = add(ro, mul(d, th));
        if (ph.x == 0.f && ph.y == 0.f) ph.x = 1e-5f * s->r;
        phi = fatan2(ph.y, ph.x);
        if (phi < 0.f) phi += 2.f * PI_F;
        if (phi > s->phimax) return 0;
    }
    if (nn) {
        float cz = ph.z / s->r;
        float theta = facos(cz < -1.f ? -1.f : (cz > 1.f ? 1.f : cz));
        float zr = sqrtf(ph.x * ph.x + ph.y * ph.y);
        float izr = 1.f / zr;
        float cphi = ph.x * izr, sphi = ph.y * izr;
        v3 dpdu = mk(-s->phimax * ph.y, s->phimax * ph.x, 0.f);
        v3 dpdv = mul(mk(ph.z * cphi, ph.z * sphi, -s->r * fsin(theta)), s->thetamax - s->thetamin);
        *nn = nrm(crs(dpdu, dpdv));
    }
    *thit = th;
    return 1;
}

static v3 sample_sphere_uniform(float u1, float u2) { /* montecarlo.cpp UniformSampleSphere */
    float z = 1.f - 2.f * u1;
    float r = sqrtf(fmaxf(0.f, 1.f - z * z));
    float phi = 2.f * PI_F * u2;
    return mk(r * fcos(phi), r * fsin(phi), z);
}

static v3 sample_cone(float u1, float u2, float ctmax, v3 x, v3 y, v3 z) { /* UniformSampleCone(frame) */
    float ct = (1.f - u1) * ctmax + u1 * 1.f;
    float st = sqrtf(1.f - ct * ct);
    float phi = u2 * 2.f * PI_F;
    return add(add(mul(x, fcos(phi) * st), mul(y, fsin(phi) * st)), mul(z, ct));
}

/* Sphere::Sample(p, u1, u2, &ns) + ShapeSet::Sample re-intersection; returns point, normal */
static v3 light_sample_point(const o_light *s, v3 p, float u1, float u2, v3 *ns) {
    v3 pc = s->c;
    v3 wc = nrm(sub(pc, p)), wcx, wcy;
    coord_system(wc, &wcx, &wcy);
    v3 ps;
    if (dsq(p, pc) - s->r * s->r < 1e-4f) {
        v3 q = mul(sample_sphere_uniform(u1, u2), s->r);
        *ns = nrm(q);
        ps = add(q, pc);
    } else {
        float st2 = s->r * s->r / dsq(p, pc);
        float ctmax = sqrtf(fmaxf(0.f, 1.f - st2));
        v3 rd = sample_cone(u1, u2, ctmax, wcx, wcy, wc);
        float th;
        if (!sphere_hit(s, p, rd, 1e-3f, INFINITY, &th, NULL)) th = dot(sub(pc, p), nrm(rd));
        ps = add(p, mul(rd, th));
        *ns = nrm(sub(ps, pc));
    }
    v3 rd2 = sub(ps, p);
    float th2 = 1.f;
    v3 nn2;
    if (sphere_hit(s, p, rd2, 1e-3f, INFINITY, &th2, &nn2)) *ns = nn2;
    return add(p, mul(rd2, th2));
}

static float light_pdf(const o_light *s, v3 p, v3 wi) { /* ShapeSet::Pdf of one Sphere */
    float pdf;
    if (dsq(p, s->c) - s->r * s->r < 1e-4f) {
        float th;
        v3 nn;
        if (!sphere_hit(s, p, wi, 1e-3f, INFINITY, &th, &nn)) pdf = 0.f;
        else {
            pdf = dsq(p, add(p, mul(wi, th))) / (absdot(nn, neg(wi)) * s->area);
            if (isinf(pdf)) pdf = 0.f;
        }
    } else {
        float st2 = s->r * s->r / dsq(p, s->c);
        float ctmax = sqrtf(fmaxf(0.f, 1.f - st2));
        pdf = 1.f / (2.f * PI_F * (1.f - ctmax));
    }
    return (0.f + s->area * pdf) / s->area;
}

/* ------------------------------------------------------------------ infinite light */
static v3 xvec3(const float *m, v3 v) { /* Transform::operator()(Vector), transform.h:215-220 */
    return mk(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[3] * v.x + m[4] * v.y + m[5] * v.z,
              m[6] * v.x + m[7] * v.y + m[8] * v.z);
}

/* Spectrum(radianceMap->Lookup(s, t), SPECTRUM_ILLUMINANT) */
static void inf_le(const o_light *L, float s, float t, float out[O_NB]) {
    float rgb[3];
    o_envmap_lookup(&L->em, s, t, rgb);
    o_from_rgb(rgb, 1, out);
}

/* InfiniteAreaLight::Le (infinite.cpp:115-120) */
static void inf_le_dir(const o_light *L, v3 d, float out[O_NB]) {
    v3 wh = nrm(xvec3(L->w2l, d));
    float z = wh.z < -1.f ? -1.f : (wh.z > 1.f ? 1.f : wh.z);
    float theta = facos(z);
    float phi = fatan2(wh.y, wh.x);
    if (phi < 0.f) phi = phi + 2 * PI_F;
    inf_le(L, phi * 0.15915494309189533577f, theta * INV_PI_F, out);
}

static int black(const float *x) {
    for (int c = 0; c < O_NB; ++c)
        if (x[c] != 0.f) return 0;
    return 1;
}

/* InfiniteAreaLight::Pdf (infinite.cpp:222-232) */
static float inf_pdf(const o_light *L, v3 w) {
    v3 wi = xvec3(L->w2l, w);
    float z = wi.z < -1.f ? -1.f : (wi.z > 1.f ? 1.f : wi.z);
    float theta = facos(z);
    float phi = fatan2(wi.y, wi.x);
    if (phi < 0.f) phi = phi + 2 * PI_F;
    float sintheta = fsin(theta);
    if (sintheta == 0.f) return 0.f;
    float p = o_envmap_pdf(&L->em, phi * 0.15915494309189533577f, theta * INV_PI_F) / (2.f * PI_F * PI_F * sintheta);
    return p;
}

/* Sample_L of either light kind: wi, pdf, shadow ray, radiance non-black flag, and for the
 * infinite light the radiance itself */
typedef struct { v3 wi, so, sd; float pdf, smint, smaxt; int nonblack; float Li[O_NB]; } lsamp;

/* InfiniteAreaLight::Sample_L (infinite.cpp:195-218) + VisibilityTester::SetRay */
static lsamp inf_sample(const o_light *L, v3 p, float peps, float u0, float u1) {
    lsamp r;
    memset(&r, 0, sizeof(r));
    float uv[2], mapPdf;
    o_envmap_sample(&L->em, u0, u1, uv, &mapPdf);
    if (mapPdf == 0.f) return r; /* "return 0.f": black, nothing contributes */
    float theta = uv[1] * PI_F, phi = uv[0] * 2.f * PI_F;
    float costheta = fcos(theta), sintheta = fsin(theta);
    float sinphi = fsin(phi), cosphi = fcos(phi);
    r.wi = xvec3(L->l2w, mk(sintheta * cosphi, sintheta * sinphi, costheta));
    r.pdf = mapPdf / (2.f * PI_F * PI_F * sintheta);
    if (sintheta == 0.f) r.pdf = 0.f;
    r.so = p;
    r.sd = r.wi;
    r.smint = peps;
    r.smaxt = INFINITY;
    inf_le(L, uv[0], uv[1], r.Li);
    r.nonblack = !black(r.Li);
    return r;
}

/* DiffuseAreaLight::Sample_L: wi, pdf, shadow segment, radiance non-black flag */
static lsamp light_sample(const o_light *L, v3 p, float peps, float u0, float u1) {
    if (L->kind) return inf_sample(L, p, peps, u0, u1);
    lsamp r;
    v3 ns;
    v3 ps = light_sample_point(L, p, u0, u1, &ns);
    r.wi = nrm(sub(ps, p));
    r.pdf = light_pdf(L, p, r.wi);
    float dist = len(sub(p, ps));
    r.so = p;
    r.sd = divf(sub(ps, p), dist);
    r.smint = peps;
    r.smaxt = dist * (1.f - 1e-3f);
    r.nonblack = dot(ns, neg(r.wi)) > 0.f;
    memcpy(r.Li, L->Le, sizeof(r.Li));
    return r;
}

/* ------------------------------------------------------------------ microfacet BSDF */
static float beck_D(float r2, v3 wh) {
    float ct = fabsf(wh.z), c2 = ct * ct, d = c2 * c2 * PI_F;
    if (d == 0.f) return 0.f;
    float irr = 1 / r2;
    float e = (c2 - 1) * irr / c2;
    return irr * fexp(e) / d;
}
static float fresnel(float cosi, float eta_i, float eta_t, int fixed) {
    cosi = cosi < -1.f ? -1.f : (cosi > 1.f ? 1.f : cosi);
    float ei = eta_i, et = eta_t;
    if (!(cosi > 0.f)) { ei = eta_t; et = eta_i; }
    float x = 1.f - cosi * cosi;
    float sint = ei / et * sqrtf(x > 0.f ? x : 0.f);
    float F;
    if (sint >= 1.f) F = 1.f;
    else {
        float y = 1.f - sint * sint;
        float cost = sqrtf(y > 0.f ? y : 0.f);
        float ci = fabsf(cosi);
        float par = ((et * ci) - (ei * cost)) / ((et * ci) + (ei * cost));
        float per = ((ei * ci) - (et * cost)) / ((ei * ci) + (et * cost));
        F = (par * par + per * per) / 2.f;
    }
    if (fixed) F = F + F * (1.f - F) * (1.f - F);
    return F;
}
static float geomG(v3 wo, v3 wi, v3 wh) {
    float a = fabsf(wh.z), wowh = absdot(wo, wh);
    float g1 = 2.f * a * fabsf(wo.z) / wowh, g2 = 2.f * a * fabsf(wi.z) / wowh;
    float m = g2 < g1 ? g2 : g1; /* std::min(g1, g2) */
    return m < 1.f ? m : 1.f;    /* std::min(1.f, m) */
}
/* Microfacet::f per band: R * D * G * F / (4 cos_i cos_o); returns 0 if the lobe is zero */
static int mf_f(const o_mat *m, v3 wo, v3 wi, float f[O_NB]) {
    float co = fabsf(wo.z), ci = fabsf(wi.z);
    if (ci == 0.f || co == 0.f) return 0;
    v3 wh = add(wi, wo);
    if (wh.x == 0.f && wh.y == 0.f && wh.z == 0.f) return 0;
    wh = nrm(wh);
    float F = fresnel(dot(wi, wh), 1.f, m->eta, m->fixed_fresnel);
    float D = beck_D(m->rough2, wh), G = geomG(wo, wi, wh), den = 4.f * ci * co;
    for (int c = 0; c < O_NB; ++c) f[c] = m->R[c] * D * G * F / den;
    return 1;
}
static float mf_pdf(const o_mat *m, v3 wo, v3 wi) {
    if (!(wo.z * wi.z > 0.f)) return 0.f;
    v3 wh = nrm(add(wo, wi));
    float ct = fabsf(wh.z);
    float p = beck_D(m->rough2, wh) * ct / (4.f * dot(wo, wh));
    if (dot(wo, wh) <= 0.f || p < 1e-20f) p = 0.f;
    return p;
}
static void mf_sample(const o_mat *m, v3 wo, float u1, float u2, v3 *wi, float *pdf) {
    float theta = fatan(sqrtf(-m->rough2 * flog(1.f - u1)));
    float ct = fcos(theta), st = fsin(theta);
    float phi = u2 * 2.f * PI_F;
    v3 wh = mk(st * fcos(phi), st * fsin(phi), ct);
    if (!(wo.z * wh.z > 0.f)) wh = neg(wh);
    float dw = dot(wo, wh);
    *wi = add(neg(wo), mul(wh, 2.f * dw));
    float p = beck_D(m->rough2, wh) * ct / (4.f * dot(wo, wh));
    if (dot(wo, wh) <= 0.f || p < 1e-20f) p = 0.f;
    *pdf = p;
}
static v3 to_local(const frame_t *f, v3 v) { return mk(dot(v, f->sn), dot(v, f->tn), dot(v, f->nn)); }
static v3 to_world(const frame_t *f, v3 v) {
    return mk(f->sn.x * v.x + f->tn.x * v.y + f->nn.x * v.z, f->sn.y * v.x + f->tn.y * v.y + f->nn.y * v.z,
              f->sn.z * v.x + f->tn.z * v.y + f->nn.z * v.z);
}
/* MicrofacetTransmission (reflection.cpp:242-281, 405-459) with Beckmann + (Fixed)FresnelDielectric */
static float beck_pdf_raw(float r2, v3 wo, v3 wi) { /* Beckmann::Pdf */
    v3 wh = nrm(add(wo, wi));
    float ct = fabsf(wh.z);
    float p = beck_D(r2, wh) * ct / (4.f * dot(wo, wh));
    if (dot(wo, wh) <= 0.f || p < 1e-20f) p = 0.f;
    return p;
}
static float mtG(v3 wo, v3 wi, v3 wh) {
    float nh = fabsf(wh.z), no = fabsf(wo.z), ni = fabsf(wi.z), oh = absdot(wo, wh), ih = absdot(wi, wh);
    float a = 2.f * nh * no / oh, b = 2.f * nh * ni / ih;
    float mm = b < a ? b : a;
    return mm < 1.f ? mm : 1.f;
}
static int mt_f(const o_mat *m, v3 wo, v3 wi, float f[O_NB]) {
    float ci = fabsf(wi.z), co = fabsf(wo.z);
    if (ci == 0.f || co == 0.f) return 0;
    int entering = wo.z > 0.f;
    float et = entering ? m->eta : 1.f / m->eta;
    v3 wh = neg(add(wo, mul(wi, et)));
    float den = lensq(wh);
    if (den == 0.f) return 0;
    wh = nrm(wh);
    float chi = dot(wi, wh), cho = dot(wo, wh);
    if (chi == 0.f || cho == 0.f) return 0;
    float F = fresnel(entering ? fabsf(cho) : -fabsf(cho), 1.f, m->eta, m->fixed_fresnel);
    float s = fabsf(chi * cho) * et * et * beck_D(m->rough2, wh) * mtG(wo, wi, wh) / (ci * co * den);
    for (int c = 0; c < O_NB; ++c) f[c] = (m->T[c] * s) * (1.f - F);
    return 1;
}
static float mt_pdf(const o_mat *m, v3 wo, v3 wi) {
    if (wo.z * wi.z > 0.f) return 0.f;
    int entering = wo.z > 0.f;
    float et = entering ? m->eta : 1.f / m->eta;
    v3 wh = neg(add(wo, mul(wi, et)));
    if (wh.x == 0.f && wh.y == 0.f && wh.z == 0.f) return 0.f;
    float den = lensq(wh);
    wh = nrm(wh);
    v3 wir = add(neg(wo), mul(wh, 2.f * dot(wo, wh)));
    float pdf = beck_pdf_raw(m->rough2, wo, wir);
    float cosi = dot(wo, wh);
    pdf *= 4 * cosi * cosi * et * et / den;
    return pdf;
}
/* ConcentricSampleDisk (montecarlo.cpp:306-348); theta *= M_PI / 4.f is a double product */
static void concentric_disk(float u1, float u2, float *dx, float *dy) {
    float r, theta;
    float sx = 2 * u1 - 1, sy = 2 * u2 - 1;
    if (sx == 0.0 && sy == 0.0) { *dx = 0.f; *dy = 0.f; return; }
    if (sx >= -sy) {
        if (sx > sy) { r = sx; theta = sy > 0.0 ? sy / r : 8.0f + sy / r; }
        else { r = sy; theta = 2.0f - sx / r; }
    } else {
        if (sx <= sy) { r = -sx; theta = 4.0f - sy / r; }
        else { r = -sy; theta = 6.0f + sx / r; }
    }
    theta = (float)((double)theta * (3.14159265358979323846 / 4.0));
    *dx = r * fcos(theta);
    *dy = r * fsin(theta);
}
/* Lambertian::f = R * INV_PI; BxDF::Pdf: SameHemisphere ? AbsCosTheta(wi) * INV_PI : 0;
 * BxDF::Sample_f: CosineSampleHemisphere (montecarlo.h:128-133), z flipped to wo's side
 * (reflection.h, reflection.cpp:566-578) */
static float lambert_pdf(v3 wo, v3 wi) { return wo.z * wi.z > 0.f ? fabsf(wi.z) * INV_PI_F : 0.f; }
static void lambert_sample(v3 wo, float u1, float u2, v3 *wi, float *pdf) {
    float x, y;
    concentric_disk(u1, u2, &x, &y);
    *wi = mk(x, y, sqrtf(fmaxf(0.f, 1.f - x * x - y * y)));
    if (wo.z < 0.f) wi->z *= -1.f;
    *pdf = lambert_pdf(wo, *wi);
}
static void mf_sample(const o_mat *m, v3 wo, float u1, float u2, v3 *wi, float *pdf);
static void mt_sample(const o_mat *m, v3 wo, float u1, float u2, v3 *wi, float *pdf) {
    mf_sample(m, wo, u1, u2, wi, pdf);
    int entering = wo.z > 0.f;
    float et = entering ? m->eta : 1.f / m->eta;
    v3 wh = add(wo, *wi);
    if (wh.x == 0.f && wh.y == 0.f && wh.z == 0.f) return;
    wh = nrm(wh);
    float cosi = dot(wo, wh);
    float sini2 = fmaxf(0.f, 1.f - cosi * cosi);
    float eta = 1.f / et;
    float sint2 = eta * eta * sini2;
    if (sint2 >= 1.f) { *pdf = 0.f; return; }
    float cost = sqrtf(fmaxf(0.f, 1.f - sint2));
    *wi = add(mul(wo, -eta), mul(wh, eta * cosi - cost));
    float den = lensq(add(wo, mul(*wi, et)));
    if (den == 0.f) { *pdf = 0.f; return; }
    *pdf *= 4 * cosi * cosi * et * et / den;
}

/* BSDF::f with the ng hemisphere test: BRDFs on the reflection side, BTDFs on the other.
 * wol / wil are the local-frame directions the BxDF sees (BSDF::Sample_f keeps the sampled
 * local wi rather than re-projecting the world one). */
static int bsdf_f(const o_mat *m, const frame_t *fr, v3 woW, v3 wiW, v3 wol, v3 wil, float f[O_NB]) {
    int ok;
    if (m->lambert) { /* one BRDF: f = 0 + R * INV_PI on the reflection side */
        if (!(dot(wiW, fr->ng) * dot(woW, fr->ng) > 0.f)) return 0;
        for (int c = 0; c < O_NB; ++c) f[c] = 0.f + m->R[c] * INV_PI_F;
        ok = 1;
    } else if (dot(wiW, fr->ng) * dot(woW, fr->ng) > 0.f)
        ok = m->has_refl && mf_f(m, wol, wil, f);
    else
        ok = m->has_trans && mt_f(m, wol, wil, f);
    if (!ok) return 0;
    for (int c = 0; c < O_NB; ++c)
        if (f[c] != 0.f) return 1;
    return 0;
}

/* BSDF::Pdf (reflection.cpp:736-751): mean over the matching lobes, R then T */
static float bsdf_pdf(const o_mat *m, v3 wo, v3 wi) {
    int n = m->has_refl + m->has_trans;
    if (n == 0) return 0.f;
    float pdf = 0.f;
    if (m->lambert) pdf += lambert_pdf(wo, wi);
    else if (m->has_refl) pdf += mf_pdf(m, wo, wi);
    if (m->has_trans) pdf += mt_pdf(m, wo, wi);
    return pdf / (float)n;
}
static float power_h(float fp, float gp) { float f = 1 * fp, g = 1 * gp; return (f * f) / (f * f + g * g); }

static float rho_at(const o_mat *m, float ct) { /* MultipoleBSSRDFData rho lookup (multipole.cpp:458-463) */
    float fid = ct * (float)(m->n_rho - 1);
    int id = (int)fid;
    id = id < 0 ? 0 : (id > m->n_rho - 2 ? m->n_rho - 2 : id);
    float t = fid - (float)id;
    return (1.f - t) * m->rho[id] + t * m->rho[id + 1];
}

/* ------------------------------------------------------------------ BVH (own median split) */
static int bvh_build_rec(o_scene *s, int lo, int hi, float *cent) {
    int id = s->nbvh++;
    o_bnode *n = &s->bvh[id];
    float bmin[3] = {INFINITY, INFINITY, INFINITY}, bmax[3] = {-INFINITY, -INFINITY, -INFINITY};
    float cmin[3] = {INFINITY, INFINITY, INFINITY}, cmax[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = lo; i < hi; ++i) {
        int t = s->order[i];
        for (int k = 0; k < 3; ++k) {
            float a = s->tp1[3 * t + k], b = a + s->te1[3 * t + k], c = a + s->te2[3 * t + k];
            float mn = fminf(a, fminf(b, c)), mx = fmaxf(a, fmaxf(b, c));
            /* the vertex positions themselves (p1 + e1 may round): widen by the mesh values */
            bmin[k] = fminf(bmin[k], mn);
            bmax[k] = fmaxf(bmax[k], mx);
            cmin[k] = fminf(cmin[k], cent[3 * t + k]);
            cmax[k] = fmaxf(cmax[k], cent[3 * t + k]);
        }
    }
    for (int k = 0; k < 3; ++k) {
        float pad = (bmax[k] - bmin[k]) * 1e-5f + 1e-7f;
        s->bvh[id].bmin[k] = bmin[k] - pad;
        s->bvh[id].bmax[k] = bmax[k] + pad;
    }
    if (hi - lo <= 4) {
        n->left = n->right = -1;
        n->first = lo;
        n->count = hi - lo;
        return id;
    }
    int ax = 0;
    for (int k = 1; k < 3; ++k)
        if (cmax[k] - cmin[k] > cmax[ax] - cmin[ax]) ax = k;
    int mid = (lo + hi) / 2;
    /* nth_element by centroid on axis: simple insertion-free quickselect */
    int l = lo, r = hi - 1;
    while (l < r) {
        float piv = cent[3 * s->order[(l + r) / 2] + ax];
        int i = l, j = r;
        while (i <= j) {
            while (cent[3 * s->order[i] + ax] < piv) ++i;
            while (cent[3 * s->order[j] + ax] > piv) --j;
            if (i <= j) { int x = s->order[i]; s->order[i] = s->order[j]; s->order[j] = x; ++i; --j; }
        }
        if (mid <= j) r = j;
        else if (mid >= i) l = i;
        else break;
    }
    int left = bvh_build_rec(s, lo, mid, cent);
    int right = bvh_build_rec(s, mid, hi, cent);
    s->bvh[id].left = left;
    s->bvh[id].right = right;
    s->bvh[id].count = 0;
    return id;
}

static void scene_prepare(o_scene *s) {
    if (s->bvh) return;
    int nt = 0;
    for (int m = 0; m < s->nmeshes; ++m) nt += s->meshes[m].nt;
    s->ntris = nt;
    s->tri_mesh = (int *)malloc(nt * sizeof(int));
    s->tri_local = (int *)malloc(nt * sizeof(int));
    s->tp1 = (float *)malloc(3 * (size_t)nt * sizeof(float));
    s->te1 = (float *)malloc(3 * (size_t)nt * sizeof(float));
    s->te2 = (float *)malloc(3 * (size_t)nt * sizeof(float));
    float *cent = (float *)malloc(3 * (size_t)nt * sizeof(float));
    int g = 0;
    for (int mi = 0; mi < s->nmeshes; ++mi) {
        const o_mesh *m = &s->meshes[mi];
        for (int t = 0; t < m->nt; ++t, ++g) {
            v3 p1 = ld(m->P, m->idx[3 * t]), p2 = ld(m->P, m->idx[3 * t + 1]), p3 = ld(m->P, m->idx[3 * t + 2]);
            v3 e1 = sub(p2, p1), e2 = sub(p3, p1);
            s->tri_mesh[g] = mi;
            s->tri_local[g] = t;
            memcpy(&s->tp1[3 * g], &p1, 12);
            memcpy(&s->te1[3 * g], &e1, 12);
            memcpy(&s->te2[3 * g], &e2, 12);
            cent[3 * g] = (p1.x + p2.x + p3.x) / 3.f;
            cent[3 * g + 1] = (p1.y + p2.y + p3.y) / 3.f;
            cent[3 * g + 2] = (p1.z + p2.z + p3.z) / 3.f;
        }
    }
    s->order = (int *)malloc(nt * sizeof(int));
    for (int i = 0; i < nt; ++i) s->order[i] = i;
    s->bvh = (o_bnode *)malloc((2 * (size_t)nt + 1) * sizeof(o_bnode));
    s->nbvh = 0;
    bvh_build_rec(s, 0, nt, cent);
    free(cent);
}

static int box_hit(const o_bnode *n, v3 o, v3 inv, float mint, float maxt) {
    float t0 = mint, t1 = maxt;
    const float oo[3] = {o.x, o.y, o.z}, ii[3] = {inv.x, inv.y, inv.z};
    for (int k = 0; k < 3; ++k) {
        float a = (n->bmin[k] - oo[k]) * ii[k], b = (n->bmax[k] - oo[k]) * ii[k];
        if (a > b) { float x = a; a = b; b = x; }
        if (a != a || b != b) continue; /* 0 * inf: axis-parallel ray inside the slab */
        t0 = a > t0 ? a : t0;
        t1 = b < t1 ? b : t1;
        if (t0 > t1) return 0;
    }
    return 1;
}

typedef struct { float t, b1, b2; int tri; v3 lnn; } hit_t; /* tri >= 0 mesh, -1-l light, INT_MIN miss */
#define NO_HIT (-2147483647 - 1)

static hit_t intersect(const o_scene *s, v3 o, v3 d, float mint, float maxt) {
    hit_t h;
    h.tri = NO_HIT;
    h.t = maxt;
    v3 inv = mk(1.f / d.x, 1.f / d.y, 1.f / d.z);
    int stack[128], sp = 0;
    stack[sp++] = 0;
    while (sp) {
        const o_bnode *n = &s->bvh[stack[--sp]];
        if (!box_hit(n, o, inv, mint, h.t)) continue;
        if (n->left < 0) {
            for (int i = 0; i < n->count; ++i) {
                int t = s->order[n->first + i];
                float tt, b1, b2;
                if (tri_hit(o, d, mint, h.t, ld(s->tp1, t), ld(s->te1, t), ld(s->te2, t), &tt, &b1, &b2)) {
                    h.t = tt; h.b1 = b1; h.b2 = b2; h.tri = t;
                }
            }
        } else {
            stack[sp++] = n->right;
            stack[sp++] = n->left;
        }
    }
    for (int l = 0; l < s->nlights; ++l) {
        float t;
        v3 nn;
        if (s->lights[l].kind) continue;
        if (sphere_hit(&s->lights[l], o, d, mint, h.t, &t, &nn)) {
            h.t = t;
            h.tri = -1 - l;
            h.lnn = nn;
        }
    }
    return h;
}

static int occluded(const o_scene *s, v3 o, v3 d, float mint, float maxt) {
    for (int l = 0; l < s->nlights; ++l) {
        float t;
        if (!s->lights[l].kind && sphere_hit(&s->lights[l], o, d, mint, maxt, &t, NULL)) return 1;
    }
    v3 inv = mk(1.f / d.x, 1.f / d.y, 1.f / d.z);
    int stack[128], sp = 0;
    stack[sp++] = 0;
    while (sp) {
        const o_bnode *n = &s->bvh[stack[--sp]];
        if (!box_hit(n, o, inv, mint, maxt)) continue;
        if (n->left < 0) {
            for (int i = 0; i < n->count; ++i) {
                int t = s->order[n->first + i];
                float tt, b1, b2;
                if (tri_hit(o, d, mint, maxt, ld(s->tp1, t), ld(s->te1, t), ld(s->te2, t), &tt, &b1, &b2)) return 1;
            }
        } else {
            stack[sp++] = n->right;
            stack[sp++] = n->left;
        }
    }
    return 0;
}

/* ------------------------------------------------------------------ tessellation */
typedef struct { float b0, b1, b2; } bary;
static const bary CENTROID = {1.f / 3.f, 1.f / 3.f, 1.f / 3.f};
static bary blerp(float t, bary a, bary b) {
    bary r = {(1.f - t) * a.b0 + t * b.b0, (1.f - t) * a.b1 + t * b.b1, (1.f - t) * a.b2 + t * b.b2};
    return r;
}
static bary beval(bary s, bary a, bary b, bary c) {
    bary r = {s.b0 * a.b0 + s.b1 * b.b0 + s.b2 * c.b0, s.b0 * a.b1 + s.b1 * b.b1 + s.b2 * c.b1,
              s.b0 * a.b2 + s.b1 * b.b2 + s.b2 * c.b2};
    return r;
}
static v3 bpoint(bary s, v3 a, v3 b, v3 c) { return add(add(mul(a, s.b0), mul(b, s.b1)), mul(c, s.b2)); }

typedef struct {
    const o_mesh *m;
    int t, incenter;
    float min_dist;
    v3 v0, v1, v2;
    o_surface_point *out;
    long n, cap;
    const o_tex *bump; /* the mesh material's bumpmap, or NULL */
} tess_ctx;

static void domain(tess_ctx *c, bary a, bary b, bary d) {
    v3 s0 = bpoint(a, c->v0, c->v1, c->v2), s1 = bpoint(b, c->v0, c->v1, c->v2), s2 = bpoint(d, c->v0, c->v1, c->v2);
    bary bc;
    if (!c->incenter) bc = beval(CENTROID, a, b, d);
    else {
        float l0 = len(sub(s1, s2)), l1 = len(sub(s2, s0)), l2 = len(sub(s0, s1));
        bary bic = {l0 / (l0 + l1 + l2), l1 / (l0 + l1 + l2), l2 / (l0 + l1 + l2)};
        bc = beval(bic, a, b, d);
    }
    if (c->out && c->n < c->cap) {
        o_surface_point *sp = &c->out[c->n];
        v3 p = bpoint(bc, c->v0, c->v1, c->v2);
        frame_t fr = tri_frame(c->m, c->t, p, bc.b0, bc.b1, bc.b2);
        v3 n = fr.nn;
        if (c->bump) { /* BumpMapping::Bump with dgs from GetDifferentialGeometries (no differentials) */
            float g[6] = {fr.u, fr.v, 0.f, 0.f, 0.f, 0.f};
            v3 dpdu_b;
            bump(c->bump, g, &fr, fr.nn, fr.ng, c->m->flip, &dpdu_b, &n);
        }
        sp->p[0] = p.x; sp->p[1] = p.y; sp->p[2] = p.z;
        sp->n[0] = n.x; sp->n[1] = n.y; sp->n[2] = n.z;
        sp->u = fr.u;
        sp->v = fr.v;
        sp->material = (uint32_t)c->m->material;
        sp->area = .5f * len(crs(sub(s1, s0), sub(s2, s0)));
        sp->ray_eps = c->min_dist / 10.f;
    }
    c->n++;
}

static void matching(tess_ctx *c, bary b0I, bary b1I, int segsI, bary b0O, bary b1O, int segsO) {
    int ip = 0, op = 0;
    while (ip < segsI || op < segsO) {
        bary bIn = segsI ? blerp((float)ip / segsI, b0I, b1I) : b0I;
        bary bOut = blerp((float)op / segsO, b0O, b1O);
        float sIn = (ip < segsI) ? fabsf((float)(ip + 1) + 1.f - (float)op / segsO * (segsI + 2)) : INFINITY;
        float sOut = (op < segsO) ? fabsf((float)ip + 1.f - (float)(op + 1) / segsO * (segsI + 2)) : INFINITY;
        if (sIn < sOut) {
            domain(c, blerp((float)(ip + 1) / segsI, b0I, b1I), bIn, bOut);
            ip++;
        } else {
            domain(c, bIn, bOut, blerp((float)(op + 1) / segsO, b0O, b1O));
            op++;
        }
    }
}

static int imax(int a, int b) { return a > b ? a : b; }

static void tessellator(tess_ctx *c, float tfe0, float tfe1, float tfe2, float tfc) {
    int e0 = imax((int)ceilf(tfe0), 1), e1 = imax((int)ceilf(tfe1), 1), e2 = imax((int)ceilf(tfe2), 1);
    int ic = imax((int)ceilf(tfc), 1);
    if (e0 > 1 || e1 > 1 || e2 > 1) ic = imax(ic, 2);
    bary B0 = {1.f, 0.f, 0.f}, B1 = {0.f, 1.f, 0.f}, B2 = {0.f, 0.f, 1.f}, BC = CENTROID;
    int rings = (ic + 1) / 2;
    for (int r = 0; r < rings - 1; ++r) {
        int inner = ic - (rings - r) * 2;
        if (inner >= 0) {
            int outer = inner + 2;
            bary i0 = blerp((float)r / rings, BC, B0), i1 = blerp((float)r / rings, BC, B1),
                 i2 = blerp((float)r / rings, BC, B2);
            bary o0 = blerp((float)(r + 1) / rings, BC, B0), o1 = blerp((float)(r + 1) / rings, BC, B1),
                 o2 = blerp((float)(r + 1) / rings, BC, B2);
            matching(c, i0, i1, inner, o0, o1, outer);
            matching(c, i1, i2, inner, o1, o2, outer);
            matching(c, i2, i0, inner, o2, o0, outer);
        } else {
            bary o0 = blerp((float)(r + 1) / rings, BC, B0), o1 = blerp((float)(r + 1) / rings, BC, B1),
                 o2 = blerp((float)(r + 1) / rings, BC, B2);
            domain(c, o0, o1, o2);
        }
    }
    int inner = ic - 2;
    if (inner >= 0) {
        float t = (float)(rings - 1) / rings;
        bary i0 = blerp(t, BC, B0), i1 = blerp(t, BC, B1), i2 = blerp(t, BC, B2);
        matching(c, i0, i1, inner, B0, B1, e2);
        matching(c, i1, i2, inner, B1, B2, e0);
        matching(c, i2, i0, inner, B2, B0, e1);
    } else {
        domain(c, B0, B1, B2);
    }
}

long o_tessellate(const o_scene *s, float min_dist, int incenter, o_surface_point *out, long cap) {
    tess_ctx c;
    memset(&c, 0, sizeof(c));
    c.out = out;
    c.cap = cap;
    c.min_dist = min_dist;
    c.incenter = incenter;
    for (int mi = 0; mi < s->nmeshes; ++mi) {
        const o_mesh *m = &s->meshes[mi];
        c.m = m;
        c.bump = (m->material >= 0 && m->material < s->nmats && s->mats[m->material].has_bump)
                     ? &s->mats[m->material].bump : NULL;
        for (int t = 0; t < m->nt; ++t) {
            c.t = t;
            c.v0 = ld(m->P, m->idx[3 * t]);
            c.v1 = ld(m->P, m->idx[3 * t + 1]);
            c.v2 = ld(m->P, m->idx[3 * t + 2]);
            float le0 = len(sub(c.v1, c.v2)), le1 = len(sub(c.v2, c.v0)), le2 = len(sub(c.v0, c.v1));
            float tfe0 = le0 / min_dist * 0.8f, tfe1 = le1 / min_dist * 0.8f, tfe2 = le2 / min_dist * 0.8f;
            float tfc = floorf((tfe0 + tfe1 + tfe2) / 3.f + .5f);
            tfe0 = floorf(tfe0 + .5f);
            tfe1 = floorf(tfe1 + .5f);
            tfe2 = floorf(tfe2 + .5f);
            tessellator(&c, tfe0, tfe1, tfe2, tfc);
        }
    }
    return c.n;
}

/* ------------------------------------------------------------------ irradiance (IrradianceTask) */
typedef struct {
    o_scene *s;
    const o_surface_point *pts;
    int n, nthreads, tid;
    uint32_t seed;
    float *E;
    const uint32_t *scr; /* reference-sampler scrambles (o_replay_irradiance_scr) or NULL */
} irr_job;

static void *irr_worker(void *arg) {
    irr_job *j = (irr_job *)arg;
    const o_scene *s = j->s;
    for (int i = j->tid; i < j->n; i += j->nthreads) {
        const o_surface_point *sp = &j->pts[i];
        v3 p = mk(sp->p[0], sp->p[1], sp->p[2]), n = mk(sp->n[0], sp->n[1], sp->n[2]);
        const o_mat *mat = sp->material < (uint32_t)s->nmats ? &s->mats[sp->material] : NULL;
        if (mat && mat->no_bssrdf) mat = NULL; /* the bssrdf == NULL branch (multipolesubsurface.cpp:100-107) */
        float E[O_NB];
        for (int c = 0; c < O_NB; ++c) E[c] = 0.f;
        for (int l = 0; l < s->nlights; ++l) {
            const o_light *L = &s->lights[l];
            float El[O_NB];
            for (int c = 0; c < O_NB; ++c) El[c] = 0.f;
            int ns = L->ns_pow2;
            uint32_t sc0, sc1;
            if (j->scr) { /* IrradianceTask: scramble[2] = {rng.RandomUInt(), rng.RandomUInt()} */
                sc0 = j->scr[((size_t)i * s->nlights + l) * 2];
                sc1 = j->scr[((size_t)i * s->nlights + l) * 2 + 1];
            } else {
                sc0 = hash3(j->seed, (uint32_t)i, 16u * l + D_IRR_POS);
                sc1 = hash3(j->seed, (uint32_t)i, 16u * l + D_IRR_POS + 8u);
            }
            for (int k = 0; k < ns; ++k) {
                lsamp ls = light_sample(L, p, sp->ray_eps, vdc((uint32_t)k, sc0), sobol((uint32_t)k, sc1));
                if (dot(ls.wi, n) <= 0.f) continue;
                if (!ls.nonblack || ls.pdf == 0.f) continue;
                if (!occluded(s, ls.so, ls.sd, ls.smint, ls.smaxt)) {
                    float ct = absdot(ls.wi, n);
                    ct = ct < 1.f ? ct : 1.f;
                    float Ft = mat ? 1.f - rho_at(mat, ct) : 1.f;
                    for (int c = 0; c < O_NB; ++c) El[c] += Ft * ls.Li[c] * ct / ls.pdf;
                }
            }
            for (int c = 0; c < O_NB; ++c) E[c] += El[c] / (float)ns;
        }
        if (mat && mat->has_alb) { /* albedo->Evaluate(dgs): (u, v) of the point, no differentials */
            float g[6] = {sp->u, sp->v, 0.f, 0.f, 0.f, 0.f}, a[O_NB];
            albedo_pow(&mat->alb, g, mat->mix, a);
            for (int c = 0; c < O_NB; ++c) E[c] *= a[c];
        } else if (mat) {
            for (int c = 0; c < O_NB; ++c) E[c] *= mat->alb_mix[c];
        }
        memcpy(&j->E[(size_t)i * O_NB], E, sizeof(E));
    }
    return NULL;
}

static void run_threads(void *(*fn)(void *), void *jobs, size_t job_size, int nthreads) {
    pthread_t *th = (pthread_t *)malloc(nthreads * sizeof(pthread_t));
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, fn, (char *)jobs + t * job_size);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    free(th);
}

static void irradiance_run(o_scene *s, int n, const o_surface_point *pts, uint32_t seed, const uint32_t *scr,
                           int nthreads, float *E) {
    scene_prepare(s);
    if (nthreads < 1) nthreads = 1;
    irr_job *jobs = (irr_job *)malloc(nthreads * sizeof(irr_job));
    for (int t = 0; t < nthreads; ++t) {
        irr_job j = {s, pts, n, nthreads, t, seed, E, scr};
        jobs[t] = j;
    }
    run_threads(irr_worker, jobs, sizeof(irr_job), nthreads);
    free(jobs);
}

void o_irradiance(o_scene *s, int n, const o_surface_point *pts, uint32_t seed, int nthreads, float *E) {
    irradiance_run(s, n, pts, seed, NULL, nthreads, E);
}

void o_irradiance_replay(o_scene *s, int n, const o_surface_point *pts, const uint32_t *scr, int nthreads, float *E) {
    irradiance_run(s, n, pts, 0, scr, nthreads, E);
}

void o_scene_set_octree(o_scene *s, int n, const float *p, const float *nr, const float *E, const float *area,
                        float max_error) {
    if (s->octree) o_octree_free(s->octree);
    s->octree = n > 0 ? o_octree_build(n, p, nr, E, area) : NULL;
    s->max_error = max_error;
}

/* ------------------------------------------------------------------ Li per camera sample */
static void to_xyz(const float L[O_NB], float xyz[3]) { /* Spectrum::ToXYZ + sample filter */
    static const float cx[O_NB] = MPSS_BAND_CIE_X_INIT, cy[O_NB] = MPSS_BAND_CIE_Y_INIT,
                       cz[O_NB] = MPSS_BAND_CIE_Z_INIT;
    float X = 0.f, Y = 0.f, Z = 0.f;
    int nan = 0;
    for (int c = 0; c < O_NB; ++c) {
        if (L[c] != L[c]) nan = 1;
        X += cx[c] * L[c];
        Y += cy[c] * L[c];
        Z += cz[c] * L[c];
    }
    float scale = (float)(700 - 400) / (float)(MPSS_CIE_Y_INTEGRAL * O_NB);
    float y = Y * (float)(700 - 400) / (float)(MPSS_CIE_Y_INTEGRAL * O_NB);
    X *= scale; Y *= scale; Z *= scale;
    if (nan || y < -1e-5f || isinf(y)) X = Y = Z = 0.f; /* samplerrenderer.cpp:119-133 */
    xyz[0] = X; xyz[1] = Y; xyz[2] = Z;
}

/* Sphere::Intersect's DifferentialGeometry at the camera ray's thit (sphere.cpp:114-152, object
 * space = world - centre) and the BSDF frame on it (reflection.cpp:754-762): nn = Normalize(Cross(dpdu,
 * dpdv)) = ng, sn = Normalize(dpdu), tn = Cross(nn, sn) */
static frame_t sphere_frame(const o_light *L, v3 o, v3 d, float t) {
    frame_t fr;
    memset(&fr, 0, sizeof(fr));
    v3 ph = add(sub(o, L->c), mul(d, t));
    if (ph.x == 0.f && ph.y == 0.f) ph.x = 1e-5f * L->r;
    float cz = ph.z / L->r;
    float theta = facos(cz < -1.f ? -1.f : (cz > 1.f ? 1.f : cz));
    float zr = sqrtf(ph.x * ph.x + ph.y * ph.y);
    float izr = 1.f / zr;
    float cphi = ph.x * izr, sphi = ph.y * izr;
    v3 dpdu = mk(-L->phimax * ph.y, L->phimax * ph.x, 0.f);
    v3 dpdv = mul(mk(ph.z * cphi, ph.z * sphi, -L->r * fsin(theta)), L->thetamax - L->thetamin);
    fr.p = add(ph, L->c);
    fr.nn = fr.ng = nrm(crs(dpdu, dpdv));
    fr.sn = nrm(dpdu);
    fr.tn = crs(fr.nn, fr.sn);
    return fr;
}

/* UniformSampleAllLights -> EstimateDirect (integrator.cpp:47-174) at shading point fr->p with
 * BSDF mat (its frame fr), rayEpsilon reps; row: reference-sampler values or NULL (hashes) */
static void direct_light(const o_scene *s, int spp, uint32_t seed, uint32_t pix, int si, const float *row,
                         const o_mat *mat, const frame_t *pfr, float reps, v3 wo, float ld[O_NB]) {
    for (int c = 0; c < O_NB; ++c) ld[c] = 0.f;
    for (int l = 0; l < s->nlights; ++l) {
        const o_light *Lt = &s->lights[l];
        const int ns = Lt->ns_pow2;
        float Ld[O_NB];
        for (int c = 0; c < O_NB; ++c) Ld[c] = 0.f;
        uint32_t xr = (spp & (spp - 1)) == 0 ? (hash3(seed, pix, 16u * l + D_PERM) & (uint32_t)(spp - 1)) : 0u;
        uint32_t base = (uint32_t)(si ^ xr) * (uint32_t)ns;
        uint32_t a0 = hash3(seed, pix, 16u * l + D_LIGHT_POS), a1 = hash3(seed, pix, 16u * l + D_LIGHT_POS + 8u);
        uint32_t b0 = hash3(seed, pix, 16u * l + D_BSDF_DIR), b1 = hash3(seed, pix, 16u * l + D_BSDF_DIR + 8u);
        uint32_t bc = hash3(seed, pix, 16u * l + D_BSDF_COMP);
        for (int j = 0; j < ns; ++j) {
            uint32_t k = base + (uint32_t)j;
            float ed[O_NB], f[O_NB];
            for (int c = 0; c < O_NB; ++c) ed[c] = 0.f;
            /* LightSample(sample, lightSampleOffsets[l], j), BSDFSample(sample, bsdfSampleOffsets[l], j) */
            float lu0, lu1, ubc, ub0, ub1;
            if (row) {
                const float *e = row + s->lights[l].replay_off + 5 * j;
                lu0 = e[0]; lu1 = e[1]; ubc = e[2]; ub0 = e[3]; ub1 = e[4];
            } else {
                lu0 = vdc(k, a0); lu1 = sobol(k, a1); ubc = vdc(k, bc); ub0 = vdc(k, b0); ub1 = sobol(k, b1);
            }
            lsamp ls = light_sample(Lt, pfr->p, reps, lu0, lu1);
            float lightPdf = ls.pdf;
            if (lightPdf > 0.f && ls.nonblack && (mat->has_refl || mat->has_trans)) {
                if (bsdf_f(mat, pfr, wo, ls.wi, to_local(pfr, wo), to_local(pfr, ls.wi), f) &&
                    !occluded(s, ls.so, ls.sd, ls.smint, ls.smaxt)) {
                    float bsdfPdf = bsdf_pdf(mat, to_local(pfr, wo), to_local(pfr, ls.wi));
                    float w = power_h(lightPdf, bsdfPdf);
                    float k1 = absdot(ls.wi, pfr->nn) * w / lightPdf;
                    for (int c = 0; c < O_NB; ++c) ed[c] += f[c] * ls.Li[c] * k1;
                }
            }
            int ncomp = mat->has_refl + mat->has_trans;
            if (ncomp > 0) {
                /* BSDF::Sample_f: component by uComponent, R before T */
                int which = (int)floorf(ubc * (float)ncomp);
                if (which > ncomp - 1) which = ncomp - 1;
                int pick_t = !mat->has_refl || which == 1;
                v3 wil, wol = to_local(pfr, wo);
                float bsdfPdf;
                if (pick_t) mt_sample(mat, wol, ub0, ub1, &wil, &bsdfPdf);
                else if (mat->lambert) lambert_sample(wol, ub0, ub1, &wil, &bsdfPdf);
                else mf_sample(mat, wol, ub0, ub1, &wil, &bsdfPdf);
                if (bsdfPdf != 0.f) {
                    v3 wi = to_world(pfr, wil);
                    if (ncomp > 1) {
                        bsdfPdf += pick_t ? mf_pdf(mat, wol, wil) : mt_pdf(mat, wol, wil);
                        bsdfPdf /= (float)ncomp;
                    }
                    if (bsdf_f(mat, pfr, wo, wi, to_local(pfr, wo), wil, f) && bsdfPdf > 0.f) {
                        lightPdf = Lt->kind ? inf_pdf(Lt, wi) : light_pdf(Lt, pfr->p, wi);
                        if (lightPdf != 0.f) {
                            float w = power_h(bsdfPdf, lightPdf);
                            hit_t hl = intersect(s, pfr->p, wi, reps, INFINITY);
                            float Li[O_NB];
                            memset(Li, 0, sizeof(Li));
                            if (hl.tri != NO_HIT) { /* Li = lightIsect.Le(-wi) if it is this light */
                                if (hl.tri == -1 - l && dot(hl.lnn, neg(wi)) > 0.f) memcpy(Li, Lt->Le, sizeof(Li));
                            } else if (Lt->kind) { /* Li = light->Le(ray) */
                                inf_le_dir(Lt, wi, Li);
                            }
                            if (!black(Li)) {
                                float adn = absdot(wi, pfr->nn);
                                for (int c = 0; c < O_NB; ++c) ed[c] += f[c] * Li[c] * adn * w / bsdfPdf;
                            }
                        }
                    }
                }
            }
            for (int c = 0; c < O_NB; ++c) Ld[c] += ed[c];
        }
        for (int c = 0; c < O_NB; ++c) ld[c] += Ld[c] / (float)ns;
    }
}

/* row: the sample's reference-sampler values (o_replay_render_table layout) or NULL (hashes) */
static void sample_li(const o_scene *s, int spp, uint32_t seed, int px, int py, int si, float X, float Y,
                      const float *row, float xyz[3]) {
    const uint32_t pix = (uint32_t)py * (uint32_t)s->xres + (uint32_t)px;
    float L[O_NB];
    for (int c = 0; c < O_NB; ++c) L[c] = 0.f;
    v3 pcam = xpoint(s->r2c, mk(X, Y, 0.f));
    v3 dcam = nrm(pcam);
    v3 o = xpoint(s->c2w, mk(0.f, 0.f, 0.f));
    v3 d = xvector(s->c2w, dcam);
    hit_t h = intersect(s, o, d, 0.f, INFINITY);
    if (h.tri == NO_HIT) { /* SamplerRenderer::Li: Li += lights[i]->Le(ray) (area lights: 0) */
        for (int l = 0; l < s->nlights; ++l) {
            float le[O_NB];
            if (s->lights[l].kind) inf_le_dir(&s->lights[l], d, le);
            else memset(le, 0, sizeof(le));
            for (int c = 0; c < O_NB; ++c) L[c] += le[c];
        }
        to_xyz(L, xyz);
        return;
    }
    if (h.tri < 0) { /* an area light's own sphere (multipolesubsurface.cpp:253-304): L = Le(wo), then
                      * Ld from every light at the sphere point with the shape's material -- pbrt's
                      * default "matte" (api.cpp:241,1085; matte.cpp:49-71: Kd 0.5, sigma 0, one
                      * Lambertian) -- and no BSSRDF; SpecularReflect/Transmit add 0 */
        const o_light *Lt = &s->lights[-1 - h.tri];
        if (dot(h.lnn, neg(d)) > 0.f)
            for (int c = 0; c < O_NB; ++c) L[c] += Lt->Le[c];
        /* R = Spectrum(0.5f); only lambert / has_refl / R are read */
#define H5 0.5f, 0.5f, 0.5f, 0.5f, 0.5f
        static const o_mat matte = {.R = {H5, H5, H5, H5, H5, H5}, .has_refl = 1, .lambert = 1};
#undef H5
        frame_t fr = sphere_frame(Lt, o, d, h.t);
        float ld[O_NB];
        direct_light(s, spp, seed, pix, si, row, &matte, &fr, 5e-4f * h.t, neg(d), ld); /* sphere.cpp:155 */
        for (int c = 0; c < O_NB; ++c) L[c] += ld[c];
        to_xyz(L, xyz);
        return;
    }
    const int mi = s->tri_mesh[h.tri], lt = s->tri_local[h.tri];
    const o_mesh *mesh = &s->meshes[mi];
    const o_mat *mat = &s->mats[mesh->material];
    v3 p = add(o, mul(d, h.t));
    float reps = 1e-3f * h.t;
    frame_t fr = tri_frame(mesh, lt, p, 1.f - h.b1 - h.b2, h.b1, h.b2);
    v3 wo = neg(d);
    float alb1[O_NB];
    if (mat->has_alb || mat->has_bump) {
        /* GenerateRayDifferential (perspective.cpp:81-113) + ScaleDifferentials(1 / sqrtf(spp)),
         * then dg.ComputeDifferentials: dgShading's (u, v) and differentials */
        v3 c0 = xpoint(s->r2c, mk(0.f, 0.f, 0.f));
        v3 dxc = sub(xpoint(s->r2c, mk(1.f, 0.f, 0.f)), c0), dyc = sub(xpoint(s->r2c, mk(0.f, 1.f, 0.f)), c0);
        v3 rxw = xvector(s->c2w, nrm(add(pcam, dxc))), ryw = xvector(s->c2w, nrm(add(pcam, dyc)));
        float k = 1.f / sqrtf((float)spp);
        v3 rxd = add(d, mul(sub(rxw, d), k)), ryd = add(d, mul(sub(ryw, d), k));
        float g[6] = {fr.u, fr.v, 0.f, 0.f, 0.f, 0.f};
        differentials(p, fr.ng, fr.dpdu, fr.dpdv, o, rxd, ryd, g);
        if (mat->has_alb) albedo_pow(&mat->alb, g, 1.f - mat->mix, alb1);
        if (mat->has_bump) { /* BSDF on the bumped dgs */
            v3 dpdu_b, nn_b;
            bump(&mat->bump, g, &fr, fr.nn, fr.ng, mesh->flip, &dpdu_b, &nn_b);
            fr.nn = nn_b;
            fr.sn = nrm(dpdu_b);
            fr.tn = crs(fr.nn, fr.sn);
        }
    }
    if (!mat->has_alb) memcpy(alb1, mat->alb_1mmix, sizeof(alb1));
    /* Mo() term (multipolesubsurface.cpp:268-290) */
    if (s->octree && !mat->no_bssrdf) {
        float q[3] = {fr.p.x, fr.p.y, fr.p.z}, mo[O_NB];
        if (mat->rgb)
            o_mo_batch_rgb(s->octree, 1, q, mat->rd, mat->L, mat->rcp, s->max_error, mo, NULL, NULL, 1);
        else
            o_mo_batch(s->octree, 1, q, mat->rd, mat->L, mat->rcp, s->max_error, mo, NULL, NULL, 1);
        float ct = absdot(wo, fr.nn);
        ct = ct < 1.f ? ct : 1.f;
        float Ft = mat->is_mc ? 1.f : 1.f - rho_at(mat, ct);
        for (int c = 0; c < O_NB; ++c) {
            float t = ((INV_PI_F * Ft) * mo[c]) * alb1[c];
            L[c] += t < 0.f ? 0.f : t;
        }
    }
    float ld[O_NB];
    direct_light(s, spp, seed, pix, si, row, mat, &fr, reps, wo, ld);
    for (int c = 0; c < O_NB; ++c) L[c] += ld[c];
    to_xyz(L, xyz);
}

/* ImageFilm::AddSample pixel range of one coordinate (0.5-wide box filter) */
static void extent(float X, int res, int *lo, int *hi) {
    float d = X - 0.5f;
    *lo = (int)ceilf(d - 0.5f);
    *hi = (int)floorf(d + 0.5f);
    if (*lo < 0) *lo = 0;
    if (*hi > res - 1) *hi = res - 1;
}

typedef struct {
    const o_scene *s;
    int spp, x0, x1, y0, y1, nthreads, tid;
    uint32_t seed;
    float *out;
    const float *vals; /* reference-sampler table (o_replay_render_table) or NULL */
    int K;
    int vx0, vy0, vw;  /* the table's window: origin pixel and width (whole extent: 0, 0, xres + 1) */
} tile_job;

/* One pixel: its own samples, then neighbours' samples whose rounded image position lands
 * on the shared edge, neighbours in row-major order (matches the product's film order). */
static void render_pixel(const tile_job *j, int px, int py, float *o4) {
    const o_scene *s = j->s;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int q = 0; q < 9; ++q) {
        int idx = q == 0 ? 4 : (q - 1 + (q > 4));
        int dx = idx % 3 - 1, dy = idx / 3 - 1;
        int qx = px + dx, qy = py + dy;
        if (qx < 0 || qy < 0 || qx >= s->xres || qy >= s->yres) continue;
        uint32_t pix = (uint32_t)qy * (uint32_t)s->xres + (uint32_t)qx;
        uint32_t su = hash3(j->seed, pix, D_IMAGE), sv = hash3(j->seed, pix, D_IMAGE + 1);
        for (int si = 0; si < j->spp; ++si) {
            const float *row = NULL;
            float X, Y;
            if (j->vals) { /* imageX = xPos + imageSamples[2 i] (montecarlo.cpp:236-237) */
                row = j->vals + (((size_t)(qy - j->vy0) * (size_t)j->vw + (size_t)(qx - j->vx0)) * (size_t)j->spp +
                                 (size_t)si) * (size_t)j->K;
                X = (float)qx + row[0];
                Y = (float)qy + row[1];
            } else {
                X = (float)qx + vdc((uint32_t)si, su);
                Y = (float)qy + sobol((uint32_t)si, sv);
            }
            int lx, hx, ly, hy;
            extent(X, s->xres, &lx, &hx);
            extent(Y, s->yres, &ly, &hy);
            if (px < lx || px > hx || py < ly || py > hy) continue;
            float xyz[3];
            sample_li(s, j->spp, j->seed, qx, qy, si, X, Y, row, xyz);
            acc[0] += 1.f * xyz[0];
            acc[1] += 1.f * xyz[1];
            acc[2] += 1.f * xyz[2];
            acc[3] += 1.f;
        }
    }
    memcpy(o4, acc, sizeof(acc));
}

static void *tile_worker(void *arg) {
    tile_job *j = (tile_job *)arg;
    int tw = j->x1 - j->x0, th = j->y1 - j->y0;
    for (int i = j->tid; i < tw * th; i += j->nthreads) {
        int px = j->x0 + i % tw, py = j->y0 + i / tw;
        render_pixel(j, px, py, &j->out[(size_t)i * 4]);
    }
    return NULL;
}

static void render_run(o_scene *s, int spp, uint32_t seed, const float *vals, int K, int vx0, int vy0, int vw, int x0,
                       int x1, int y0, int y1, int nthreads, float *xyzw) {
    scene_prepare(s);
    if (nthreads < 1) nthreads = 1;
    tile_job *jobs = (tile_job *)malloc(nthreads * sizeof(tile_job));
    for (int t = 0; t < nthreads; ++t) {
        tile_job j = {s, spp, x0, x1, y0, y1, nthreads, t, seed, xyzw, vals, K, vx0, vy0, vw};
        jobs[t] = j;
    }
    run_threads(tile_worker, jobs, sizeof(tile_job), nthreads);
    free(jobs);
}

void o_render_tile(o_scene *s, int spp, uint32_t seed, int x0, int x1, int y0, int y1, int nthreads, float *xyzw) {
    render_run(s, spp, seed, NULL, 0, 0, 0, 0, x0, x1, y0, y1, nthreads, xyzw);
}

void o_render_tile_replay(o_scene *s, int spp, const float *vals, int K, int x0, int x1, int y0, int y1,
                          int nthreads, float *xyzw) {
    render_run(s, spp, 0, vals, K, 0, 0, s->xres + 1, x0, x1, y0, y1, nthreads, xyzw);
}

void o_render_tile_replay_window(o_scene *s, int spp, const float *vals, int K, int vx0, int vx1, int vy0, int vy1,
                                 int x0, int x1, int y0, int y1, int nthreads, float *xyzw) {
    (void)vy1;
    render_run(s, spp, 0, vals, K, vx0, vy0, vx1 - vx0, x0, x1, y0, y1, nthreads, xyzw);
}

/* ---- the CPU baseline: SamplerRenderer::Render's task loop (samplerrenderer.cpp:191-225) ----
 * nTasks = RoundUpPow2(max(32 * cores, W * H / 256)) sub-windows (Sampler::ComputeSubWindow of the
 * image), taken from one shared counter by a pool of nthreads workers (parallel.cpp's task queue)
 * in the order order[0..ntasks) until `seconds` have passed; each task renders its pixels with the
 * hash sampler into a private buffer. Returns the pixels rendered; tasks_done / elapsed out. */
typedef struct {
    o_scene *s;
    int spp, ntasks, cores;
    uint32_t seed;
    const int *order;
    double deadline;
    int next;
    long pixels, tasks;
    pthread_mutex_t mu;
} base_job;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void sub_window(int num, int count, int xs, int xe, int ys, int ye, int *x0, int *x1, int *y0, int *y1);

static void *base_worker(void *arg) {
    base_job *b = (base_job *)arg;
    o_scene *s = b->s;
    tile_job j = {s, b->spp, 0, 0, 0, 0, 1, 0, b->seed, NULL, NULL, 0, 0, 0, 0};
    float *buf = NULL;
    size_t cap = 0;
    long px = 0, nt = 0;
    for (;;) {
        pthread_mutex_lock(&b->mu);
        int k = b->next < b->ntasks && now_s() < b->deadline ? b->next++ : -1;
        pthread_mutex_unlock(&b->mu);
        if (k < 0) break;
        int x0, x1, y0, y1;
        sub_window(b->order[k], b->ntasks, 0, s->xres, 0, s->yres, &x0, &x1, &y0, &y1);
        size_t n = (size_t)(x1 - x0) * (size_t)(y1 - y0);
        if (n > cap) {
            free(buf);
            cap = n;
            buf = (float *)malloc(4 * sizeof(float) * cap);
        }
        for (int y = y0; y < y1; ++y)
            for (int x = x0; x < x1; ++x) render_pixel(&j, x, y, &buf[4 * ((size_t)(y - y0) * (x1 - x0) + (x - x0))]);
        px += (long)n;
        ++nt;
    }
    free(buf);
    pthread_mutex_lock(&b->mu);
    b->pixels += px;
    b->tasks += nt;
    pthread_mutex_unlock(&b->mu);
    return NULL;
}

long o_cpu_baseline(o_scene *s, int spp, uint32_t seed, int cores, int nthreads, double seconds, const int *order,
                    int norder, long *tasks_done, double *elapsed) {
    scene_prepare(s);
    if (nthreads < 1) nthreads = 1;
    base_job b;
    memset(&b, 0, sizeof(b));
    b.s = s;
    b.spp = spp;
    b.seed = seed;
    b.cores = cores;
    b.ntasks = norder;
    b.order = order;
    pthread_mutex_init(&b.mu, NULL);
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nthreads);
    double t0 = now_s();
    b.deadline = t0 + seconds;
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, base_worker, &b);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    *elapsed = now_s() - t0;
    *tasks_done = b.tasks;
    free(th);
    pthread_mutex_destroy(&b.mu);
    return b.pixels;
}

/* nTasks of SamplerRenderer::Render for an image and a core count */
int o_render_task_count(int xres, int yres, int cores) {
    int a = 32 * cores, b = (int)(((long)xres * yres) / (16 * 16)), m = a > b ? a : b, r = 1;
    while (r < m) r <<= 1;
    return r;
}

void o_sub_window(int num, int count, int xs, int xe, int ys, int ye, int *out) {
    sub_window(num, count, xs, xe, ys, ye, &out[0], &out[1], &out[2], &out[3]);
}

/* ------------------------------------------------------------------ the reference sampler */
/* Shuffle (montecarlo.h:183-189) */
static void shuffle(float *samp, uint32_t count, uint32_t dims, o_mt *rng) {
    for (uint32_t i = 0; i < count; ++i) {
        uint32_t other = i + (o_mt_u32(rng) % (count - i));
        for (uint32_t j = 0; j < dims; ++j) {
            float t = samp[dims * i + j];
            samp[dims * i + j] = samp[dims * other + j];
            samp[dims * other + j] = t;
        }
    }
}

/* LDShuffleScrambled1D (montecarlo.h:314-322) */
static void ld_shuffle_scrambled_1d(int n, int npix, float *samples, o_mt *rng) {
    uint32_t scramble = o_mt_u32(rng);
    for (int i = 0; i < n * npix; ++i) samples[i] = vdc((uint32_t)i, scramble);
    for (int i = 0; i < npix; ++i) shuffle(samples + i * n, (uint32_t)n, 1, rng);
    shuffle(samples, (uint32_t)npix, (uint32_t)n, rng);
}

/* LDShuffleScrambled2D (montecarlo.h:325-333); the scrambles are drawn left to right */
static void ld_shuffle_scrambled_2d(int n, int npix, float *samples, o_mt *rng) {
    uint32_t scramble[2];
    scramble[0] = o_mt_u32(rng);
    scramble[1] = o_mt_u32(rng);
    for (int i = 0; i < n * npix; ++i) { /* Sample02 */
        samples[2 * i] = vdc((uint32_t)i, scramble[0]);
        samples[2 * i + 1] = sobol((uint32_t)i, scramble[1]);
    }
    for (int i = 0; i < npix; ++i) shuffle(samples + 2 * i * n, (uint32_t)n, 2, rng);
    shuffle(samples, (uint32_t)npix, (uint32_t)(2 * n), rng);
}

/* Sampler::ComputeSubWindow (sampler.cpp:55-78) */
static void sub_window(int num, int count, int xs, int xe, int ys, int ye, int *x0, int *x1, int *y0, int *y1) {
    int dx = xe - xs, dy = ye - ys;
    int nx = count, ny = 1;
    while ((nx & 0x1) == 0 && 2 * dx * ny < dy * nx) {
        nx >>= 1;
        ny <<= 1;
    }
    int xo = num % nx, yo = num / nx;
    float tx0 = (float)xo / (float)nx, tx1 = (float)(xo + 1) / (float)nx;
    float ty0 = (float)yo / (float)ny, ty1 = (float)(yo + 1) / (float)ny;
    *x0 = (int)floorf((1.f - tx0) * (float)xs + tx0 * (float)xe); /* Floor2Int(Lerp(..)) */
    *x1 = (int)floorf((1.f - tx1) * (float)xs + tx1 * (float)xe);
    *y0 = (int)floorf((1.f - ty0) * (float)ys + ty0 * (float)ye);
    *y1 = (int)floorf((1.f - ty1) * (float)ys + ty1 * (float)ye);
}

typedef struct {
    o_scene *s;
    int spp, K, li_draws, ntasks, next;
    float *vals;
    int vx0, vx1, vy0, vy1;  /* rows are kept for pixels of this window of the sample extent */
    pthread_mutex_t mu;
} rtab_job;

/* SamplerRendererTask::Run (samplerrenderer.cpp:60-167) for task `task`: RNG(task), then per pixel
 * LDSampler::GetMoreSamples -> LDPixelSample (lowdiscrepancy.cpp:69-82, montecarlo.cpp:200-250),
 * then per sample the camera ray and, when it hits, Li's BSDFSample(rng) draws. */
static void render_task(rtab_job *jb, int task) {
    o_scene *s = jb->s;
    const int spp = jb->spp, K = jb->K, W1 = s->xres + 1, H1 = s->yres + 1;
    int x0, x1, y0, y1;
    sub_window(task, jb->ntasks, 0, W1, 0, H1, &x0, &x1, &y0, &y1);
    if (x0 == x1 || y0 == y1) return; /* GetSubSampler returns NULL */
    /* a task's stream is its own (RNG(taskNum)): tasks outside the window are skipped whole */
    if (x1 <= jb->vx0 || x0 >= jb->vx1 || y1 <= jb->vy0 || y0 >= jb->vy1) return;
    const int vw = jb->vx1 - jb->vx0;
    o_mt rng;
    o_mt_seed(&rng, (uint32_t)task);
    /* n1D: per light comp (L), comp (BSDF); then the emission integrator's 1, 1. n2D: pos, dir. */
    const int nl = s->nlights, c1 = 2 * nl + 2, c2 = 2 * nl;
    int n1[2 * 254 + 2], n2[2 * 254];
    for (int l = 0; l < nl; ++l) {
        n1[2 * l] = n1[2 * l + 1] = s->lights[l].ns_pow2;
        n2[2 * l] = n2[2 * l + 1] = s->lights[l].ns_pow2;
    }
    n1[2 * nl] = n1[2 * nl + 1] = 1;
    float *image = (float *)malloc(sizeof(float) * 2 * spp), *lens = (float *)malloc(sizeof(float) * 2 * spp);
    float *time = (float *)malloc(sizeof(float) * spp);
    float **one = (float **)malloc(sizeof(float *) * (c1 + 1)), **two = (float **)malloc(sizeof(float *) * (c2 + 1));
    for (int a = 0; a < c1; ++a) one[a] = (float *)malloc(sizeof(float) * n1[a] * spp);
    for (int a = 0; a < c2; ++a) two[a] = (float *)malloc(sizeof(float) * 2 * n2[a] * spp);
    v3 o = xpoint(s->c2w, mk(0.f, 0.f, 0.f));
    for (int y = y0; y < y1; ++y)
        for (int x = x0; x < x1; ++x) {
            ld_shuffle_scrambled_2d(1, spp, image, &rng);
            ld_shuffle_scrambled_2d(1, spp, lens, &rng);
            ld_shuffle_scrambled_1d(1, spp, time, &rng);
            for (int a = 0; a < c1; ++a) ld_shuffle_scrambled_1d(n1[a], spp, one[a], &rng);
            for (int a = 0; a < c2; ++a) ld_shuffle_scrambled_2d(n2[a], spp, two[a], &rng);
            const int keep = x >= jb->vx0 && x < jb->vx1 && y >= jb->vy0 && y < jb->vy1;
            for (int i = 0; keep && i < spp; ++i) {
                float *row = jb->vals + (((size_t)(y - jb->vy0) * vw + (x - jb->vx0)) * spp + i) * K;
                row[0] = image[2 * i];
                row[1] = image[2 * i + 1];
                for (int l = 0; l < nl; ++l) {
                    const int n = n1[2 * l];
                    for (int j = 0; j < n; ++j) { /* samples[i].oneD[a][j] = oneD[a][n i + j], twoD: 2 (n i + j) */
                        float *e = row + s->lights[l].replay_off + 5 * j;
                        e[0] = two[2 * l][2 * (n * i + j)];
                        e[1] = two[2 * l][2 * (n * i + j) + 1];
                        e[2] = one[2 * l + 1][n * i + j];
                        e[3] = two[2 * l + 1][2 * (n * i + j)];
                        e[4] = two[2 * l + 1][2 * (n * i + j) + 1];
                    }
                }
            }
            if (jb->li_draws > 0)
                for (int i = 0; i < spp; ++i) {
                    float X = (float)x + image[2 * i], Y = (float)y + image[2 * i + 1];
                    v3 d = xvector(s->c2w, nrm(xpoint(s->r2c, mk(X, Y, 0.f))));
                    if (intersect(s, o, d, 0.f, INFINITY).tri != NO_HIT)
                        for (int k = 0; k < jb->li_draws; ++k) (void)o_mt_u32(&rng);
                }
        }
    for (int a = 0; a < c1; ++a) free(one[a]);
    for (int a = 0; a < c2; ++a) free(two[a]);
    free(one); free(two); free(image); free(lens); free(time);
}

static void *rtab_worker(void *arg) {
    rtab_job *jb = (rtab_job *)arg;
    for (;;) {
        pthread_mutex_lock(&jb->mu);
        int task = jb->next++;
        pthread_mutex_unlock(&jb->mu);
        if (task >= jb->ntasks) break;
        render_task(jb, task);
    }
    return NULL;
}

static int round_pow2_int(int v) { int r = 1; while (r < v) r <<= 1; return r; }

int o_replay_render_table_window(o_scene *s, int spp, int cores, int li_draws, int nthreads, int vx0, int vx1,
                                 int vy0, int vy1, float *vals);

int o_replay_render_table(o_scene *s, int spp, int cores, int li_draws, int nthreads, float *vals) {
    return o_replay_render_table_window(s, spp, cores, li_draws, nthreads, 0, s->xres + 1, 0, s->yres + 1, vals);
}

int o_replay_render_table_window(o_scene *s, int spp, int cores, int li_draws, int nthreads, int vx0, int vx1,
                                 int vy0, int vy1, float *vals) {
    int K = 2;
    for (int l = 0; l < s->nlights; ++l) {
        s->lights[l].replay_off = K;
        K += 5 * s->lights[l].ns_pow2;
    }
    if (!vals) return K;
    scene_prepare(s);
    /* nTasks = RoundUpPow2(max(32 * NumSystemCores(), nPixels / (16 * 16))) */
    int a = 32 * cores, b = (int)(((long)s->xres * s->yres) / (16 * 16));
    rtab_job jb;
    memset(&jb, 0, sizeof(jb));
    jb.s = s; jb.spp = spp; jb.K = K; jb.li_draws = li_draws; jb.vals = vals;
    jb.vx0 = vx0; jb.vx1 = vx1; jb.vy0 = vy0; jb.vy1 = vy1;
    jb.ntasks = round_pow2_int(a > b ? a : b);
    pthread_mutex_init(&jb.mu, NULL);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, rtab_worker, &jb);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    pthread_mutex_destroy(&jb.mu);
    return K;
}

/* IrradianceTask::Run (multipolesubsurface.cpp:72-152) with nTasks = RoundUpPow2(max(32 cores, N/4096)) */
void o_replay_irradiance_scr(int n, int nlights, int cores, uint32_t *scr) {
    int a = 32 * cores, b = n / 4096;
    int T = round_pow2_int(a > b ? a : b);
    for (int k = 0; k < T; ++k) {
        size_t i0 = (size_t)((uint64_t)k * (uint64_t)n / (uint64_t)T);
        size_t i1 = (size_t)((uint64_t)(k + 1) * (uint64_t)n / (uint64_t)T);
        if (i0 == i1) continue;
        o_mt rng;
        o_mt_seed(&rng, (uint32_t)k * 47u);
        for (size_t i = i0; i < i1; ++i)
            for (int l = 0; l < nlights; ++l) {
                scr[(i * nlights + l) * 2] = o_mt_u32(&rng);
                scr[(i * nlights + l) * 2 + 1] = o_mt_u32(&rng);
                (void)o_mt_u32(&rng); /* compScramble */
            }
    }
}

void o_scene_free(o_scene *s) {
    if (!s) return;
    for (int m = 0; m < s->nmeshes; ++m) {
        free(s->meshes[m].P); free(s->meshes[m].N); free(s->meshes[m].S); free(s->meshes[m].uv);
        free(s->meshes[m].idx);
    }
    for (int m = 0; m < s->nmats; ++m) {
        free(s->mats[m].rho);
        free(s->mats[m].rd);
        if (s->mats[m].has_alb) o_tex_free(&s->mats[m].alb);
        if (s->mats[m].has_bump) o_tex_free(&s->mats[m].bump);
    }
    for (int l = 0; l < s->nlights; ++l)
        if (s->lights[l].kind) o_envmap_free(&s->lights[l].em);
    free(s->meshes); free(s->lights); free(s->mats);
    free(s->tri_mesh); free(s->tri_local); free(s->tp1); free(s->te1); free(s->te2);
    free(s->bvh); free(s->order);
    if (s->octree) o_octree_free(s->octree);
    free(s);
}

/* ------------------------------------------------------------------ Poisson point finder
 * FindPoissonPointDistribution -> SurfacePointsRenderer::Render (renderers/surfacepoints.cpp:
 * 115-150) with one SurfacePointTask (:175-284). Paths are traced one after another and their
 * candidates tested in path order (the reference tests a batch's candidates after tracing it;
 * tracing never depends on the test, so the order of tests is the same), the give-up test
 * after every 20000 paths. Random numbers: counter-based per (seed, path, draw), replay mode. */
static float pu01(uint32_t seed, uint32_t path, uint32_t k) { return (float)(hash3(seed, path, k) >> 8) * 0x1p-24f; }
static v3 ffwd(v3 n, v3 v) { return dot(n, v) < 0.f ? neg(n) : n; }
static v3 sph_point(const o_light *L, v3 o, v3 d, float t) {
    v3 ph = add(sub(o, L->c), mul(d, t));
    if (ph.x == 0.f && ph.y == 0.f) ph.x = 1e-5f * L->r;
    return add(ph, L->c);
}

typedef struct { int64_t key; int first; } pcell;
typedef struct {
    pcell *tab; size_t mask; int *next; float md;
} pgrid;
static uint64_t pkey(int64_t x, int64_t y, int64_t z) {
    return ((uint64_t)(x & 0x1fffff) << 42) | ((uint64_t)(y & 0x1fffff) << 21) | (uint64_t)(z & 0x1fffff);
}
static pcell *pfind(pgrid *g, uint64_t k, int insert) {
    size_t h = (size_t)(mix32((uint32_t)k ^ mix32((uint32_t)(k >> 32)))) & g->mask;
    for (;;) {
        pcell *c = &g->tab[h];
        if (c->first < 0) {
            if (!insert) return NULL;
            c->key = (int64_t)k;
            return c;
        }
        if ((uint64_t)c->key == k) return c;
        h = (h + 1) & g->mask;
    }
}

long o_poisson_points(o_scene *s, float min_dist, int quick, uint32_t seed, o_surface_point *out, long cap) {
    scene_prepare(s);
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int mi = 0; mi < s->nmeshes; ++mi) {
        const o_mesh *m = &s->meshes[mi];
        for (int t = 0; t < 3 * m->nt; ++t)
            for (int k = 0; k < 3; ++k) {
                float v = m->P[3 * m->idx[t] + k];
                lo[k] = fminf(lo[k], v);
                hi[k] = fmaxf(hi[k], v);
            }
    }
    for (int l = 0; l < s->nlights; ++l) {
        const o_light *L = &s->lights[l];
        if (L->kind) continue;
        float c[3] = {L->c.x, L->c.y, L->c.z};
        for (int k = 0; k < 3; ++k) {
            lo[k] = fminf(lo[k], c[k] + -L->r);
            hi[k] = fmaxf(hi[k], c[k] + L->r);
        }
    }
    /* BBox::BoundingSphere, and the ReverseOrientation sphere there */
    o_light bound;
    memset(&bound, 0, sizeof(bound));
    bound.c = mk(.5f * lo[0] + .5f * hi[0], .5f * lo[1] + .5f * hi[1], .5f * lo[2] + .5f * hi[2]);
    int inside = bound.c.x >= lo[0] && bound.c.x <= hi[0] && bound.c.y >= lo[1] && bound.c.y <= hi[1] &&
                 bound.c.z >= lo[2] && bound.c.z <= hi[2];
    bound.r = inside ? len(sub(bound.c, mk(hi[0], hi[1], hi[2]))) : 0.f;
    bound.phimax = (PI_F / 180.f) * 360.f;
    bound.thetamin = facos(-1.f);
    bound.thetamax = facos(1.f);
    bound.area = bound.phimax * bound.r * (bound.r - -bound.r);
    const v3 origin = xpoint(s->c2w, mk(0.f, 0.f, 0.f));
    const uint32_t sd = mix32(seed * 37u + 0x5eed1u);
    const int max_fails = quick ? (200 > 10 ? 200 : 10) : 2000;
    const float md2 = min_dist * min_dist;
    const float area = PI_F * (min_dist / 2.f) * (min_dist / 2.f);
    pgrid g;
    size_t tsz = 1;
    while (tsz < 2 * (size_t)(cap > 0 ? cap : 1)) tsz <<= 1;
    g.tab = (pcell *)malloc(tsz * sizeof(pcell));
    for (size_t i = 0; i < tsz; ++i) g.tab[i].first = -1;
    g.mask = tsz - 1;
    g.next = (int *)malloc((size_t)(cap > 0 ? cap : 1) * sizeof(int));
    long n = 0;
    int fails = 0, done = 0;
    for (uint32_t path = 0; !done; ++path) {
        uint32_t k = 0;
        float u1 = pu01(sd, path, k++), u2 = pu01(sd, path, k++);
        v3 o = origin, d = sample_sphere_uniform(u1, u2);
        float mint = 0.f;
        for (int depth = 0; depth < 30 && !done; ++depth) {
            hit_t h = intersect(s, o, d, mint, INFINITY);
            v3 p, nn;
            float eps;
            int cand = 0;
            o_surface_point sp;
            if (h.tri == NO_HIT) {
                float t;
                v3 snn;
                if (!sphere_hit(&bound, o, d, mint, INFINITY, &t, &snn)) break;
                p = sph_point(&bound, o, d, t);
                nn = ffwd(snn, neg(d));
                eps = 5e-4f * t;
            } else if (h.tri < 0) {
                p = sph_point(&s->lights[-1 - h.tri], o, d, h.t);
                nn = ffwd(h.lnn, neg(d));
                eps = 5e-4f * h.t;
            } else {
                const int mi = s->tri_mesh[h.tri], lt = s->tri_local[h.tri];
                const o_mesh *mesh = &s->meshes[mi];
                p = add(o, mul(d, h.t));
                frame_t fr = tri_frame(mesh, lt, p, 1.f - h.b1 - h.b2, h.b1, h.b2);
                nn = ffwd(fr.ng, neg(d));
                eps = 1e-3f * h.t;
                if (depth >= 3) { /* every material on this path is LayeredSkin: GetBSSRDF != NULL */
                    v3 sn = (!mesh->N && !mesh->S) ? nn : fr.nn;
                    const o_mat *mt = &s->mats[mesh->material];
                    if (mt->has_bump) { /* Bump(hitGeometry, dgShading) without differentials */
                        float g[6] = {fr.u, fr.v, 0.f, 0.f, 0.f, 0.f};
                        v3 dpdu_b;
                        bump(&mt->bump, g, &fr, sn, nn, mesh->flip, &dpdu_b, &sn);
                    }
                    sp.p[0] = p.x; sp.p[1] = p.y; sp.p[2] = p.z;
                    sp.n[0] = sn.x; sp.n[1] = sn.y; sp.n[2] = sn.z;
                    sp.u = fr.u; sp.v = fr.v;
                    sp.material = (uint32_t)mesh->material;
                    sp.area = area;
                    sp.ray_eps = eps;
                    cand = 1;
                }
            }
            if (cand) { /* PoissonCheck against every accepted point within a cell of p */
                int64_t cx = (int64_t)floor((double)sp.p[0] / (double)min_dist);
                int64_t cy = (int64_t)floor((double)sp.p[1] / (double)min_dist);
                int64_t cz = (int64_t)floor((double)sp.p[2] / (double)min_dist);
                int fail = 0;
                for (int dz = -1; dz <= 1 && !fail; ++dz)
                    for (int dy = -1; dy <= 1 && !fail; ++dy)
                        for (int dx = -1; dx <= 1 && !fail; ++dx) {
                            pcell *c = pfind(&g, pkey(cx + dx, cy + dy, cz + dz), 0);
                            for (int q = c ? c->first : -1; q >= 0; q = g.next[q]) {
                                float ex = out[q].p[0] - sp.p[0], ey = out[q].p[1] - sp.p[1], ez = out[q].p[2] - sp.p[2];
                                if (ex * ex + ey * ey + ez * ez < md2) { fail = 1; break; }
                            }
                        }
                if (fail) {
                    if (++fails >= max_fails) done = 1;
                } else {
                    if (n >= cap) { free(g.tab); free(g.next); return -1; }
                    fails = 0;
                    pcell *c = pfind(&g, pkey(cx, cy, cz), 1);
                    g.next[n] = c->first;
                    c->first = (int)n;
                    out[n++] = sp;
                }
            }
            if (done) break;
            u1 = pu01(sd, path, k++);
            u2 = pu01(sd, path, k++);
            d = ffwd(sample_sphere_uniform(u1, u2), nn);
            o = p;
            mint = eps;
        }
        if (!done && (path + 1) % 20000 == 0 && (long)(path + 1) > 50000 && n == 0) { done = 1; n = -2; }
    }
    free(g.tab);
    free(g.next);
    return n;
}
