/* oracle/octree.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 * Restates SubsurfaceOctreeNode::{Insert, InitHierarchy, Mo} (reference
 * src/integrators/diffusionutil.h:86-234), octreeChildBound (core/octree.h:87-97),
 * the Preprocess octree build loop (integrators/multipolesubsurface.cpp:301-321)
 * and MultipoleReflectance -> sampleProfile (core/multipole.cpp:60-113); the alternate Rd
 * functor DiffusionReflectance (diffusionutil.h:38-83), the single dipole that the
 * dipolesubsurface integrator hands to the same Mo (dipolesubsurface.cpp:171-172).
 * Points are inserted in index order (the reference inserts in mutex-completion
 * order, multipolesubsurface.cpp:230-234; index order is the deterministic choice
 * both this oracle and the product make). */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

typedef struct onode {
    float p[3], n[3];
    int is_leaf;
    float Et[O_NB];
    float sum_area;
    struct onode *child[8];
    int ips[8]; /* point indices, -1 = empty */
} onode;

struct o_octree {
    int npts;
    float *p, *n, *E, *area;
    float bmin[3], bmax[3];
    onode *root;
    int nnodes;
    onode **pool;
    int pool_n, pool_cap;
};

static onode *alloc_node(o_octree *t) {
    onode *nd = (onode *)calloc(1, sizeof(onode));
    nd->is_leaf = 1;
    for (int i = 0; i < 8; ++i) nd->ips[i] = -1;
    if (t->pool_n == t->pool_cap) {
        t->pool_cap = t->pool_cap ? t->pool_cap * 2 : 1024;
        t->pool = (onode **)realloc(t->pool, sizeof(onode *) * t->pool_cap);
    }
    t->pool[t->pool_n++] = nd;
    t->nnodes++;
    return nd;
}

static void child_bound(int c, const float bmin[3], const float bmax[3], const float mid[3], float cmin[3],
                        float cmax[3]) {
    cmin[0] = (c & 4) ? mid[0] : bmin[0];
    cmax[0] = (c & 4) ? bmax[0] : mid[0];
    cmin[1] = (c & 2) ? mid[1] : bmin[1];
    cmax[1] = (c & 2) ? bmax[1] : mid[1];
    cmin[2] = (c & 1) ? mid[2] : bmin[2];
    cmax[2] = (c & 1) ? bmax[2] : mid[2];
}

static void insert(o_octree *t, onode *nd, const float bmin[3], const float bmax[3], int ip, int depth) {
    if (depth > 96) abort(); /* >8 coincident points recurse forever in the reference too */
    float mid[3];
    for (int k = 0; k < 3; ++k) mid[k] = .5f * bmin[k] + .5f * bmax[k];
    if (nd->is_leaf) {
        for (int i = 0; i < 8; ++i)
            if (nd->ips[i] < 0) { nd->ips[i] = ip; return; }
        nd->is_leaf = 0;
        int local[8];
        for (int i = 0; i < 8; ++i) { local[i] = nd->ips[i]; nd->child[i] = NULL; }
        for (int i = 0; i < 8; ++i) {
            const float *pp = t->p + 3 * local[i];
            int c = (pp[0] > mid[0] ? 4 : 0) + (pp[1] > mid[1] ? 2 : 0) + (pp[2] > mid[2] ? 1 : 0);
            if (!nd->child[c]) nd->child[c] = alloc_node(t);
            float cmin[3], cmax[3];
            child_bound(c, bmin, bmax, mid, cmin, cmax);
            insert(t, nd->child[c], cmin, cmax, local[i], depth + 1);
        }
    }
    const float *pp = t->p + 3 * ip;
    int c = (pp[0] > mid[0] ? 4 : 0) + (pp[1] > mid[1] ? 2 : 0) + (pp[2] > mid[2] ? 1 : 0);
    if (!nd->child[c]) nd->child[c] = alloc_node(t);
    float cmin[3], cmax[3];
    child_bound(c, bmin, bmax, mid, cmin, cmax);
    insert(t, nd->child[c], cmin, cmax, ip, depth + 1);
}

static void init_hier(o_octree *t, onode *nd) {
    float sum_wt = 0.f;
    if (nd->is_leaf) {
        for (int i = 0; i < 8; ++i) {
            if (nd->ips[i] < 0) break;
            int ip = nd->ips[i];
            float et[O_NB];
            for (int c = 0; c < O_NB; ++c) et[c] = t->E[(size_t)ip * O_NB + c] * t->area[ip];
            float wt = o_y(et);
            for (int c = 0; c < O_NB; ++c) nd->Et[c] += et[c];
            for (int k = 0; k < 3; ++k) nd->p[k] += t->p[3 * ip + k] * wt;
            for (int k = 0; k < 3; ++k) nd->n[k] += t->n[3 * ip + k] * wt;
            sum_wt += wt;
            nd->sum_area += t->area[ip];
        }
    } else {
        for (int i = 0; i < 8; ++i) {
            onode *ch = nd->child[i];
            if (!ch) continue;
            init_hier(t, ch);
            float wt = o_y(ch->Et);
            for (int c = 0; c < O_NB; ++c) nd->Et[c] += ch->Et[c];
            for (int k = 0; k < 3; ++k) nd->p[k] += ch->p[k] * wt;
            for (int k = 0; k < 3; ++k) nd->n[k] += ch->n[k] * wt;
            sum_wt += wt;
            nd->sum_area += ch->sum_area;
        }
    }
    if (sum_wt > 0.f) {
        float inv = 1.f / sum_wt;
        for (int k = 0; k < 3; ++k) { nd->p[k] *= inv; nd->n[k] *= inv; }
    }
}

o_octree *o_octree_build(int n, const float *p, const float *nrm, const float *E, const float *area) {
    o_octree *t = (o_octree *)calloc(1, sizeof(o_octree));
    t->npts = n;
    t->p = (float *)malloc(sizeof(float) * 3 * (size_t)n);
    t->n = (float *)malloc(sizeof(float) * 3 * (size_t)n);
    t->E = (float *)malloc(sizeof(float) * O_NB * (size_t)n);
    t->area = (float *)malloc(sizeof(float) * (size_t)n);
    memcpy(t->p, p, sizeof(float) * 3 * (size_t)n);
    memcpy(t->n, nrm, sizeof(float) * 3 * (size_t)n);
    memcpy(t->E, E, sizeof(float) * O_NB * (size_t)n);
    memcpy(t->area, area, sizeof(float) * (size_t)n);
    for (int k = 0; k < 3; ++k) { t->bmin[k] = INFINITY; t->bmax[k] = -INFINITY; }
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) {
            float v = p[3 * i + k];
            t->bmin[k] = (v < t->bmin[k]) ? v : t->bmin[k]; /* std::min(a,b) = b<a ? b : a */
            t->bmax[k] = (t->bmax[k] < v) ? v : t->bmax[k];
        }
    t->root = alloc_node(t);
    for (int i = 0; i < n; ++i) insert(t, t->root, t->bmin, t->bmax, i, 0);
    init_hier(t, t->root);
    return t;
}

void o_octree_free(o_octree *t) {
    if (!t) return;
    for (int i = 0; i < t->pool_n; ++i) free(t->pool[i]);
    free(t->pool);
    free(t->p); free(t->n); free(t->E); free(t->area);
    free(t);
}

int o_octree_num_nodes(const o_octree *t) { return t->nnodes; }
void o_octree_bounds(const o_octree *t, float bmin[3], float bmax[3]) {
    for (int k = 0; k < 3; ++k) { bmin[k] = t->bmin[k]; bmax[k] = t->bmax[k]; }
}

static int is_black(const float *s) {
    for (int c = 0; c < O_NB; ++c)
        if (s[c] != 0.) return 0;
    return 1;
}

typedef struct {
    const o_octree *t;
    const float *tab;
    int len;
    const float *rcp;
    float max_error;
    long nodes, points;
    const o_diffusion *dip; /* non-NULL: DiffusionReflectance instead of the profile table */
    int rgb;                /* rgbprofile: tab rows 0..2 are the R, G, B profiles */
} mo_ctx;

/* ---- DiffusionReflectance (diffusionutil.h:38-83) ---- */
/* Fdr, core/reflection.h:64-71 */
static float fdr_eta(float eta) {
    if (eta >= 1) return -1.4399f / (eta * eta) + 0.7099f / eta + 0.6681f + 0.0636f * eta;
    return -0.4399f + .7099f / eta - .3319f / (eta * eta) + .0636f / (eta * eta * eta);
}

/* pbrt.h:196 redefines M_PI as a float literal */
#define O_PI_F 3.14159265358979323846f

void o_diffusion_init(const float sigma_a[O_NB], const float sigmap_s[O_NB], float eta, o_diffusion *d) {
    /* constructor, diffusionutil.h:40-48; spectrum ops are per-band float ops (spectrum.h:125-240) */
    d->A = (1.f + fdr_eta(eta)) / (1.f - fdr_eta(eta));
    for (int c = 0; c < O_NB; ++c) {
        d->sigmap_t[c] = sigma_a[c] + sigmap_s[c];
        /* 3.f * sigma_a is s * 3.f (operator*(float, Spectrum), spectrum.h:180-184), then * sigmap_t */
        d->sigma_tr[c] = sqrtf((sigma_a[c] * 3.f) * d->sigmap_t[c]);
        d->alphap[c] = sigmap_s[c] / d->sigmap_t[c];
        d->zpos[c] = 1.f / d->sigmap_t[c];
        d->zneg[c] = (-d->zpos[c]) * (1.f + (4.f / 3.f) * d->A);
    }
}

/* operator()(float d2), diffusionutil.h:49-58: Rd = (alphap / (4 M_PI)) * (pos - neg), Clamp() */
void o_diffusion_eval(const o_diffusion *d, float d2, float out[O_NB]) {
    const float four_pi = 4.f * O_PI_F;
    for (int c = 0; c < O_NB; ++c) {
        float dpos = sqrtf(d2 + d->zpos[c] * d->zpos[c]);
        float dneg = sqrtf(d2 + d->zneg[c] * d->zneg[c]);
        float e_pos = (float)exp((double)((-d->sigma_tr[c]) * dpos));
        float e_neg = (float)exp((double)((-d->sigma_tr[c]) * dneg));
        float pos = ((d->zpos[c] * (dpos * d->sigma_tr[c] + 1.f)) * e_pos) / ((dpos * dpos) * dpos);
        float neg = ((d->zneg[c] * (dneg * d->sigma_tr[c] + 1.f)) * e_neg) / ((dneg * dneg) * dneg);
        float rd = (d->alphap[c] / four_pi) * (pos - neg);
        /* Spectrum::Clamp(0, INFINITY) -> ::Clamp (pbrt.h) */
        out[c] = rd < 0.f ? 0.f : (rd > INFINITY ? INFINITY : rd);
    }
}

/* TotalReflectance, diffusionutil.h:69-77 */
void o_diffusion_total(const o_diffusion *d, float out[O_NB]) {
    for (int c = 0; c < O_NB; ++c) {
        float mfp = 1.f / d->sigmap_t[c];
        float step = ((4.f * mfp) * (4.f * mfp)) / 1024.f;
        float integral = 0.f;
        for (int i = 0; i < 1024; ++i) {
            float v[O_NB];
            o_diffusion_eval(d, step * (float)i, v); /* the Spectrum-d2 overload, band c */
            integral += v[c];
        }
        out[c] = (integral * step) * O_PI_F;
    }
}

static float dist2(const float *a, const float *b) {
    float x = a[0] - b[0], y = a[1] - b[1], z = a[2] - b[2];
    return x * x + y * y + z * z;
}

static void rd_eval(const mo_ctx *m, float d2, float out[O_NB]) {
    if (m->dip) {
        o_diffusion_eval(m->dip, d2, out);
        return;
    }
    if (m->rgb) {
        /* MultipoleProfileData::reflectance with isRGBProfile (multipole.cpp:85-107):
           Spectrum::FromRGBSpectrum(sampleRGBProfile(...)) = SampledSpectrum::FromRGB(rgb, reflectance) */
        float rgb[3];
        for (int k = 0; k < 3; ++k) rgb[k] = o_sample_profile(m->tab + (size_t)k * m->len, m->len, m->rcp[k], d2);
        o_from_rgb(rgb, 0, out);
        return;
    }
    for (int c = 0; c < O_NB; ++c) out[c] = o_sample_profile(m->tab + (size_t)c * m->len, m->len, m->rcp[c], d2);
}

/* SubsurfaceOctreeNode::Mo, diffusionutil.h:175-210 */
static void mo_rec(mo_ctx *m, const onode *nd, const float bmin[3], const float bmax[3], const float *pt,
                   float out[O_NB]) {
    m->nodes++;
    for (int c = 0; c < O_NB; ++c) out[c] = 0.f;
    if (is_black(nd->Et)) return;
    float dw = nd->sum_area / dist2(pt, nd->p);
    int inside = pt[0] >= bmin[0] && pt[0] <= bmax[0] && pt[1] >= bmin[1] && pt[1] <= bmax[1] &&
                 pt[2] >= bmin[2] && pt[2] <= bmax[2];
    if (dw < m->max_error && !inside) {
        float rd[O_NB];
        rd_eval(m, dist2(pt, nd->p), rd);
        for (int c = 0; c < O_NB; ++c) out[c] = rd[c] * nd->Et[c];
        return;
    }
    if (nd->is_leaf) {
        for (int i = 0; i < 8; ++i) {
            int ip = nd->ips[i];
            if (ip < 0) break;
            const float *E = m->t->E + (size_t)ip * O_NB;
            if (is_black(E)) continue;
            m->points++;
            float rd[O_NB];
            rd_eval(m, dist2(pt, m->t->p + 3 * ip), rd);
            float a = m->t->area[ip];
            for (int c = 0; c < O_NB; ++c) out[c] += rd[c] * E[c] * a;
        }
    } else {
        float mid[3];
        for (int k = 0; k < 3; ++k) mid[k] = .5f * bmin[k] + .5f * bmax[k];
        for (int c8 = 0; c8 < 8; ++c8) {
            if (!nd->child[c8]) continue;
            float cmin[3], cmax[3], sub[O_NB];
            child_bound(c8, bmin, bmax, mid, cmin, cmax);
            mo_rec(m, nd->child[c8], cmin, cmax, pt, sub);
            for (int c = 0; c < O_NB; ++c) out[c] += sub[c];
        }
    }
}

typedef struct {
    const o_octree *t;
    int q;
    const float *pts, *tab, *rcp;
    int len;
    float max_error;
    float *mo;
    int32_t *nn, *np;
    int next;
    pthread_mutex_t mu;
    const o_diffusion *dip;
    int rgb;
} mo_job;

static void *mo_worker(void *arg) {
    mo_job *j = (mo_job *)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        int start = j->next;
        j->next += 256;
        pthread_mutex_unlock(&j->mu);
        if (start >= j->q) break;
        int end = start + 256 < j->q ? start + 256 : j->q;
        for (int i = start; i < end; ++i) {
            mo_ctx m = {j->t, j->tab, j->len, j->rcp, j->max_error, 0, 0, j->dip, j->rgb};
            mo_rec(&m, j->t->root, j->t->bmin, j->t->bmax, j->pts + 3 * (size_t)i, j->mo + (size_t)i * O_NB);
            if (j->nn) j->nn[i] = (int32_t)m.nodes;
            if (j->np) j->np[i] = (int32_t)m.points;
        }
    }
    return NULL;
}

static void mo_run(mo_job *jp, int nthreads);

void o_mo_batch_diffusion(const o_octree *t, int q, const float *pts, const o_diffusion *d, float max_error,
                          float *mo, int32_t *nn, int32_t *np, int nthreads) {
    mo_job j;
    memset(&j, 0, sizeof(j));
    j.t = t; j.q = q; j.pts = pts; j.max_error = max_error; j.mo = mo; j.nn = nn; j.np = np; j.dip = d;
    mo_run(&j, nthreads);
}

void o_mo_batch(const o_octree *t, int q, const float *pts, const float *tab, int len, const float rcp[O_NB],
                float max_error, float *mo, int32_t *nn, int32_t *np, int nthreads) {
    mo_job j;
    memset(&j, 0, sizeof(j));
    j.t = t; j.q = q; j.pts = pts; j.tab = tab; j.rcp = rcp; j.len = len; j.max_error = max_error;
    j.mo = mo; j.nn = nn; j.np = np;
    mo_run(&j, nthreads);
}

void o_mo_batch_rgb(const o_octree *t, int q, const float *pts, const float *tab, int len, const float rcp[3],
                    float max_error, float *mo, int32_t *nn, int32_t *np, int nthreads) {
    mo_job j;
    memset(&j, 0, sizeof(j));
    j.t = t; j.q = q; j.pts = pts; j.tab = tab; j.rcp = rcp; j.len = len; j.max_error = max_error;
    j.mo = mo; j.nn = nn; j.np = np; j.rgb = 1;
    mo_run(&j, nthreads);
}

static void mo_run(mo_job *jp, int nthreads) {
    pthread_mutex_init(&jp->mu, NULL);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    for (int i = 0; i < nthreads; ++i) pthread_create(&th[i], NULL, mo_worker, jp);
    for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
    pthread_mutex_destroy(&jp->mu);
}

/* Pre-order flattening (children in index order 0..7, leaves keep ips[] order). */
typedef struct {
    float *np, *na, *ne, *bn, *bx;
    int32_t *dep, *skip, *lf, *lc, *order;
    int n, npo;
} exp_ctx;

static void exp_rec(exp_ctx *e, const o_octree *t, const onode *nd, const float bmin[3], const float bmax[3], int d) {
    int me = e->n++;
    if (e->np) {
        for (int k = 0; k < 3; ++k) {
            e->np[3 * me + k] = nd->p[k];
            e->bn[3 * me + k] = bmin[k];
            e->bx[3 * me + k] = bmax[k];
        }
        e->na[me] = nd->sum_area;
        memcpy(e->ne + (size_t)me * O_NB, nd->Et, sizeof(float) * O_NB);
        e->dep[me] = d;
    }
    if (nd->is_leaf) {
        int cnt = 0;
        if (e->lf) e->lf[me] = e->npo;
        for (int i = 0; i < 8 && nd->ips[i] >= 0; ++i) {
            if (e->order) e->order[e->npo] = nd->ips[i];
            e->npo++;
            cnt++;
        }
        if (e->lc) e->lc[me] = cnt;
    } else {
        if (e->lf) { e->lf[me] = -1; e->lc[me] = 0; }
        float mid[3];
        for (int k = 0; k < 3; ++k) mid[k] = .5f * bmin[k] + .5f * bmax[k];
        for (int c = 0; c < 8; ++c) {
            if (!nd->child[c]) continue;
            float cmin[3], cmax[3];
            child_bound(c, bmin, bmax, mid, cmin, cmax);
            exp_rec(e, t, nd->child[c], cmin, cmax, d + 1);
        }
    }
    if (e->skip) e->skip[me] = e->n;
}

int o_octree_export(const o_octree *t, float *node_p, float *node_area, float *node_et, float *bmin, float *bmax,
                    int32_t *depth, int32_t *skip, int32_t *leaf_first, int32_t *leaf_count, int32_t *order) {
    exp_ctx e = {node_p, node_area, node_et, bmin, bmax, depth, skip, leaf_first, leaf_count, order, 0, 0};
    exp_rec(&e, t, t->root, t->bmin, t->bmax, 0);
    return e.n;
}
