/* oracle/mpc.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 * Restates the MultipoleProfileCalculator (reference
 * src/multipole/MultipoleProfileCalculator/{MultipoleProfileCalculator.cpp:151-426,
 * DipoleCalculator.cpp:38-91, numutil.h:62-281}) and the per-channel driver
 * MultipoleProfileTask::Run (src/core/multipole.cpp:241-295), plus sampleProfile
 * (multipole.cpp:60-73). Float where the reference is float, double where double. */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

void o_free(void *p) { free(p); }

/* ---- DipoleCalculator.cpp:38-91 ---- */
static const float O_PI_MPC = 3.141592654f;            /* numutil.h:45 */
#define O_INV_FOURPI (0.25f / O_PI_MPC)                 /* numutil.h:46 */

static float fdr(float eta) { /* DipoleCalculator.cpp:38-46 */
    if (eta >= 1.f) return -1.4399f / (eta * eta) + 0.7099f / eta + 0.6681f + 0.0636f * eta;
    float eta2 = eta * eta;
    return -0.4399f + 0.7099f / eta - 0.3319f / eta2 + 0.0636f / (eta2 * eta);
}
static float afn(float F) { return (1.f + F) / (1.f - F); }

typedef struct { float d, zpos, zneg, sigma_tr, alphap; } dipole;

static void dipole_init(dipole *dc, float eta0, float etad, float d, float sa, float sps, int zi, int lerp) {
    dc->d = d;
    float spt = sa + sps;
    dc->sigma_tr = sqrtf(3 * sa * spt);
    dc->alphap = sps / spt;
    float A0 = afn(fdr(eta0)), Ad = afn(fdr(etad));
    float D = 1.f / (3.f * spt);
    float zb0 = 2.f * A0 * D, zbd = 2.f * Ad * D;
    float l = 1.f / spt;
    if (lerp && l > d * .5f) l = d * .5f;
    dc->zpos = 2.f * (float)zi * (d + zb0 + zbd) + l;
    dc->zneg = dc->zpos - 2.f * (l + zb0);
}
static float dipole_rd(const dipole *dc, float dsq) {
    float dp = sqrtf(dsq + dc->zpos * dc->zpos);
    float dn = sqrtf(dsq + dc->zneg * dc->zneg);
    float dp3 = dp * dp * dp, dn3 = dn * dn * dn;
    return dc->alphap * O_INV_FOURPI *
           (dc->zpos * (1 + dc->sigma_tr * dp) * expf(-dc->sigma_tr * dp) / dp3 -
            dc->zneg * (1 + dc->sigma_tr * dn) * expf(-dc->sigma_tr * dn) / dn3);
}
static float dipole_td(const dipole *dc, float dsq) {
    float a = dc->d - dc->zpos, b = dc->d - dc->zneg;
    float dp = sqrtf(dsq + a * a);
    float dn = sqrtf(dsq + b * b);
    float dp3 = dp * dp * dp, dn3 = dn * dn * dn;
    return dc->alphap * O_INV_FOURPI *
           (a * (1 + dc->sigma_tr * dp) * expf(-dc->sigma_tr * dp) / dp3 -
            b * (1 + dc->sigma_tr * dn) * expf(-dc->sigma_tr * dn) / dn3);
}
float o_dipole_rd(float eta0, float etad, float d, float mua, float musp, int zi, int lerp, float dsq) {
    dipole dc;
    dipole_init(&dc, eta0, etad, d, mua, musp, zi, lerp);
    return dipole_rd(&dc, dsq);
}

/* ---- ComputeLayerProfile, MultipoleProfileCalculator.cpp:151-230 ---- */
static void layer_profile(const o_layer_spec *spec, float ior_up, float ior_lo, float step, int lerp_thin,
                          int len, double *R, double *T) {
    memset(R, 0, sizeof(double) * len * len);
    memset(T, 0, sizeof(double) * len * len);
    float thickness = spec->thickness;
    double mfp2 = 2. / (spec->mua + spec->musp);
    double lerp = 1.;
    if (lerp_thin) {
        lerp = (thickness < mfp2) ? (1. - exp(-thickness * 2. / mfp2)) / (1. - exp(-2.)) : 1.;
        if (thickness < 0.01 * mfp2) thickness = (float)(0.01 * mfp2);
    }
    int center = (len - 1) / 2, extent = center;
    dipole dcs[11];
    int nd = 0;
    for (int pair = -5; pair <= 5; ++pair)
        dipole_init(&dcs[nd++], ior_up, ior_lo, thickness, spec->mua, spec->musp, pair, lerp_thin);
    double nf = step * step;
#define AT(M, r, c) (M)[(size_t)(r) * len + (c)]
    for (int row = 0; row <= extent; ++row)
        for (int col = row; col <= extent; ++col) {
            double dr2 = (double)((unsigned)row * (unsigned)row), dc2 = (double)((unsigned)col * (unsigned)col);
            double r2 = (dr2 + dc2) * (step * step);
            for (int k = 0; k < nd; ++k) {
                double rd = dipole_rd(&dcs[k], (float)r2) * nf;
                double td = dipole_td(&dcs[k], (float)r2) * nf;
                AT(R, center + row, center + col) += rd;
                AT(T, center + row, center + col) += td;
            }
        }
    if (lerp < 1.) {
        for (int row = 0; row <= extent; ++row)
            for (int col = row; col <= extent; ++col) {
                AT(R, center + row, center + col) *= lerp;
                AT(T, center + row, center + col) *= lerp;
            }
        AT(T, center, center) += 1. - lerp;
    }
    for (int row = 1; row <= extent; ++row)
        for (int col = 0; col < row; ++col) {
            AT(R, center + row, center + col) = AT(R, center + col, center + row);
            AT(T, center + row, center + col) = AT(T, center + col, center + row);
        }
    for (int row = 0; row <= extent; ++row)
        for (int col = 0; col <= extent; ++col) {
            double rd = AT(R, center + row, center + col);
            AT(R, center - row, center + col) = rd;
            AT(R, center + row, center - col) = rd;
            AT(R, center - row, center - col) = rd;
            double td = AT(T, center + row, center + col);
            AT(T, center - row, center + col) = td;
            AT(T, center + row, center - col) = td;
            AT(T, center - row, center - col) = td;
        }
#undef AT
}

/* ToFrequencyDomain (:233-240) with ScaleAndShift (numutil.h:201-213) */
static o_cpx *to_freq(const double *P, int len) {
    int cl = len * 2, center = (len - 1) / 2, nrb = cl / 2 + 1;
    double *big = (double *)calloc((size_t)cl * cl, sizeof(double));
    for (int i = 0; i < len; ++i) {
        int ii = cl - center + i; if (ii >= cl) ii -= cl;
        for (int j = 0; j < len; ++j) {
            int jj = cl - center + j; if (jj >= cl) jj -= cl;
            big[(size_t)ii * cl + jj] = P[(size_t)i * len + j];
        }
    }
    o_cpx *out = (o_cpx *)malloc(sizeof(o_cpx) * (size_t)cl * nrb);
    o_kiss_fftndr2(cl, cl, big, out);
    free(big);
    return out;
}

/* ToTimeDomain (:243-250): IFFT (:133-139) then ScaleAndShiftReversed (numutil.h:214-226) */
static void to_time(const o_cpx *F, int len, double *out) {
    int cl = len * 2, center = (len - 1) / 2;
    double *big = (double *)malloc(sizeof(double) * (size_t)cl * cl);
    o_kiss_fftndri2(cl, cl, F, big);
    double s = (double)1 / (cl * cl);
    for (size_t k = 0; k < (size_t)cl * cl; ++k) big[k] *= s;
    for (int i = 0; i < len; ++i) {
        int ii = cl - center + i; if (ii >= cl) ii -= cl;
        for (int j = 0; j < len; ++j) {
            int jj = cl - center + j; if (jj >= cl) jj -= cl;
            out[(size_t)i * len + j] = big[(size_t)ii * cl + jj];
        }
    }
    free(big);
}

static void cmul_(o_cpx *a, o_cpx b) { /* MultipoleProfileCalculator.cpp:56-61 */
    double r = a->r * b.r - a->i * b.i;
    double i = a->r * b.i + a->i * b.r;
    a->r = r; a->i = i;
}
static void cdiv_(o_cpx *a, o_cpx b) { /* :63-70 */
    double div = b.r * b.r + b.i * b.i;
    double acbd = a->r * b.r + a->i * b.i;
    double bcad = a->i * b.r - a->r * b.i;
    a->r = acbd / div;
    a->i = bcad / div;
}

/* CombineLayerProfiles, :253-280 */
static void combine(int len, const double *R1, const double *T1, const double *R2, const double *T2,
                    double *R12, double *T12) {
    size_t nf = (size_t)(len * 2) * (len + 1);
    o_cpx *fR1 = to_freq(R1, len), *fR2 = to_freq(R2, len), *fT1 = to_freq(T1, len), *fT2 = to_freq(T2, len);
    o_cpx *one = (o_cpx *)malloc(sizeof(o_cpx) * nf);
    o_cpx *acc = (o_cpx *)malloc(sizeof(o_cpx) * nf);
    for (size_t k = 0; k < nf; ++k) {
        o_cpx x = fR2[k];
        cmul_(&x, fR1[k]);
        x.r = 1. - x.r; x.i = 0. - x.i; /* OneMinusSelf: makecpx(1) - th */
        one[k] = x;
        o_cpx y = fT1[k];
        cmul_(&y, fR2[k]);
        cmul_(&y, fT1[k]);
        cdiv_(&y, x);
        y.r += fR1[k].r; y.i += fR1[k].i;
        acc[k] = y;
    }
    to_time(acc, len, R12);
    for (size_t k = 0; k < nf; ++k) {
        o_cpx y = fT1[k];
        cmul_(&y, fT2[k]);
        cdiv_(&y, one[k]);
        acc[k] = y;
    }
    to_time(acc, len, T12);
    free(fR1); free(fR2); free(fT1); free(fT2); free(one); free(acc);
}

static double kahan_sum(const double *v, size_t n) { /* numutil.h:236-246 */
    double sum = 0, c = 0;
    for (size_t i = 0; i < n; ++i) {
        double y = v[i] - c;
        double t = sum + y;
        c = (t - sum) - y;
        sum = t;
    }
    return sum;
}

static int cmpf(const void *a, const void *b) {
    float x = *(const float *)a, y = *(const float *)b;
    return x < y ? -1 : x > y ? 1 : 0;
}

static float clampf_(float v, float lo, float hi) { return v < lo ? lo : v > hi ? hi : v; }
static int clampi_(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }

/* resample, :355-402 */
static void resample1(int len, const float *d, const float *R, const float *T, float dsq, float *r, float *t) {
    float ext = d[len - 1];
    if (dsq > ext) { *r = *t = 0.f; return; }
    unsigned lo = 0, hi = len - 1;
    float d2lo = d[lo];
    if (lo + 32 < hi) {
        float d2hi = d[hi];
        do {
            unsigned mid = clampi_((int)((dsq - d2lo) / (d2hi - d2lo) * (float)(hi - lo)), 0, (int)(hi - lo - 1)) + lo;
            float d2mid = d[mid];
            if (dsq > d2mid) { lo = mid + 1; d2lo = d[lo]; }
            else { hi = mid; d2hi = d2mid; }
        } while (lo + 32 < hi);
    }
    while (lo < hi && dsq > d2lo) { lo++; d2lo = d[lo]; }
    if (lo) {
        float la = clampf_((dsq - d[lo - 1]) / (d[lo] - d[lo - 1]), 0.f, 1.f);
        if (la != la) la = 0.5f;
        *r = (1.f - la) * R[lo - 1] + la * R[lo];
        *t = (1.f - la) * T[lo - 1] + la * T[lo];
    } else {
        *r = R[0];
        *t = T[0];
    }
}

static unsigned round_up_pow2(unsigned v) {
    v--; v |= v >> 1; v |= v >> 2; v |= v >> 4; v |= v >> 8; v |= v >> 16;
    return v + 1;
}

/* MPC_ComputeDiffusionProfile (:294-346) [+ MPC_ResampleForUniformDistanceSquaredDistribution :404-426] */
int o_mpc_profile(int nlayers, const o_layer_spec *sp, float step, int desired_length, int lerp_thin,
                  int resample, float **dsq_out, float **r_out, float **t_out, float *total_r, float *total_t) {
    int length = (int)round_up_pow2((unsigned)desired_length);
    int L = length * 2;
    size_t nn = (size_t)L * L;
    double *R0 = (double *)malloc(sizeof(double) * nn), *T0 = (double *)malloc(sizeof(double) * nn);
    float ior_lo = nlayers > 1 ? sp[0].ior / sp[1].ior : sp[0].ior;
    layer_profile(&sp[0], sp[0].ior, ior_lo, step, lerp_thin, L, R0, T0);
    for (int i = 1; i < nlayers; ++i) {
        ior_lo = nlayers > i + 1 ? sp[i].ior / sp[i + 1].ior : sp[i].ior;
        double *R1 = (double *)malloc(sizeof(double) * nn), *T1 = (double *)malloc(sizeof(double) * nn);
        layer_profile(&sp[i], sp[i].ior / sp[i - 1].ior, ior_lo, step, lerp_thin, L, R1, T1);
        double *R12 = (double *)malloc(sizeof(double) * nn), *T12 = (double *)malloc(sizeof(double) * nn);
        combine(L, R0, T0, R1, T1, R12, T12);
        free(R0); free(T0); free(R1); free(T1);
        R0 = R12; T0 = T12;
    }
    /* unique d^2 entries, std::set<OutEntry> semantics: first insertion wins, sorted by dsq */
    unsigned center = (unsigned)length - 1, extent = center;
    float denorm = 1.f / (step * step);
    size_t cap = 0;
    for (unsigned i = 0; i <= extent; ++i)
        for (unsigned j = i; i * i + j * j <= extent * extent; ++j) cap++;
    /* key array: (dsq, insertion order) */
    typedef struct { float dsq; unsigned ord; float r, t; } ent;
    ent *e = (ent *)malloc(sizeof(ent) * cap);
    size_t ne = 0;
    for (unsigned i = 0; i <= extent; ++i)
        for (unsigned j = i; i * i + j * j <= extent * extent; ++j) {
            e[ne].dsq = (float)(i * i + j * j) * step * step;
            e[ne].ord = (unsigned)ne;
            e[ne].r = (float)R0[(size_t)(center + i) * L + (center + j)] * denorm;
            e[ne].t = (float)T0[(size_t)(center + i) * L + (center + j)] * denorm;
            ne++;
        }
    /* stable sort by dsq keeps insertion order among equal keys -> keep first of each run */
    /* simple insertion via qsort on (dsq, ord) */
    int cmp_ent(const void *a, const void *b);
    qsort(e, ne, sizeof(ent), cmp_ent);
    size_t nu = 0;
    for (size_t k = 0; k < ne; ++k)
        if (nu == 0 || e[k].dsq != e[nu - 1].dsq) e[nu++] = e[k];
    *total_r = (float)kahan_sum(R0, nn);
    *total_t = (float)kahan_sum(T0, nn);
    free(R0); free(T0);
    float *d = (float *)malloc(sizeof(float) * nu), *r = (float *)malloc(sizeof(float) * nu),
          *t = (float *)malloc(sizeof(float) * nu);
    for (size_t k = 0; k < nu; ++k) { d[k] = e[k].dsq; r[k] = e[k].r; t[k] = e[k].t; }
    free(e);
    int outlen = (int)nu;
    if (resample) {
        int tl = outlen * 2;
        float ext = d[outlen - 1];
        float *nd = (float *)malloc(sizeof(float) * tl), *nr = (float *)malloc(sizeof(float) * tl),
              *nt = (float *)malloc(sizeof(float) * tl);
        for (int i = 0; i < tl; ++i) {
            float q = (float)i * ext / (float)(tl - 1);
            nd[i] = q;
            resample1(outlen, d, r, t, q, nr + i, nt + i);
        }
        free(d); free(r); free(t);
        d = nd; r = nr; t = nt;
        outlen = tl;
    }
    *dsq_out = d;
    *r_out = r;
    *t_out = t;
    return outlen;
}

/* MPC_ResampleDistribution (MultipoleProfileCalculator.cpp:429-448): the profile at distances
 * points[i] (squared before the lookup). */
void o_mpc_resample(int len, const float *d, const float *R, const float *T, int n, const float *points, float *r,
                    float *t) {
    for (int i = 0; i < n; ++i) resample1(len, d, R, T, points[i] * points[i], r + i, t + i);
}

/* MPC_ResampleForUniformDistanceSquaredDistribution (:404-426) with an explicit target length:
 * out[i] = the profile at d^2 = (float)i * d[len-1] / (float)(target - 1). */
void o_mpc_resample_uniform(int len, const float *d, const float *R, int target, float *out) {
    float ext = d[len - 1], dummy;
    for (int i = 0; i < target; ++i) resample1(len, d, R, R, (float)i * ext / (float)(target - 1), out + i, &dummy);
}

int cmp_ent(const void *a, const void *b) {
    typedef struct { float dsq; unsigned ord; float r, t; } ent;
    const ent *x = (const ent *)a, *y = (const ent *)b;
    if (x->dsq < y->dsq) return -1;
    if (x->dsq > y->dsq) return 1;
    return x->ord < y->ord ? -1 : x->ord > y->ord ? 1 : 0;
}

/* ---- per-channel driver, multipole.cpp:241-295 ---- */
typedef struct {
    const float (*mua)[O_NB];
    const float (*musp)[O_NB];
    const float *eta, *thick;
    int desired, lerp;
    float *tables[O_NB];
    int lens[O_NB];
    float rcp[O_NB], spacing[O_NB], tr[O_NB];
    int next;
    pthread_mutex_t mu;
} prof_job;

static void prof_channel(prof_job *j, int sc) {
    float mfp_total = 0.f;
    for (int l = 0; l < 2; ++l) mfp_total += 1.f / (j->mua[l][sc] + j->musp[l][sc]);
    float mfp = mfp_total / (float)2;
    o_layer_spec ls[2];
    for (int l = 0; l < 2; ++l) {
        ls[l].ior = j->eta[l];
        ls[l].mua = j->mua[l][sc];
        ls[l].musp = j->musp[l][sc];
        ls[l].thickness = j->thick[l];
    }
    float step = 12.f * mfp / (float)j->desired;
    float *d, *r, *t, trr, ttt;
    int len = o_mpc_profile(2, ls, step, j->desired, j->lerp, 1, &d, &r, &t, &trr, &ttt);
    j->spacing[sc] = d[len - 1] / (float)(len - 1);
    j->rcp[sc] = (float)(len - 1) / d[len - 1];
    j->tr[sc] = trr;
    j->tables[sc] = r;
    j->lens[sc] = len;
    free(d);
    free(t);
}

static void *prof_worker(void *arg) {
    prof_job *j = (prof_job *)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        int sc = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (sc >= O_NB) break;
        prof_channel(j, sc);
    }
    return NULL;
}

int o_compute_profile(const float mua[2][O_NB], const float musp[2][O_NB], const float eta[2],
                      const float thickness[2], int desired_length, int lerp_thin, int nthreads,
                      float **table, float rcp[O_NB], float spacing[O_NB], float total_r[O_NB]) {
    prof_job j;
    memset(&j, 0, sizeof(j));
    j.mua = mua; j.musp = musp; j.eta = eta; j.thick = thickness;
    j.desired = desired_length; j.lerp = lerp_thin;
    pthread_mutex_init(&j.mu, NULL);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    pthread_t th[64];
    for (int i = 0; i < nthreads; ++i) pthread_create(&th[i], NULL, prof_worker, &j);
    for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
    pthread_mutex_destroy(&j.mu);
    int len = j.lens[0];
    for (int c = 1; c < O_NB; ++c)
        if (j.lens[c] != len) return -1; /* every channel has the same entry count (same grid) */
    float *tab = (float *)malloc(sizeof(float) * (size_t)O_NB * len);
    for (int c = 0; c < O_NB; ++c) {
        memcpy(tab + (size_t)c * len, j.tables[c], sizeof(float) * len);
        free(j.tables[c]);
        rcp[c] = j.rcp[c];
        spacing[c] = j.spacing[c];
        total_r[c] = j.tr[c];
    }
    *table = tab;
    return len;
}

/* sampleProfile, multipole.cpp:60-73.  Note: distanceSquared * rcpDsqSpacing is a float
 * product (both operands float) that is then widened to double. */
float o_sample_profile(const float *data, int len, float rcp, float dsq) {
    double f = (double)(dsq * rcp);
    if (f >= (double)(len - 1)) return 0.f;
    unsigned s = (unsigned)f;
    float t = (float)(f - (double)s);
    return (1.f - t) * data[s] + t * data[s + 1];
}
