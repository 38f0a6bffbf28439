/* oracle/kissfft.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 * Restatement of the vendored kissfft v1.3.0 (reference src/multipole/libkissfft,
 * kiss_fft_scalar forced to double at kiss_fft.h:48) for the sizes the MPC uses:
 * mixed-radix recursive decimation (kiss_fft.c kf_work / kf_factor), radix-2/3/4/5
 * and generic butterflies, the packed real transform (tools/kiss_fftr.c) and the
 * 2-D real driver (tools/kiss_fftndr.c + tools/kiss_fftnd.c for one complex dim).
 * Same operation order as the reference so results are bit-identical in IEEE double. */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

#define MAXF 32
typedef struct {
    int nfft, inverse;
    int factors[2 * MAXF];
    o_cpx *tw;
} kcfg;

static void cmul(o_cpx *m, o_cpx a, o_cpx b) {
    m->r = a.r * b.r - a.i * b.i;
    m->i = a.r * b.i + a.i * b.r;
}

/* kiss_fft.c kf_factor */
static void kf_factor(int n, int *fb) {
    int p = 4;
    double fs = floor(sqrt((double)n));
    do {
        while (n % p) {
            switch (p) {
            case 4: p = 2; break;
            case 2: p = 3; break;
            default: p += 2; break;
            }
            if (p > fs) p = n;
        }
        n /= p;
        *fb++ = p;
        *fb++ = n;
    } while (n > 1);
}

static void kcfg_init(kcfg *st, int nfft, int inverse) {
    st->nfft = nfft;
    st->inverse = inverse;
    st->tw = (o_cpx *)malloc(sizeof(o_cpx) * nfft);
    for (int i = 0; i < nfft; ++i) {
        const double pi = 3.141592653589793238462643383279502884197169399375105820974944;
        double phase = -2 * pi * i / nfft;
        if (inverse) phase *= -1;
        st->tw[i].r = cos(phase);
        st->tw[i].i = sin(phase);
    }
    kf_factor(nfft, st->factors);
}

static void bfly2(o_cpx *F, size_t fs, const kcfg *st, int m) {
    o_cpx *F2 = F + m, *tw1 = st->tw, t;
    do {
        cmul(&t, *F2, *tw1);
        tw1 += fs;
        F2->r = F->r - t.r; F2->i = F->i - t.i;
        F->r += t.r; F->i += t.i;
        ++F2; ++F;
    } while (--m);
}

static void bfly4(o_cpx *F, size_t fs, const kcfg *st, size_t m) {
    o_cpx *tw1, *tw2, *tw3, s[6];
    size_t k = m, m2 = 2 * m, m3 = 3 * m;
    tw3 = tw2 = tw1 = st->tw;
    do {
        cmul(&s[0], F[m], *tw1);
        cmul(&s[1], F[m2], *tw2);
        cmul(&s[2], F[m3], *tw3);
        s[5].r = F->r - s[1].r; s[5].i = F->i - s[1].i;
        F->r += s[1].r; F->i += s[1].i;
        s[3].r = s[0].r + s[2].r; s[3].i = s[0].i + s[2].i;
        s[4].r = s[0].r - s[2].r; s[4].i = s[0].i - s[2].i;
        F[m2].r = F->r - s[3].r; F[m2].i = F->i - s[3].i;
        tw1 += fs; tw2 += fs * 2; tw3 += fs * 3;
        F->r += s[3].r; F->i += s[3].i;
        if (st->inverse) {
            F[m].r = s[5].r - s[4].i; F[m].i = s[5].i + s[4].r;
            F[m3].r = s[5].r + s[4].i; F[m3].i = s[5].i - s[4].r;
        } else {
            F[m].r = s[5].r + s[4].i; F[m].i = s[5].i - s[4].r;
            F[m3].r = s[5].r - s[4].i; F[m3].i = s[5].i + s[4].r;
        }
        ++F;
    } while (--k);
}

static void bfly3(o_cpx *F, size_t fs, const kcfg *st, size_t m) {
    size_t k = m, m2 = 2 * m;
    o_cpx *tw1, *tw2, s[5], epi3 = st->tw[fs * m];
    tw1 = tw2 = st->tw;
    do {
        cmul(&s[1], F[m], *tw1);
        cmul(&s[2], F[m2], *tw2);
        s[3].r = s[1].r + s[2].r; s[3].i = s[1].i + s[2].i;
        s[0].r = s[1].r - s[2].r; s[0].i = s[1].i - s[2].i;
        tw1 += fs; tw2 += fs * 2;
        F[m].r = F->r - s[3].r * .5f;
        F[m].i = F->i - s[3].i * .5f;
        s[0].r *= epi3.i; s[0].i *= epi3.i;
        F->r += s[3].r; F->i += s[3].i;
        F[m2].r = F[m].r + s[0].i; F[m2].i = F[m].i - s[0].r;
        F[m].r -= s[0].i; F[m].i += s[0].r;
        ++F;
    } while (--k);
}

static void bfly5(o_cpx *F, size_t fs, const kcfg *st, int m) {
    o_cpx *F0 = F, *F1 = F + m, *F2 = F + 2 * m, *F3 = F + 3 * m, *F4 = F + 4 * m;
    o_cpx s[13], *tw = st->tw, ya = tw[fs * m], yb = tw[fs * 2 * m];
    for (int u = 0; u < m; ++u) {
        s[0] = *F0;
        cmul(&s[1], *F1, tw[u * fs]);
        cmul(&s[2], *F2, tw[2 * u * fs]);
        cmul(&s[3], *F3, tw[3 * u * fs]);
        cmul(&s[4], *F4, tw[4 * u * fs]);
        s[7].r = s[1].r + s[4].r; s[7].i = s[1].i + s[4].i;
        s[10].r = s[1].r - s[4].r; s[10].i = s[1].i - s[4].i;
        s[8].r = s[2].r + s[3].r; s[8].i = s[2].i + s[3].i;
        s[9].r = s[2].r - s[3].r; s[9].i = s[2].i - s[3].i;
        F0->r += s[7].r + s[8].r;
        F0->i += s[7].i + s[8].i;
        s[5].r = s[0].r + s[7].r * ya.r + s[8].r * yb.r;
        s[5].i = s[0].i + s[7].i * ya.r + s[8].i * yb.r;
        s[6].r = s[10].i * ya.i + s[9].i * yb.i;
        s[6].i = -(s[10].r * ya.i) - s[9].r * yb.i;
        F1->r = s[5].r - s[6].r; F1->i = s[5].i - s[6].i;
        F4->r = s[5].r + s[6].r; F4->i = s[5].i + s[6].i;
        s[11].r = s[0].r + s[7].r * yb.r + s[8].r * ya.r;
        s[11].i = s[0].i + s[7].i * yb.r + s[8].i * ya.r;
        s[12].r = -(s[10].i * yb.i) + s[9].i * ya.i;
        s[12].i = s[10].r * yb.i - s[9].r * ya.i;
        F2->r = s[11].r + s[12].r; F2->i = s[11].i + s[12].i;
        F3->r = s[11].r - s[12].r; F3->i = s[11].i - s[12].i;
        ++F0; ++F1; ++F2; ++F3; ++F4;
    }
}

static void bfly_generic(o_cpx *F, size_t fs, const kcfg *st, int m, int p) {
    o_cpx *tw = st->tw, t;
    int No = st->nfft;
    o_cpx *sc = (o_cpx *)malloc(sizeof(o_cpx) * p);
    for (int u = 0; u < m; ++u) {
        int k = u;
        for (int q1 = 0; q1 < p; ++q1) { sc[q1] = F[k]; k += m; }
        k = u;
        for (int q1 = 0; q1 < p; ++q1) {
            int twidx = 0;
            F[k] = sc[0];
            for (int q = 1; q < p; ++q) {
                twidx += (int)(fs * k);
                if (twidx >= No) twidx -= No;
                cmul(&t, sc[q], tw[twidx]);
                F[k].r += t.r; F[k].i += t.i;
            }
            k += m;
        }
    }
    free(sc);
}

/* kiss_fft.c kf_work (non-OpenMP path) */
static void kf_work(o_cpx *Fout, const o_cpx *f, size_t fs, int in_stride, const int *factors,
                    const kcfg *st) {
    o_cpx *Fbeg = Fout;
    const int p = *factors++;
    const int m = *factors++;
    const o_cpx *Fend = Fout + p * m;
    if (m == 1) {
        do {
            *Fout = *f;
            f += fs * in_stride;
        } while (++Fout != Fend);
    } else {
        do {
            kf_work(Fout, f, fs * p, in_stride, factors, st);
            f += fs * in_stride;
        } while ((Fout += m) != Fend);
    }
    Fout = Fbeg;
    switch (p) {
    case 2: bfly2(Fout, fs, st, m); break;
    case 3: bfly3(Fout, fs, st, m); break;
    case 4: bfly4(Fout, fs, st, m); break;
    case 5: bfly5(Fout, fs, st, m); break;
    default: bfly_generic(Fout, fs, st, m, p); break;
    }
}

static void kfft(const kcfg *st, const o_cpx *fin, o_cpx *fout) {
    if (fin == fout) {
        o_cpx *tmp = (o_cpx *)malloc(sizeof(o_cpx) * st->nfft);
        kf_work(tmp, fin, 1, 1, st->factors, st);
        memcpy(fout, tmp, sizeof(o_cpx) * st->nfft);
        free(tmp);
    } else
        kf_work(fout, fin, 1, 1, st->factors, st);
}

void o_kiss_fft(int nfft, int inverse, const o_cpx *fin, o_cpx *fout) {
    kcfg st;
    kcfg_init(&st, nfft, inverse);
    kfft(&st, fin, fout);
    free(st.tw);
}

/* tools/kiss_fftr.c */
typedef struct {
    kcfg sub;
    o_cpx *tmp, *super;
} krcfg;

static void krcfg_init(krcfg *st, int nfft, int inverse) {
    nfft >>= 1;
    kcfg_init(&st->sub, nfft, inverse);
    st->tmp = (o_cpx *)malloc(sizeof(o_cpx) * nfft);
    st->super = (o_cpx *)malloc(sizeof(o_cpx) * (nfft / 2));
    for (int i = 0; i < nfft / 2; ++i) {
        double phase = -3.14159265358979323846264338327 * ((double)(i + 1) / nfft + .5);
        if (inverse) phase *= -1;
        st->super[i].r = cos(phase);
        st->super[i].i = sin(phase);
    }
}
static void krcfg_free(krcfg *st) {
    free(st->sub.tw);
    free(st->tmp);
    free(st->super);
}

static void kfftr(krcfg *st, const double *td, o_cpx *fd) {
    int ncfft = st->sub.nfft;
    kfft(&st->sub, (const o_cpx *)td, st->tmp);
    o_cpx tdc = st->tmp[0];
    fd[0].r = tdc.r + tdc.i;
    fd[ncfft].r = tdc.r - tdc.i;
    fd[ncfft].i = fd[0].i = 0;
    for (int k = 1; k <= ncfft / 2; ++k) {
        o_cpx fpk = st->tmp[k], fpnk, f1k, f2k, tw;
        fpnk.r = st->tmp[ncfft - k].r;
        fpnk.i = -st->tmp[ncfft - k].i;
        f1k.r = fpk.r + fpnk.r; f1k.i = fpk.i + fpnk.i;
        f2k.r = fpk.r - fpnk.r; f2k.i = fpk.i - fpnk.i;
        cmul(&tw, f2k, st->super[k - 1]);
        fd[k].r = (f1k.r + tw.r) * .5f;
        fd[k].i = (f1k.i + tw.i) * .5f;
        fd[ncfft - k].r = (f1k.r - tw.r) * .5f;
        fd[ncfft - k].i = (tw.i - f1k.i) * .5f;
    }
}

static void kfftri(krcfg *st, const o_cpx *fd, double *td) {
    int ncfft = st->sub.nfft;
    st->tmp[0].r = fd[0].r + fd[ncfft].r;
    st->tmp[0].i = fd[0].r - fd[ncfft].r;
    for (int k = 1; k <= ncfft / 2; ++k) {
        o_cpx fk = fd[k], fnkc, fek, fok, tmp;
        fnkc.r = fd[ncfft - k].r;
        fnkc.i = -fd[ncfft - k].i;
        fek.r = fk.r + fnkc.r; fek.i = fk.i + fnkc.i;
        tmp.r = fk.r - fnkc.r; tmp.i = fk.i - fnkc.i;
        cmul(&fok, tmp, st->super[k - 1]);
        st->tmp[k].r = fek.r + fok.r; st->tmp[k].i = fek.i + fok.i;
        st->tmp[ncfft - k].r = fek.r - fok.r; st->tmp[ncfft - k].i = fek.i - fok.i;
        st->tmp[ncfft - k].i *= -1;
    }
    kfft(&st->sub, st->tmp, (o_cpx *)td);
}

/* tools/kiss_fftndr.c kiss_fftndr for dims = {rows, cols} */
void o_kiss_fftndr2(int rows, int cols, const double *in, o_cpx *out) {
    int nrbins = cols / 2 + 1;
    krcfg r;
    kcfg c;
    krcfg_init(&r, cols, 0);
    kcfg_init(&c, rows, 0);
    o_cpx *tmp1 = (o_cpx *)malloc(sizeof(o_cpx) * (nrbins > rows ? nrbins : rows));
    o_cpx *tmp2 = (o_cpx *)malloc(sizeof(o_cpx) * (size_t)rows * nrbins);
    for (int k1 = 0; k1 < rows; ++k1) {
        kfftr(&r, in + (size_t)k1 * cols, tmp1);
        for (int k2 = 0; k2 < nrbins; ++k2) tmp2[(size_t)k2 * rows + k1] = tmp1[k2];
    }
    for (int k2 = 0; k2 < nrbins; ++k2) {
        kfft(&c, tmp2 + (size_t)k2 * rows, tmp1);
        for (int k1 = 0; k1 < rows; ++k1) out[(size_t)k1 * nrbins + k2] = tmp1[k1];
    }
    free(tmp1);
    free(tmp2);
    krcfg_free(&r);
    free(c.tw);
}

/* tools/kiss_fftndr.c kiss_fftndri */
void o_kiss_fftndri2(int rows, int cols, const o_cpx *in, double *out) {
    int nrbins = cols / 2 + 1;
    krcfg r;
    kcfg c;
    krcfg_init(&r, cols, 1);
    kcfg_init(&c, rows, 1);
    o_cpx *tmp1 = (o_cpx *)malloc(sizeof(o_cpx) * (nrbins > rows ? nrbins : rows));
    o_cpx *tmp2 = (o_cpx *)malloc(sizeof(o_cpx) * (size_t)rows * nrbins);
    for (int k2 = 0; k2 < nrbins; ++k2) {
        for (int k1 = 0; k1 < rows; ++k1) tmp1[k1] = in[(size_t)k1 * nrbins + k2];
        kfft(&c, tmp1, tmp2 + (size_t)k2 * rows);
    }
    for (int k1 = 0; k1 < rows; ++k1) {
        for (int k2 = 0; k2 < nrbins; ++k2) tmp1[k2] = tmp2[(size_t)k2 * rows + k1];
        kfftri(&r, tmp1, out + (size_t)k1 * cols);
    }
    free(tmp1);
    free(tmp2);
    krcfg_free(&r);
    free(c.tw);
}
