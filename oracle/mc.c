/*
 * mc.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Scalar restatement of the Monte-Carlo layered profile renderer:
 *   MiniScene::Intersect            src/renderers/mcprofile.cpp:153-185
 *   TraceSinglePhoton               src/renderers/mcprofile.cpp:236-327
 *   MonteCarloProfileRenderer::Render normalisation  :455-498
 * in FP64 like the reference (DVector/DPoint/DRay). Random numbers come from the same
 * per-photon splitmix64 streams as the product (replay mode); u1 is drawn before u2 in
 * UniformSampleSphereD.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

typedef struct { uint64_t s; } rng_t;
static void rng_init(rng_t *r, uint64_t seed, uint64_t photon) { r->s = mix64(seed * 0x9e3779b97f4a7c15ull ^ mix64(photon)); }
static double rng_next(rng_t *r) {
    r->s += 0x9e3779b97f4a7c15ull;
    return (double)(mix64(r->s) >> 11) * 0x1p-53;
}

static double frdiel(double cosi, double cost, double etai, double etat) {
    double rparl = ((etat * cosi) - (etai * cost)) / ((etat * cosi) + (etai * cost));
    double rperp = ((etai * cosi) - (etat * cost)) / ((etai * cosi) + (etat * cost));
    return (rparl * rparl + rperp * rperp) / 2.;
}

int o_mc_profile(const o_mc_layer *layers, int n, float mfp_range, int nseg, uint64_t nphotons, uint64_t seed,
                 uint64_t photon_begin, uint64_t photon_end, double *raw_r, double *raw_t, double *extent_out) {
    if (n < 1 || nseg < 1) return -1;
    double depth[65];
    double d = 0., mfp_total = 0.;
    depth[0] = 0.;
    for (int i = 0; i < n && i < 64; ++i) {
        depth[i + 1] = d += (double)layers[i].thickness;
        mfp_total += 1. / (double)(layers[i].mua + layers[i].musp); /* float sum (mcprofile.cpp:458-460) */
    }
    const double extent = mfp_range * (mfp_total / (double)n);
    if (extent_out) *extent_out = extent;
    for (uint64_t id = photon_begin; id < photon_end && id < nphotons; ++id) {
        rng_t rng;
        rng_init(&rng, seed, id);
        double ox = 0., oy = 0., oz = 0., dx = 0., dy = 0., dz = 1.;
        int cur = 0;
        double thr = 1., len = 0.;
        while (cur >= 0 && cur < n) {
            const o_mc_layer *L = &layers[cur];
            int target = cur;
            double smfp = 1. / L->musp;
            len *= smfp;
            do {
                if (len == 0.) len = fmin(-log((double)1.f - rng_next(&rng)), 1e7) * smfp;
                /* MiniScene::Intersect with ray.maxt = len */
                int hit = 0, iface = 0;
                double t = 0., inv = 1.;
                double ct = dz;
                if (ct != 0.) {
                    if (dz > 0.) {
                        double nd = depth[cur + 1];
                        if (nd - oz < ct * len) {
                            hit = 1;
                            iface = cur + 1;
                            t = (nd - oz) / ct;
                            double nior = (cur + 1 == n) ? 1. : (double)layers[cur + 1].ior;
                            inv = (double)L->ior / nior;
                        }
                    } else {
                        double nd = depth[cur];
                        if (nd - oz > ct * len) {
                            hit = 1;
                            iface = cur;
                            t = (nd - oz) / ct;
                            double nior = (cur == 0) ? 1. : (double)layers[cur - 1].ior;
                            inv = (double)L->ior / nior;
                        }
                    }
                }
                if (hit) {
                    double px = ox + dx * t, py = oy + dy * t, pz = oz + dz * t;
                    double ex = px - ox, ey = py - oy, ez = pz - oz;
                    double dist = sqrt(ex * ex + ey * ey + ez * ez);
                    thr *= exp((double)-L->mua * dist);
                    len = fmax(1e-7 * smfp, len - dist);
                    double cosi = fmin(fmax(dz, -1.), 1.);
                    int up = dz < 0.;
                    double sint2 = (1. - cosi * cosi) * inv * inv;
                    double cost = 0.;
                    int reflect;
                    if (sint2 >= 1.) {
                        reflect = 1;
                    } else {
                        cost = sqrt(fmax(0., 1. - sint2));
                        double F = frdiel(fabs(cosi), cost, inv, 1.);
                        reflect = rng_next(&rng) < F;
                    }
                    if (reflect) {
                        dz = -dz;
                    } else {
                        target = up ? cur - 1 : cur + 1;
                        dx = inv * dx;
                        dy = inv * dy;
                        dz = up ? -cost : cost;
                    }
                    ox = px;
                    oy = py;
                    oz = pz;
                    if (cur != target) {
                        if (iface == 0 || iface == n) {
                            double rd = sqrt(px * px + py * py + 0. * 0.);
                            int seg = (int)(rd * nseg / extent);
                            if (rd < extent && seg < nseg) {
                                if (iface == 0) raw_r[seg] += thr;
                                else raw_t[seg] += thr;
                            }
                        }
                    }
                } else {
                    ox = ox + dx * len;
                    oy = oy + dy * len;
                    oz = oz + dz * len;
                    thr *= exp((double)-L->mua * len);
                    len = 0.;
                    double u1 = rng_next(&rng), u2 = rng_next(&rng);
                    double z = 1. - 2. * u1;
                    double r = sqrt(fmax(0., 1. - z * z));
                    double phi = 2. * (double)3.14159265358979323846f * u2; /* pbrt's float M_PI (pbrt.h:196) */
                    dx = r * cos(phi);
                    dy = r * sin(phi);
                    dz = z;
                }
            } while (cur == target);
            cur = target;
            if (thr < 1e-5) {
                double q = thr * 1e5;
                if (rng_next(&rng) > q) break;
                thr /= q;
            }
            len *= L->musp;
        }
    }
    return 0;
}
