// mc_profile.hip -- ProfileRendererTask::TraceSinglePhoton (reference src/renderers/
// mcprofile.cpp:229-326) as a persistent-lane GPU kernel, plus the host driver that normalises
// the tallies like MonteCarloProfileRenderer::Render (:482-533).
//
// Each lane owns one photon at a time and advances it one event per loop trip (a free-flight
// sample ends either in a scatter inside the layer or on an interface). A lane whose photon
// has finished takes the next photon id from a global counter (one atomic per wave), so lanes
// stay busy however long individual random walks run. Ring tallies accumulate in LDS doubles
// (ds_add_f64) and are flushed to HBM once per workgroup. All arithmetic is FP64 as in the
// reference (DVector / DRay / DPoint, mcprofile.cpp:46-49).
#include "mc_profile.h"
#include "material.h"

#include <algorithm>
#include <cstring>
#include <vector>

namespace mpss {

namespace {

constexpr int kMcMaxSegments = 4096;
constexpr int kMcPool = 256;  // photon ids a wave takes from the global counter at a time  // ComputeMonteCarloProfile tallies 4096 rings (multipole.cpp:322)
// pbrt's M_PI is the float literal 3.14159265358979323846f (core/pbrt.h:193-196); the walk and the
// ring normalisation use it widened to double
constexpr double kPbrtPi = (double)3.14159265358979323846f;

// UniformSampleSphereD (mcprofile.cpp:51-58); u1 is drawn before u2
__device__ __forceinline__ void sample_sphere_d(double u1, double u2, double &x, double &y, double &z) {
    z = 1. - 2. * u1;
    const double r = sqrt(fmax(0., 1. - z * z));
    const double phi = 2. * kPbrtPi * u2;
    double sp, cp;
    sincos(phi, &sp, &cp);  // one range reduction for both (the same values as cos / sin)
    x = r * cp;
    y = r * sp;
}

// FrDiel<double> (core/reflection.cpp:72-80) with etat = 1
__device__ __forceinline__ double fr_diel_d(double cosi, double cost, double etai, double etat) {
    const double rparl = ((etat * cosi) - (etai * cost)) / ((etat * cosi) + (etai * cost));
    const double rperp = ((etai * cosi) - (etat * cost)) / ((etai * cosi) + (etat * cost));
    return (rparl * rparl + rperp * rperp) / 2.;
}

struct McArgs {
    McScene sc;
    uint64_t nphotons, seed;
    unsigned long long *next;  // photon counter
    double *refl, *trans;      // [nsegments] global tallies
    unsigned long long *events;  // nullable: total free-flight events
};

template <int NSEG>
__global__ __launch_bounds__(256) void mc_profile_kernel(McArgs a) {
    __shared__ double h_r[NSEG], h_t[NSEG];
    const McScene &sc = a.sc;
    for (int i = threadIdx.x; i < sc.nsegments; i += blockDim.x) h_r[i] = h_t[i] = 0.;
    __syncthreads();
    const int lane = (int)(threadIdx.x & 63);
    bool alive = false, exhausted = false;
    double ox = 0., oy = 0., oz = 0., dx = 0., dy = 0., dz = 1.;
    double thr = 1., len = 0., mfp = 1.;
    int layer = 0;
    McRng rng;
    rng.s = 0;
    unsigned long long nev = 0;
    // the wave's own run of photon ids [pool, pool + pool_left), taken kMcPool at a time from the
    // global counter: one atomic per kMcPool photons instead of one per refill (photons finish one
    // by one, and a single counter serves only ~1e8 atomics/s)
    uint64_t pool = 0;
    int pool_left = 0;
    for (;;) {
        // refill lanes whose photon has finished
        if (!exhausted) {
            const uint64_t need = __builtin_amdgcn_ballot_w64(!alive);
            if (need) {
                if (pool_left == 0) {
                    unsigned long long base = 0;
                    if (lane == 0) base = atomicAdd(a.next, (unsigned long long)kMcPool);
                    base = __shfl(base, 0);
                    pool = base;
                    pool_left = base < a.nphotons ? (int)(a.nphotons - base < (uint64_t)kMcPool ? a.nphotons - base
                                                                                                 : (uint64_t)kMcPool)
                                                  : 0;
                    if (pool_left == 0) exhausted = true;
                }
                const int rank = __builtin_popcountll(need & ((1ull << lane) - 1ull));
                if (!alive && rank < pool_left) {
                    const uint64_t id = pool + (uint64_t)rank;
                    {
                        // TraceSinglePhoton setup (:233-241), then the outer loop's head (:245-248)
                        rng.init(a.seed, id);
                        ox = oy = oz = 0.;
                        dx = dy = 0.;
                        dz = 1.;
                        thr = 1.;
                        len = 0.;
                        layer = 0;
                        mfp = sc.mfp[0];
                        len *= mfp;
                        alive = true;
                    }
                }
                const int used = __builtin_popcountll(need) < pool_left ? __builtin_popcountll(need) : pool_left;
                pool += (uint64_t)used;
                pool_left -= used;
            }
        }
        if (__builtin_amdgcn_ballot_w64(alive) == 0) break;
        if (!alive) continue;
        ++nev;
        const McLayer &L = sc.layer[layer];
        // free flight (:251-252)
        if (len == 0.) len = fmin(-log((double)1.f - rng.next()), 1e7) * mfp;
        // MiniScene::Intersect (:153-185) with maxt = len
        bool hit = false;
        int iface = 0;
        double t = 0., inv = 1.;
        const double ct = dz;
        if (ct != 0.) {
            if (dz > 0.) {
                const double nd = sc.depth[layer + 1];
                if (nd - oz < ct * len) {
                    hit = true;
                    iface = layer + 1;
                    t = (nd - oz) / ct;
                    inv = sc.eta_dn[layer];
                }
            } else {
                const double nd = sc.depth[layer];
                if (nd - oz > ct * len) {
                    hit = true;
                    iface = layer;
                    t = (nd - oz) / ct;
                    inv = sc.eta_up[layer];
                }
            }
        }
        // the step's attenuation: to the interface (a hit) or over the free flight (a scatter) --
        // one exp for the wave, whichever branch each lane takes
        double px = 0., py = 0., pz = 0., dist = 0.;
        if (hit) {
            px = ox + dx * t;
            py = oy + dy * t;
            pz = oz + dz * t;
            const double ex = px - ox, ey = py - oy, ez = pz - oz;
            dist = sqrt(ex * ex + ey * ey + ez * ez);
        }
        thr *= exp((double)-L.mua * (hit ? dist : len));
        if (hit) {
            len = fmax(1e-7 * mfp, len - dist);
            const double cosi = fmin(fmax(dz, -1.), 1.);
            const bool up = dz < 0.;
            const double sint2 = (1. - cosi * cosi) * inv * inv;
            double cost = 0.;
            bool reflect;
            if (sint2 >= 1.) {
                reflect = true;  // total internal reflection
            } else {
                cost = sqrt(fmax(0., 1. - sint2));
                const double F = fr_diel_d(fabs(cosi), cost, inv, 1.);
                reflect = rng.next() < F;
            }
            int target = layer;
            if (reflect) {
                dz = -dz;
            } else {
                target = up ? layer - 1 : layer + 1;
                dx = inv * dx;
                dy = inv * dy;
                dz = up ? -cost : cost;
            }
            ox = px;
            oy = py;
            oz = pz;
            if (target != layer) {
                // book-keeping (:303-316)
                if (iface == 0 || iface == sc.nlayers) {
                    const double rd = sqrt(px * px + py * py + 0. * 0.);
                    const int seg = (int)(rd * sc.nsegments / sc.extent);
                    if (rd < sc.extent && seg < sc.nsegments) atomicAdd(iface == 0 ? &h_r[seg] : &h_t[seg], thr);
                }
                // outer loop tail (:330-340): roulette, then remaining length in the old layer's mfp units
                bool dead = false;
                if (thr < 1e-5) {
                    const double q = thr * 1e5;
                    if (rng.next() > q)
                        dead = true;
                    else
                        thr /= q;
                }
                if (!dead) {
                    len *= (double)L.musp;
                    layer = target;
                    if (layer < 0 || layer >= sc.nlayers) {
                        dead = true;
                    } else {
                        mfp = sc.mfp[layer];  // next outer loop's head
                        len *= mfp;
                    }
                }
                if (dead) alive = false;
            }
        } else {
            // scatter inside the layer (:319-327)
            ox = ox + dx * len;
            oy = oy + dy * len;
            oz = oz + dz * len;
            len = 0.;
            const double u1 = rng.next(), u2 = rng.next();
            sample_sphere_d(u1, u2, dx, dy, dz);
        }
    }
    if (a.events) atomicAdd(a.events, nev);
    __syncthreads();
    for (int i = threadIdx.x; i < sc.nsegments; i += blockDim.x) {
        if (h_r[i] != 0.) atomicAdd(&a.refl[i], h_r[i]);
        if (h_t[i] != 0.) atomicAdd(&a.trans[i], h_t[i]);
    }
}

}  // namespace

McScene make_mc_scene(const McLayer *layers, int n, double mfp_range, int nsegments) {
    if (n < 1 || n > kMcMaxLayers) throw Error(-1, "mc_profile: 1..8 layers supported");
    if (nsegments < 1 || nsegments > kMcMaxSegments) throw Error(-1, "mc_profile: 1..4096 segments supported");
    McScene sc{};
    sc.nlayers = n;
    double depth = 0., mfp_total = 0.;
    sc.depth[0] = 0.;
    for (int i = 0; i < n; ++i) {
        if (!(layers[i].musp > 0.f) || !(layers[i].mua >= 0.f) || !(layers[i].thickness > 0.f))
            throw Error(-1, "mc_profile: layers need musp > 0, mua >= 0, thickness > 0");
        sc.layer[i] = layers[i];
        sc.depth[i + 1] = depth += (double)layers[i].thickness;
        mfp_total += 1. / (double)(layers[i].mua + layers[i].musp);  // float sum (Render :458-460)
    }
    sc.extent = mfp_range * (mfp_total / (double)n);
    sc.nsegments = nsegments;
    for (int i = 0; i < n; ++i) {
        sc.mfp[i] = 1. / (double)layers[i].musp;
        sc.eta_dn[i] = (double)layers[i].ior / (i + 1 == n ? 1. : (double)layers[i + 1].ior);
        sc.eta_up[i] = (double)layers[i].ior / (i == 0 ? 1. : (double)layers[i - 1].ior);
    }
    return sc;
}

void run_mc_profile(const McScene &sc, uint64_t nphotons, uint64_t seed, double *refl, double *trans,
                    double *total_r, double *total_t, uint64_t *events, hipStream_t stream) {
    DevBuf<double> d_r, d_t;
    DevBuf<unsigned long long> d_cnt;
    d_r.alloc(sc.nsegments);
    d_t.alloc(sc.nsegments);
    d_cnt.alloc(2);
    MPSS_HIP(hipMemsetAsync(d_r.ptr, 0, sizeof(double) * sc.nsegments, stream));
    MPSS_HIP(hipMemsetAsync(d_t.ptr, 0, sizeof(double) * sc.nsegments, stream));
    MPSS_HIP(hipMemsetAsync(d_cnt.ptr, 0, sizeof(unsigned long long) * 2, stream));
    McArgs a{sc, nphotons, seed, d_cnt.ptr, d_r.ptr, d_t.ptr, d_cnt.ptr + 1};
    int dev = 0, ncu = 0;
    MPSS_HIP(hipGetDevice(&dev));
    MPSS_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    const uint64_t lanes_needed = (nphotons + 255) / 256;
    const unsigned blocks = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)ncu * 8, lanes_needed));
    // LDS ring tallies: 32 KB up to 2048 rings; 64 KB for ComputeMonteCarloProfile's 4096
    if (nphotons > 0) {
        if (sc.nsegments <= 2048)
            hipLaunchKernelGGL(mc_profile_kernel<2048>, dim3(blocks), dim3(256), 0, stream, a);
        else
            hipLaunchKernelGGL(mc_profile_kernel<kMcMaxSegments>, dim3(blocks), dim3(256), 0, stream, a);
    }
    MPSS_HIP(hipGetLastError());
    std::vector<double> r(sc.nsegments), t(sc.nsegments);
    unsigned long long cnt[2];
    MPSS_HIP(hipMemcpyAsync(r.data(), d_r.ptr, sizeof(double) * sc.nsegments, hipMemcpyDeviceToHost, stream));
    MPSS_HIP(hipMemcpyAsync(t.data(), d_t.ptr, sizeof(double) * sc.nsegments, hipMemcpyDeviceToHost, stream));
    MPSS_HIP(hipMemcpyAsync(cnt, d_cnt.ptr, sizeof(cnt), hipMemcpyDeviceToHost, stream));
    MPSS_HIP(hipStreamSynchronize(stream));
    // normalise by photons and ring area (Render, :482-498)
    double tr = 0., tt = 0.;
    for (int i = 0; i < sc.nsegments; ++i) {
        const double sum = (double)(2 * i + 1) * sc.extent / sc.nsegments;
        const double h = sc.extent / sc.nsegments;
        const double area = kPbrtPi * sum * h;
        const double factor = (double)nphotons * area;
        tr += r[i];
        tt += t[i];
        refl[i] = r[i] / factor;
        trans[i] = t[i] / factor;
    }
    *total_r = tr / (double)nphotons;
    *total_t = tt / (double)nphotons;
    if (events) *events = cnt[1];
}

void build_profile_mc(const LayerParams &lp, uint64_t photons, uint64_t seed, ProfileTables &out) {
    constexpr int kSegments = 4096;        // multipole.cpp:318
    constexpr double kMfpRange = 12.0f;    // :319
    constexpr int kTarget = kSegments * 16;  // :341
    std::vector<double> refl(kSegments), trans(kSegments);
    out.length = kTarget;
    out.table.resize((size_t)NB * kTarget);
    std::vector<float> tab;
    for (int c = 0; c < NB; ++c) {
        McLayer l[2];
        for (int k = 0; k < 2; ++k) l[k] = McLayer{lp.mua[k][c], lp.musp[k][c], lp.eta[k], lp.thickness[k]};
        const McScene sc = make_mc_scene(l, 2, kMfpRange, kSegments);
        double tr = 0., tt = 0.;
        // every band walks the same photon streams, as every band's MonteCarloProfileRenderer
        // seeds its tasks alike (RNG(89 * taskId), mcprofile.cpp:223)
        run_mc_profile(sc, photons, seed, refl.data(), trans.data(), &tr, &tt, nullptr, nullptr);
        profile_from_rings(refl.data(), kSegments, sc.extent, kTarget, tab, out.rcp[c], out.spacing[c]);
        out.total_reflectance[c] = (float)tr;
        std::copy(tab.begin(), tab.end(), out.table.begin() + (size_t)c * kTarget);
    }
}

}  // namespace mpss
