// replay_gen.hip -- the reference sampler's values for one window of the sample extent, on the
// GPU (replay.h; render.h ReplayWindow). pbrt draws a task's samples from one sequential MT19937
// stream, so a task cannot be split across lanes; it is split across the stream instead: one wave
// per task, its 624-word state in LDS, the lanes twisting, tempering and consuming the stream's
// draws together and computing the camera samples of a pixel side by side.
//
// Per pixel, LDPixelSample (lowdiscrepancy.cpp:69-82, montecarlo.cpp:200-250) draws in this
// order: image (2D, 1 per sample), lens (2D), time (1D), then every 1D array (per light: the light
// component, the BSDF component), the emission integrator's two 1D(1) arrays, every 2D array (per
// light: light position, BSDF direction); then Li draws 6 values for every sample whose camera ray
// hits the scene (integrator.cpp:177-185). An array of n values per sample is LDShuffleScrambled
// (montecarlo.h:314-333): its scrambles, the (0,2) values, n draws per sample for the shuffle of
// the sample's own n values, spp draws for the shuffle of the samples (Shuffle, montecarlo.h:183-189).
//
// A wave never moves values around: each shuffle is replayed on an index array (the samples'
// block shuffle, sequential over the spp swaps, on one lane; each sample's own shuffle on its
// lane), and every value is then computed at its final place from the index it ends up holding --
// the (0,2) point of that index. The arrays the kernels read (image, light position, BSDF
// component, BSDF direction) are written to the window table -- the light arrays only for samples
// whose camera ray hits, the only ones shaded -- and the others only advance the stream.
//
// Whether a camera ray hits decides how far its pixel's Li advances the stream, so each is tested
// here, against the pixel's candidate triangles (scene.h CameraBins: the triangles whose projection
// can contain a point of the pixel) rather than by a BVH walk: the walks of the rays that pass close
// by the head without hitting it made the tasks around its silhouette the launch's longest
// (profiles/r05l_bins_ab.txt: 13.5 -> 7.5 ms per C2 frame).
#include "../../include/mpss.h"
#include "bvh_trace.h"
#include "render.h"

#include <algorithm>

namespace mpss {

namespace {

// MPSS_REPLAY_TASKTIME (a diagnostic build only): each wave prints its task's wall time (the
// real-time counter), pixel and camera-hit counts at the end (tools/replay_tasktime.py): the spread
// of task times against the launch, which ends with its slowest task.

constexpr int kMaxWaves = 4;  // waves per workgroup (fewer when a wave's LDS needs more room)

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }
// orders one wave's LDS accesses (a wave's LDS operations complete in issue order)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t temper(uint32_t y) {  // RNG::RandomUInt's output transform
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

// One wave's MT19937 (core/rng.cpp): the state in LDS, i = the next word.
struct WaveMt {
    uint32_t *st;
    int i;

    __device__ void seed(uint32_t v) {  // RNG::Seed: a 624-step recurrence, on lane 0
        if (lane_id() == 0) {
            st[0] = v;
            for (int k = 1; k < 624; ++k) {
                v = 1812433253u * (v ^ (v >> 30)) + (uint32_t)k;
                st[k] = v;
            }
        }
        wave_sync();
        i = 624;
    }
    // the generator step over all 624 words, 64 at a time in word order: word k reads words k + 1
    // and k + 397 not yet rewritten (k < 227) or word k - 227 already rewritten, as the sequential
    // loop does; a block's reads precede its writes
    __device__ void twist() {
        const int lane = lane_id();
        for (int base = 0; base < 624; base += 64) {
            const int k = base + lane;
            uint32_t v = 0;
            if (k < 624) {
                const uint32_t y = (st[k] & 0x80000000u) | (st[k + 1 < 624 ? k + 1 : 0] & 0x7fffffffu);
                v = st[k + 397 < 624 ? k + 397 : k - 227] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
            }
            wave_sync();
            if (k < 624) st[k] = v;
            wave_sync();
        }
        i = 0;
    }
    // the next `count` draws into db[0, count), in stream order
    __device__ void fetch(uint32_t *db, int count) {
        const int lane = lane_id();
        int done = 0;
        while (done < count) {
            if (i >= 624) twist();
            const int take = min(count - done, 624 - i);
            for (int k = lane; k < take; k += 64) db[done + k] = temper(st[i + k]);
            i += take;
            done += take;
        }
        wave_sync();
    }
    __device__ void skip(int64_t count) {  // draws whose values are not needed
        while (count > 0) {
            if (i >= 624) twist();
            const int take = (int)min<int64_t>(count, 624 - i);
            i += take;
            count -= take;
        }
    }
    __device__ uint2 two() {  // two draws, wave-uniform
        uint32_t *db = st + 624;  // (the draw buffer follows the state)
        fetch(db, 2);
        return make_uint2(db[0], db[1]);
    }
    __device__ uint32_t one() {
        uint32_t *db = st + 624;
        fetch(db, 1);
        return db[0];
    }
};

// Whether a camera ray through pixel (x, y) of the sample extent hits the scene (SamplerRenderer::Li's
// scene->Intersect, samplerrenderer.cpp:97-112: a hit is what makes Li draw its 6 values): the light
// spheres, then the pixel's candidate triangles (scene.h CameraBins: every triangle a ray through the
// pixel can meet in front of the camera) and the triangles every pixel tests. The answer is the BVH
// walk's: a ray hits iff it meets some triangle, whichever the walk would have found first. The
// candidates are wave-uniform (one pixel per wave), so each is one scalar load and one test per lane;
// the wave stops once every lane has hit.
__device__ bool cam_hit(const RenderScene &sc, const ReplayWindow &g, int x, int y, V3 o, V3 d, bool active) {
    bool hit = false;
    if (active)
        for (int l = 0; l < sc.nlights; ++l) {
            float t;
            if (!sc.lights[l].kind && sphere_hit_ool(sc.lights[l].s, o, d, 0.f, INFINITY, t, nullptr)) {
                hit = true;
                break;
            }
        }
    const cptr<TriRec> tris = as_const(sc.tris);
    auto test = [&](int t) {
        const TriRec tr = tris[t];
        float th, b1, b2;
        if (active && !hit &&
            tri_intersect(o, d, 0.f, INFINITY, V3{tr.p1[0], tr.p1[1], tr.p1[2]}, V3{tr.e1[0], tr.e1[1], tr.e1[2]},
                          V3{tr.e2[0], tr.e2[1], tr.e2[2]}, th, b1, b2))
            hit = true;
    };
    const cptr<int32_t> all = as_const(g.bin_all), cand = as_const(g.bin_tri);
    for (int k = 0; k < g.bin_nall; ++k) {
        if (__builtin_amdgcn_ballot_w64(active && !hit) == 0) return hit;
        test(all[k]);
    }
    const int p = __builtin_amdgcn_readfirstlane(y * g.bin_w + x);
    const cptr<uint32_t> off = as_const(g.bin_off);
    const uint32_t lo = off[p], hi = off[p + 1];
    for (uint32_t k = lo; k < hi; ++k) {
        if (__builtin_amdgcn_ballot_w64(active && !hit) == 0) break;
        test(cand[k]);
    }
    return hit;
}

// Shuffle(samples, count, dims) of whole samples replayed on idx (idx[i] = the original sample at
// position i afterwards), from its count draws already in d: first each draw becomes its swap
// partner i + d[i] % (count - i) (all lanes), then the swaps run in order on lane `who`
__device__ void shuffle_partners(uint32_t *d, uint32_t *idx, int count) {
    for (int i = lane_id(); i < count; i += 64) {
        idx[i] = (uint32_t)i;
        d[i] = (uint32_t)i + d[i] % (uint32_t)(count - i);
    }
}
// The swaps are a chain through idx (one LDS round trip each); the partners are not, so they are read
// eight at a time ahead of their swaps.
__device__ void shuffle_swaps(const uint32_t *o, uint32_t *idx, int count) {
    int i = 0;
    for (; i + 8 <= count; i += 8) {
        uint32_t p[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) p[k] = o[i + k];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t t = idx[i + k];
            idx[i + k] = idx[p[k]];
            idx[p[k]] = t;
        }
    }
    for (; i < count; ++i) {
        const uint32_t p = o[i];
        const uint32_t t = idx[i];
        idx[i] = idx[p];
        idx[p] = t;
    }
}

// A sample's own shuffle of 4 values (Shuffle(samp, 4, 1), the usual light-sample count): the four
// swaps on 2-bit places of one register, the partners j + dd[j] % (4 - j) with constant divisors,
// the result stored as one 4-byte word (sg is 4-byte aligned: the arrays' sig rows are n bytes).
__device__ __forceinline__ void own_shuffle4(const uint32_t *dd, uint8_t *sg) {
    const uint32_t r0 = dd[0], r1 = dd[1], r2 = dd[2];  // (dd[3] % 1 = 0: the last swap is with itself)
    const uint32_t o[3] = {r0 & 3u, 1u + r1 % 3u, 2u + (r2 & 1u)};
    uint32_t perm = 0xe4u;  // places 0..3 hold 0, 1, 2, 3
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const uint32_t t = ((perm >> (2 * j)) ^ (perm >> (2 * o[j]))) & 3u;
        perm ^= (t << (2 * j)) | (t << (2 * o[j]));
    }
    *(uint32_t *)sg = (perm & 3u) | ((perm & 0xcu) << 6) | ((perm & 0x30u) << 12) | ((perm & 0xc0u) << 18);
}

// One of a pixel's light-sample arrays (LDShuffleScrambled1D/2D(n, spp)): its draws in stream order
// at d -- hdr scrambles, spp x n own-shuffle draws, spp block-shuffle draws.
struct ReplayArray {
    uint32_t *d;
    uint32_t *idx;  // [spp]
    uint8_t *sig;   // [spp][n]
    int n, hdr, col;  // col: the first window-table column (-1: not read, only drawn)
};

// The arrays of a pixel after its image array that the kernels read, in LDPixelSample's order:
// per light the BSDF component (1D, column 2), then per light the light position (2D, columns 0-1)
// and the BSDF direction (2D, columns 3-4). (The light components and the emission integrator's
// two 1D(1) arrays are drawn between them and not read.) Array a of 3 x nlights, its draws at
// adraw + the draws of the arrays before it.
__device__ ReplayArray replay_array(const RenderScene &sc, int spp, int nmax, uint32_t *adraw, uint32_t *aidx,
                                    uint8_t *asig, int a) {
    const int nl = sc.nlights;
    auto shape = [&](int b, int &n, int &hdr, int &col) {
        const int l = b < nl ? b : (b - nl) >> 1;
        n = sc.lights[l].nsamples_round;
        hdr = b < nl ? 1 : 2;
        col = sc.lights[l].replay_off + (b < nl ? 2 : (((b - nl) & 1) ? 3 : 0));
    };
    int off = 0, n, hdr, col;
    for (int b = 0; b < a; ++b) {
        shape(b, n, hdr, col);
        off += hdr + spp * n + spp;
    }
    shape(a, n, hdr, col);
    return ReplayArray{adraw + off, aidx + (size_t)a * spp, asig + (size_t)a * spp * nmax, n, hdr, col};
}

// skip: 0, except in a diagnostic build (-DMPSS_DIAGNOSTICS: MPSS_REPLAY_SKIP, launch_replay_window; the
// values are then wrong): bit 0
// the per-sample own shuffles and the block shuffles' partners, 1 the block swaps, 2 the camera rays'
// hit tests, 3 the light arrays' values, 4 the draws' copies (the stream still advances) -- the cost of each
// section of the pixel loop, measured by leaving it out.
__global__ __launch_bounds__(64 * kMaxWaves) void replay_window_kernel(RenderScene sc, ReplayWindow g, int words,
                                                                       int skip) {
    extern __shared__ uint32_t smem[];
    const int wv = (int)(threadIdx.x >> 6), lane = lane_id();
    const int nwv = (int)(blockDim.x >> 6);
    const int wid = (int)blockIdx.x * nwv + wv;
    if (wid >= g.nxr * g.nyr) return;  // (wave-uniform; no workgroup barrier below)
    const int task = (g.yo0 + wid / g.nxr) * g.nx + g.xo0 + wid % g.nxr;
    int x0, x1, y0, y1;
    replay_sub_window(task, g.ntasks, 0, sc.xres + 1, 0, sc.yres + 1, x0, x1, y0, y1);
    const int ix0 = max(x0, g.x0), ix1 = min(x1, g.x0 + g.w), iy0 = max(y0, g.y0), iy1 = min(y1, g.y0 + g.h);
    if (ix0 >= ix1 || iy0 >= iy1) return;
    const int tw = x1 - x0, spp = g.spp;
    const int first = (iy0 - y0) * tw + (ix0 - x0), last = (iy1 - 1 - y0) * tw + (ix1 - 1 - x0);
    // this wave's LDS (replay_lds_words): state [624], image draws [max(spp, 2)], image idx [spp], the
    // arrays' draws, idx [arrays][spp], sig [arrays][spp][nmax] bytes
    uint32_t *base = smem + (size_t)wv * words;
    WaveMt mt{base, 624};
    uint32_t *dimg = base + 624;
    uint32_t *idx0 = dimg + max(spp, 2);
    uint32_t *adraw = idx0 + spp;
    uint32_t *aidx = adraw + g.arr_draws;
    const int na = 3 * sc.nlights;
    uint8_t *asig = (uint8_t *)(aidx + (size_t)na * spp);
    auto array = [&](int a) { return replay_array(sc, spp, g.nmax, adraw, aidx, asig, a); };

    uint32_t *gst = g.cur.mt + (size_t)task * 624;
    int ord = g.cur.cur_pix[task];
    if (ord < 0 || ord > first) {  // not seeded, or the window lies behind the cursor: RNG(task)
        mt.seed((uint32_t)task);
        ord = 0;
    } else {
        for (int k = lane; k < 624; k += 64) mt.st[k] = gst[k];
        wave_sync();
        mt.i = g.cur.cur_mti[task];
    }
    const V3 cam_o = xform_point(sc.camera_to_world, V3{0.f, 0.f, 0.f});
    const int64_t npix = (int64_t)g.w * g.h;
#ifdef MPSS_REPLAY_TASKTIME
    const uint64_t tt0 = __builtin_amdgcn_s_memrealtime();
    int tt_hits = 0, tt_pix = 0;
#endif
    for (; ord <= last; ++ord) {
        const int x = x0 + ord % tw, y = y0 + ord / tw;
        const bool keep = x >= g.x0 && x < g.x0 + g.w && y >= g.y0 && y < g.y0 + g.h;
        // value k of sample i of this pixel: out[k * npix * spp + i]
        float *out = keep ? g.out + ((int64_t)(y - g.y0) * g.w + (x - g.x0)) * spp : nullptr;
        auto put = [&](int k, int i, float v) { out[(int64_t)k * npix * spp + i] = v; };
        // every draw of the pixel's arrays first, in stream order: image (LDShuffleScrambled2D(1,
        // spp): its own-value shuffles, 1 draw each, keep the order), lens and time (only advance the
        // stream), then per light the light component (advances) and the BSDF component, the emission
        // integrator's two 1D(1) arrays (advance), per light the light position and BSDF direction
        const uint2 si = mt.two();
        mt.skip(spp);
        if (skip & 16) mt.skip(spp); else mt.fetch(dimg, spp);
        mt.skip(2 + 2 * (int64_t)spp);  // lens: LDShuffleScrambled2D(1, spp)
        mt.skip(1 + 2 * (int64_t)spp);  // time: LDShuffleScrambled1D(1, spp)
        for (int l = 0; l < sc.nlights; ++l) {
            mt.skip(1 + (int64_t)spp * sc.lights[l].nsamples_round + spp);
            const ReplayArray A = array(l);
            if (skip & 16) mt.skip(A.hdr + spp * A.n + spp); else mt.fetch(A.d, A.hdr + spp * A.n + spp);
        }
        mt.skip(2 * (1 + 2 * (int64_t)spp));
        for (int a = sc.nlights; a < na; ++a) {
            const ReplayArray A = array(a);
            if (skip & 16) mt.skip(A.hdr + spp * A.n + spp); else mt.fetch(A.d, A.hdr + spp * A.n + spp);
        }
        // each sample's own shuffle (lane per sample) and every block shuffle's partners
        if (!(skip & 1)) {
        shuffle_partners(dimg, idx0, spp);
        for (int a = 0; a < na; ++a) {
            const ReplayArray A = array(a);
            for (int i = lane; i < spp; i += 64) {
                uint8_t *sg = A.sig + (size_t)i * A.n;
                const uint32_t *dd = A.d + A.hdr + i * A.n;
                if (A.n == 4) {
                    own_shuffle4(dd, sg);
                    continue;
                }
                for (int j = 0; j < A.n; ++j) sg[j] = (uint8_t)j;
                for (int j = 0; j < A.n; ++j) {
                    const int o = j + (int)(dd[j] % (uint32_t)(A.n - j));
                    const uint8_t t = sg[j];
                    sg[j] = sg[o];
                    sg[o] = t;
                }
            }
            shuffle_partners(A.d + A.hdr + spp * A.n, A.idx, spp);
        }
        }
        wave_sync();
        // the block shuffles side by side, one per lane in one pass: unit 0 the image's, unit 1 + a array
        // a's, lane l taking units l, l + 64, ... (any light count)
        if (!(skip & 2))
            for (int u = lane; u <= na; u += 64) {
                const uint32_t *o = dimg;
                uint32_t *ix = idx0;
                if (u > 0) {
                    const ReplayArray A = array(u - 1);
                    o = A.d + A.hdr + spp * A.n;
                    ix = A.idx;
                }
                shuffle_swaps(o, ix, spp);
            }
        wave_sync();
        // the image samples and the camera rays (samplerrenderer.cpp:97-103): only whether they hit
        int hits = 0;
        // which of this lane's samples (lane + 64 m: bit m) hit: only those are shaded, so only their
        // light-sample values are read (render.hip); the others' are not written unless g.all_values
        uint64_t hm = 0;
        const bool traced = g.li_draws > 0 && !(skip & 4);
        for (int c = 0; c < spp; c += 64) {
            const int i = c + lane;
            const uint32_t b = idx0[i < spp ? i : 0];
            const float u = van_der_corput(b, si.x), v = sobol2(b, si.y);
            if (keep && i < spp) {
                put(0, i, u);
                put(1, i, v);
            }
            if (traced) {
                const float X = (float)x + u, Y = (float)y + v;
                const V3 pcam = xform_point(sc.raster_to_camera, V3{X, Y, 0.f});
                const V3 d = xform_vector(sc.camera_to_world, normalize(pcam));
                const bool hit = cam_hit(sc, g, x, y, cam_o, d, i < spp);
                hits += __popcll(__ballot(hit && i < spp));
                if (hit) hm |= 1ull << (c >> 6);
            }
        }
        if (keep && !(skip & 8))
            for (int a = 0; a < na; ++a) {
                const ReplayArray A = array(a);
                const uint32_t s0 = A.d[0], s1 = A.d[A.hdr - 1];
                for (int i = lane, m = 0; i < spp; i += 64, ++m) {
                    if (traced && !g.all_values && !((hm >> m) & 1)) continue;
                    const uint32_t b = A.idx[i];
                    const uint8_t *sg = A.sig + (size_t)b * A.n;
                    for (int j = 0; j < A.n; ++j) {
                        const uint32_t k = b * A.n + sg[j];
                        put(A.col + j * kReplayPerLightSample, i, van_der_corput(k, s0));
                        if (A.hdr == 2) put(A.col + j * kReplayPerLightSample + 1, i, sobol2(k, s1));
                    }
                }
            }
        wave_sync();
        mt.skip((int64_t)g.li_draws * hits);  // Li, per camera ray that hits
#ifdef MPSS_REPLAY_TASKTIME
        tt_hits += hits;
        ++tt_pix;
#endif
    }
#ifdef MPSS_REPLAY_TASKTIME
    if (lane == 0)
        printf("tasktime %d %d %d %d %d %llu\n", task, x0, y0, tt_pix, tt_hits,
               (unsigned long long)(__builtin_amdgcn_s_memrealtime() - tt0));
#endif
    for (int k = lane; k < 624; k += 64) gst[k] = mt.st[k];
    if (lane == 0) {
        g.cur.cur_pix[task] = last + 1;
        g.cur.cur_mti[task] = mt.i;
    }
}

}  // namespace

void replay_window_tasks(int xres, int yres, int ntasks, int x0, int x1, int y0, int y1, ReplayWindow &w) {
    const int ew = xres + 1, eh = yres + 1;
    int nx = ntasks, ny = 1;  // ComputeSubWindow's split (replay_sub_window)
    while ((nx & 0x1) == 0 && 2 * ew * ny < eh * nx) {
        nx >>= 1;
        ny <<= 1;
    }
    w.ntasks = ntasks;
    w.nx = nx;
    int lo = -1, hi = -1;
    for (int xo = 0; xo < nx; ++xo) {
        int a0, a1, b0, b1;
        replay_sub_window(xo, ntasks, 0, ew, 0, eh, a0, a1, b0, b1);
        if (a0 < x1 && a1 > x0) {
            if (lo < 0) lo = xo;
            hi = xo;
        }
    }
    w.xo0 = lo < 0 ? 0 : lo;
    w.nxr = lo < 0 ? 0 : hi - lo + 1;
    lo = hi = -1;
    for (int yo = 0; yo < ny; ++yo) {
        int a0, a1, b0, b1;
        replay_sub_window(yo * nx, ntasks, 0, ew, 0, eh, a0, a1, b0, b1);
        if (b0 < y1 && b1 > y0) {
            if (lo < 0) lo = yo;
            hi = yo;
        }
    }
    w.yo0 = lo < 0 ? 0 : lo;
    w.nyr = lo < 0 ? 0 : hi - lo + 1;
    w.x0 = x0;
    w.y0 = y0;
    w.w = x1 - x0;
    w.h = y1 - y0;
}

// One generator wave's LDS words (replay_window_kernel): MT state, image draws and idx, the arrays'
// draws, idx and sig.
static size_t replay_wave_words(int spp, int nlights, int nmax, int arr_draws) {
    const size_t na = 3 * (size_t)nlights;
    return 624 + (size_t)std::max(spp, 2) + spp + arr_draws + na * spp + (na * spp * nmax + 3) / 4;
}

void replay_check_lds(int spp, const int *light_samples, int nlights, const char *who) {
    int nmax = 1, arr_draws = 0;
    for (int l = 0; l < nlights; ++l) {
        const int n = replay_round_up_pow2(light_samples[l]);
        if (n < 1 || n > 256) throw Error(MPSS_ERR_INVALID, std::string(who) + ": the reference sampler takes light "
                                                           "sample counts (rounded up to a power of 2) in [1, 256]");
        nmax = std::max(nmax, n);
        arr_draws += 3 * (spp * n + spp) + 5;
    }
    const size_t bytes = sizeof(uint32_t) * replay_wave_words(spp, nlights, nmax, arr_draws);
    if (bytes > kReplayMaxLds)
        throw Error(MPSS_ERR_INVALID,
                    std::string(who) + ": the reference sampler replays a pbrt task's stream in one wave whose LDS holds "
                    "a pixel's draws, index arrays and shuffles: " + std::to_string(spp) + " spp with these lights' sample "
                    "counts needs " + std::to_string(bytes / 1024) + " KB, more than the 160 KB of LDS (fewer pixel "
                    "samples or light samples fit)");
}

void launch_replay_window(const RenderScene &sc, const ReplayWindow &w, hipStream_t stream) {
    const int nw = w.nxr * w.nyr;
    if (nw <= 0) return;
    if (w.nmax < 1 || w.nmax > 256) throw Error(MPSS_ERR_INVALID, "replay: light sample counts must be in [1, 256]");
    if (w.spp < 1 || w.spp > kReplayMaxSpp) throw Error(MPSS_ERR_INVALID, "replay: spp out of range");
    const int words = (int)replay_wave_words(w.spp, w.nlights, w.nmax, w.arr_draws);
    auto lds_of = [&](int nwv) { return sizeof(uint32_t) * (size_t)nwv * words; };
    int nwv = kMaxWaves;
    while (nwv > 1 && lds_of(nwv) > 64 * 1024) --nwv;  // two workgroups per CU where it fits
    const size_t lds = lds_of(nwv);
    if (lds > kReplayMaxLds)
        throw Error(MPSS_ERR_INVALID, "replay: spp x light samples too large for the replay generator's LDS");
    if (lds > 64 * 1024)
        MPSS_HIP(hipFuncSetAttribute((const void *)replay_window_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds));
#ifdef MPSS_DIAGNOSTICS  // (a diagnostic build only: a release library always generates every value)
    static const int skip = getenv("MPSS_REPLAY_SKIP") ? atoi(getenv("MPSS_REPLAY_SKIP")) : 0;
#else
    constexpr int skip = 0;
#endif
    hipLaunchKernelGGL(replay_window_kernel, dim3((unsigned)((nw + nwv - 1) / nwv)), dim3(64 * nwv), lds, stream, sc,
                       w, words, skip);
    MPSS_HIP(hipGetLastError());
}

}  // namespace mpss
