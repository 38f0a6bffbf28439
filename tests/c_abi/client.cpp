// client.cpp -- a compiled C++ client of include/mpss.h, driven the way pbrt-v2-skin would drive the
// drop-in: plain C entry points, its own HIP streams, no Python, no torch.
//
//   client SCENE_DIR OUT_DIR X0 X1 Y0 Y1 SPP SEED NQ
//
// SCENE_DIR holds skin.pbrt as the scene loader parsed it (tests/test_c_abi_client_gpu.py writes it):
// the mpss_config and mpss_layeredskin structs as raw bytes (the ABI's own layout), the triangle mesh
// (world-space P, object-space N / S, uv, indices, ObjectToWorld / WorldToObject), the area light and
// the camera. The client
//   1. builds the scene through the C entry points (mpss_create, mpss_add_layeredskin, mpss_add_mesh,
//      mpss_add_sphere_light, mpss_set_camera) and runs mpss_preprocess -- MultipoleSubsurface-
//      Integrator::Preprocess (multipolesubsurface.cpp:170-238);
//   2. takes NQ surface points as shading points and evaluates Mo() (SubsurfaceOctreeNode::Mo,
//      diffusionutil.h:175-210) with mpss_mo_batch: once on one thread, then from 8 pthreads at once,
//      each on its own hipStream_t with its own slice -- Li is const and runs concurrently on pbrt's
//      worker threads (integrator.h:51-72, parallel.cpp:800-878) -- in the default sharded gather and
//      in the reference-order gather (exact_mo = 1, a second context); threaded == serial bit for bit;
//   3. renders the window [X0, X1) x [Y0, Y1) with mpss_render_tile (SamplerRendererTask::Run,
//      samplerrenderer.cpp:60-167) into OUT_DIR/tile.f32 (float4 XYZW per pixel);
//   4. checks the error convention: an unknown material id returns MPSS_ERR_INVALID with a message
//      (the adaptor turns it into pbrt's Severe()).
// Exit status 0 only if every check passed. Writes OUT_DIR/mo_exact.f32 (the reference-order Mo of
// the NQ points) and OUT_DIR/points.f32 (their positions) for the test to hold against the oracle.
#include <hip/hip_runtime_api.h>
#include <pthread.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mpss.h"

namespace {

[[noreturn]] void die(const char *what) {
    fprintf(stderr, "client: %s\n", what);
    exit(1);
}

void check(int rc, const char *what) {
    if (rc != MPSS_OK) {
        fprintf(stderr, "client: %s failed (%d): %s\n", what, rc, mpss_last_error());
        exit(1);
    }
}

void hip(hipError_t e, const char *what) {
    if (e != hipSuccess) {
        fprintf(stderr, "client: %s: %s\n", what, hipGetErrorString(e));
        exit(1);
    }
}

template <class T>
std::vector<T> read_file(const std::string &path, size_t want = 0) {
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) die(("cannot open " + path).c_str());
    fseek(f, 0, SEEK_END);
    const long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    if (n < 0 || n % (long)sizeof(T)) die(("bad size: " + path).c_str());
    std::vector<T> v((size_t)n / sizeof(T));
    if (!v.empty() && fread(v.data(), sizeof(T), v.size(), f) != v.size()) die(("short read: " + path).c_str());
    fclose(f);
    if (want && v.size() != want) die(("unexpected length: " + path).c_str());
    return v;
}

template <class T>
void write_file(const std::string &path, const T *data, size_t n) {
    FILE *f = fopen(path.c_str(), "wb");
    if (!f || fwrite(data, sizeof(T), n, f) != n) die(("cannot write " + path).c_str());
    fclose(f);
}

struct Scene {
    mpss_config cfg;
    mpss_layeredskin skin;
    std::vector<float> P, N, S, uv, o2w, w2o, r2c, c2w, light;
    std::vector<int32_t> idx, res;
};

Scene load(const std::string &dir) {
    Scene s;
    const auto cfg = read_file<uint8_t>(dir + "/config.bin", sizeof(mpss_config));
    memcpy(&s.cfg, cfg.data(), sizeof(mpss_config));
    const auto skin = read_file<uint8_t>(dir + "/skin.bin", sizeof(mpss_layeredskin));
    memcpy(&s.skin, skin.data(), sizeof(mpss_layeredskin));
    s.P = read_file<float>(dir + "/P.f32");
    s.N = read_file<float>(dir + "/N.f32");
    s.S = read_file<float>(dir + "/S.f32");
    s.uv = read_file<float>(dir + "/uv.f32");
    s.idx = read_file<int32_t>(dir + "/indices.i32");
    s.o2w = read_file<float>(dir + "/o2w.f32", 16);
    s.w2o = read_file<float>(dir + "/w2o.f32", 16);
    s.r2c = read_file<float>(dir + "/raster_to_camera.f32", 16);
    s.c2w = read_file<float>(dir + "/camera_to_world.f32", 16);
    s.res = read_file<int32_t>(dir + "/res.i32", 2);
    s.light = read_file<float>(dir + "/light.f32", 3 + 1 + MPSS_NBANDS + 1);  // center, radius, L[30], nsamples
    return s;
}

// One MultipoleSubsurfaceIntegrator: the scene through the C entry points, then Preprocess.
mpss_ctx *build(const Scene &s, int exact_mo, uint32_t *mid) {
    mpss_config cfg = s.cfg;
    cfg.exact_mo = exact_mo;
    mpss_ctx *ctx = nullptr;
    check(mpss_create(&cfg, &ctx), "mpss_create");
    check(mpss_add_layeredskin(ctx, &s.skin, mid), "mpss_add_layeredskin");
    const uint32_t nv = (uint32_t)(s.P.size() / 3), nt = (uint32_t)(s.idx.size() / 3);
    check(mpss_add_mesh(ctx, nv, s.P.data(), s.N.empty() ? nullptr : s.N.data(), s.S.empty() ? nullptr : s.S.data(),
                        s.uv.empty() ? nullptr : s.uv.data(), nt, s.idx.data(), s.o2w.data(), s.w2o.data(), 0, *mid),
          "mpss_add_mesh");
    check(mpss_add_sphere_light(ctx, s.light.data(), s.light[3], s.light.data() + 4, (int)s.light[4 + MPSS_NBANDS]),
          "mpss_add_sphere_light");
    check(mpss_set_camera(ctx, s.r2c.data(), s.c2w.data(), s.res[0], s.res[1]), "mpss_set_camera");
    check(mpss_preprocess(ctx, 1), "mpss_preprocess");
    return ctx;
}

// Mo of points [lo, hi) on the caller's own stream (one pbrt worker's batch of shading points).
struct Job {
    mpss_ctx *ctx;
    uint32_t mid;
    const float *pts;  // host, 3 per point
    float *mo;         // host, 30 per point
    uint32_t lo, hi;
    int rc;
    char err[256];
};

void *run_job(void *arg) {
    Job &j = *static_cast<Job *>(arg);
    const uint32_t q = j.hi - j.lo;
    hipStream_t st = nullptr;
    float *p_dev = nullptr, *mo_dev = nullptr;
    j.rc = -100;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return nullptr;
    if (hipMalloc((void **)&p_dev, sizeof(float) * 3 * (q ? q : 1)) != hipSuccess ||
        hipMalloc((void **)&mo_dev, sizeof(float) * MPSS_NBANDS * (q ? q : 1)) != hipSuccess)
        return nullptr;
    if (hipMemcpyAsync(p_dev, j.pts + 3 * (size_t)j.lo, sizeof(float) * 3 * q, hipMemcpyHostToDevice, st) !=
        hipSuccess)
        return nullptr;
    j.rc = mpss_mo_batch(j.ctx, j.mid, q, p_dev, mo_dev, nullptr, st);
    if (j.rc != MPSS_OK) snprintf(j.err, sizeof(j.err), "%s", mpss_last_error());  // thread-local message
    if (hipMemcpyAsync(j.mo + (size_t)MPSS_NBANDS * j.lo, mo_dev, sizeof(float) * MPSS_NBANDS * q,
                       hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        j.rc = -101;
    (void)hipFree(p_dev);
    (void)hipFree(mo_dev);
    (void)hipStreamDestroy(st);
    return nullptr;
}

std::vector<float> mo_threads(mpss_ctx *ctx, uint32_t mid, const std::vector<float> &pts, int nthreads) {
    const uint32_t n = (uint32_t)(pts.size() / 3);
    std::vector<float> mo((size_t)n * MPSS_NBANDS, -1.f);
    std::vector<Job> jobs((size_t)nthreads);
    std::vector<pthread_t> th((size_t)nthreads);
    for (int t = 0; t < nthreads; ++t) {
        // ragged slices, as pbrt's tasks are
        const uint32_t lo = (uint32_t)((uint64_t)n * t / nthreads), hi = (uint32_t)((uint64_t)n * (t + 1) / nthreads);
        jobs[t] = Job{ctx, mid, pts.data(), mo.data(), lo, hi, 0, {0}};
        if (pthread_create(&th[t], nullptr, run_job, &jobs[t])) die("pthread_create");
    }
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], nullptr);
    for (int t = 0; t < nthreads; ++t)
        if (jobs[t].rc != MPSS_OK) {
            fprintf(stderr, "client: thread %d: mpss_mo_batch rc %d: %s\n", t, jobs[t].rc, jobs[t].err);
            exit(1);
        }
    return mo;
}

bool same_bits(const std::vector<float> &a, const std::vector<float> &b) {
    return a.size() == b.size() && memcmp(a.data(), b.data(), sizeof(float) * a.size()) == 0;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc != 10) die("usage: client SCENE_DIR OUT_DIR X0 X1 Y0 Y1 SPP SEED NQ");
    const std::string in = argv[1], out = argv[2];
    const int x0 = atoi(argv[3]), x1 = atoi(argv[4]), y0 = atoi(argv[5]), y1 = atoi(argv[6]);
    const int spp = atoi(argv[7]);
    const uint32_t seed = (uint32_t)strtoul(argv[8], nullptr, 10), nq_want = (uint32_t)strtoul(argv[9], nullptr, 10);
    if (mpss_abi_version() < 10) die("libmpss ABI older than this client");
    const Scene s = load(in);

    uint32_t mid = 0, mid_exact = 0;
    mpss_ctx *ctx = build(s, 0, &mid);
    mpss_ctx *ctx_exact = build(s, 1, &mid_exact);

    // shading points: the first NQ surface points (SurfacePoint records, p at byte 0)
    uint32_t npts = 0;
    check(mpss_get_surface_points(ctx, nullptr, &npts), "mpss_get_surface_points (count)");
    std::vector<uint8_t> recs((size_t)npts * 44);
    check(mpss_get_surface_points(ctx, recs.data(), &npts), "mpss_get_surface_points");
    const uint32_t nq = nq_want < npts ? nq_want : npts;
    std::vector<float> pts((size_t)3 * nq);
    for (uint32_t i = 0; i < nq; ++i) memcpy(&pts[3 * (size_t)i], &recs[44 * (size_t)i], 12);

    int fails = 0;
    for (int pass = 0; pass < 2; ++pass) {
        mpss_ctx *c = pass ? ctx_exact : ctx;
        const uint32_t m = pass ? mid_exact : mid;
        const std::vector<float> serial = mo_threads(c, m, pts, 1);
        const std::vector<float> threaded = mo_threads(c, m, pts, 8);
        const bool ok = same_bits(serial, threaded);
        bool nonzero = false;
        for (float v : serial) nonzero = nonzero || v > 0.f;
        printf("mo_batch %s: %u points, 8 threads on 8 streams %s the serial call%s\n",
               pass ? "exact_mo=1" : "sharded", nq, ok ? "==" : "!=", nonzero ? "" : " (ALL ZERO)");
        if (!ok || !nonzero) ++fails;
        if (pass) write_file(out + "/mo_exact.f32", serial.data(), serial.size());
    }
    write_file(out + "/points.f32", pts.data(), pts.size());

    // one window of the frame
    const size_t npx = (size_t)(x1 - x0) * (size_t)(y1 - y0);
    float *tile_dev = nullptr;
    hipStream_t st = nullptr;
    hip(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
    hip(hipMalloc((void **)&tile_dev, sizeof(float) * 4 * npx), "hipMalloc");
    check(mpss_render_tile(ctx, spp, seed, x0, x1, y0, y1, tile_dev, st), "mpss_render_tile");
    std::vector<float> tile(4 * npx);
    hip(hipMemcpyAsync(tile.data(), tile_dev, sizeof(float) * tile.size(), hipMemcpyDeviceToHost, st), "copy tile");
    hip(hipStreamSynchronize(st), "sync");
    write_file(out + "/tile.f32", tile.data(), tile.size());
    (void)hipFree(tile_dev);
    (void)hipStreamDestroy(st);

    // the error convention: no exception, a code and a message
    float dummy[MPSS_NBANDS * 4] = {0.f};
    const int rc = mpss_mo_batch(ctx, 999, 1, dummy, dummy, nullptr, nullptr);
    const bool err_ok = rc == MPSS_ERR_INVALID && strstr(mpss_last_error(), "material") != nullptr;
    printf("unknown material: rc %d, \"%s\" %s\n", rc, mpss_last_error(), err_ok ? "ok" : "UNEXPECTED");
    if (!err_ok) ++fails;

    mpss_destroy(ctx_exact);
    mpss_destroy(ctx);
    printf(fails ? "client: %d check(s) FAILED\n" : "client: all checks passed\n", fails);
    return fails ? 1 : 0;
}
