// l2_width.hip -- what one lane lookup costs on the gather's memory path by load width (MI355X,
// gfx950): the common-grid gather reads a group row pair as two 16-byte loads from one 32-byte
// sector per lane, the per-band path four 8-byte lerp pairs from four unrelated lines per lane.
//
// Table: 8 band groups x 2 MB (one XCD's L2 per group, block % 8 as in the gather), per-lane
// offsets from an LCG, 64 distinct lines per instruction. Each step issues the variant's loads and
// consumes them together. Printed: lane loads per second and the CU cycles one wave instruction
// occupies (2.4 GHz), the quantity the gather's TA busy counter tracks.
//
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/l2_width.hip -o tools/microbench/l2_width
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e = (x);                                                                   \
        if (e != hipSuccess) {                                                                \
            fprintf(stderr, "%s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);     \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

constexpr int kLog = 19;  // 2^19 floats = 2 MB per group
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

enum { W4 = 0, W8, W16, ROW32, PAIRS4, W16X4, ROW16X2, ROW64, ROW16X2_S, ROW16X2_H, ROW16X2_L, V_COUNT };
static const char *kNames[V_COUNT] = {"dword (4 B)", "dwordx2 (8 B)", "dwordx4 (16 B)",
                                      "2 x dwordx4, one 32-B sector (group row pair)",
                                      "4 x dwordx2, four lines (per-band pairs)", "4 x dwordx4, four lines",
                                      "2 x dwordx4, 32 contiguous bytes at 16-B alignment (16-B rows u, u + 1)",
                                      "4 x dwordx4, one 64-B segment (8-band row)",
                                      "2 x dwordx4 at 16 and 32 mod 64 (two sectors of one 64-B half)",
                                      "2 x dwordx4 at 48 and 64 mod 128 (the two 64-B halves of one line)",
                                      "2 x dwordx4 at 112 mod 128 and the next line"};
static const int kInsts[V_COUNT] = {1, 1, 1, 2, 4, 4, 2, 4, 2, 2, 2};

__device__ __forceinline__ uint32_t lcg(uint32_t &s) {
    s = s * 1664525u + 1013904223u;
    return s;
}

template <int V>
__global__ __launch_bounds__(1024) void width_kernel(const float *__restrict__ tables, int steps, float *out) {
    const int grp = blockIdx.x & 7;
    const float *t = tables + ((size_t)grp << kLog);
    uint32_t s = (blockIdx.x * 1024u + threadIdx.x) * 2654435761u + 12345u;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < steps; ++i) {
        if (V == W4) {
            const uint32_t o = lcg(s) >> (32 - kLog);
            acc.x += t[o];
        } else if (V == W8) {
            const uint32_t o = (lcg(s) >> (32 - kLog)) & ~1u;
            const f2 v = *(const f2 *)(t + o);
            acc.x += v.x + v.y;
        } else if (V == W16) {
            const uint32_t o = (lcg(s) >> (32 - kLog)) & ~3u;
            acc += *(const f4 *)(t + o);
        } else if (V == ROW32) {
            const uint32_t o = (lcg(s) >> (32 - kLog)) & ~7u;
            const f4 a = *(const f4 *)(t + o), b = *(const f4 *)(t + o + 4);
            acc += a + b;
        } else if (V == PAIRS4) {
            f2 v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = *(const f2 *)(t + ((lcg(s) >> (32 - kLog)) & ~1u));
            acc.x += v[0].x + v[1].x + v[2].x + v[3].x;
            acc.y += v[0].y + v[1].y + v[2].y + v[3].y;
        } else if (V == ROW16X2) {
            const uint32_t o = (lcg(s) >> (32 - kLog)) & ~3u;
            const uint32_t o2 = o + 4 < (1u << kLog) ? o + 4 : o;
            const f4 a = *(const f4 *)(t + o), b = *(const f4 *)(t + o2);
            acc += a + b;
        } else if (V == ROW16X2_S || V == ROW16X2_H || V == ROW16X2_L) {
            // the first load at a fixed offset in its 128-B line: 16 B (sectors 0, 1), 48 (halves), 112 (lines)
            const uint32_t in = V == ROW16X2_S ? 4u : (V == ROW16X2_H ? 12u : 28u);
            const uint32_t o = (((lcg(s) >> (32 - kLog)) & ~31u) + in) & ((1u << kLog) - 8u);
            const uint32_t o2 = o + 4;
            const f4 a = *(const f4 *)(t + o), b = *(const f4 *)(t + o2);
            acc += a + b;
        } else if (V == ROW64) {
            const uint32_t o = (lcg(s) >> (32 - kLog)) & ~15u;
            const f4 a = *(const f4 *)(t + o), b = *(const f4 *)(t + o + 4);
            const f4 c = *(const f4 *)(t + o + 8), d = *(const f4 *)(t + o + 12);
            acc += (a + b) + (c + d);
        } else {
            f4 v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = *(const f4 *)(t + ((lcg(s) >> (32 - kLog)) & ~3u));
            acc += v[0] + v[1] + v[2] + v[3];
        }
    }
    if (acc.x + acc.y + acc.z + acc.w == 12345.f) out[0] = acc.y;  // keep the loads
}

template <int V>
void launch(int blocks, const float *d, int steps, float *o) {
    hipLaunchKernelGGL(width_kernel<V>, dim3(blocks), dim3(1024), 0, 0, d, steps, o);
}

int main(int argc, char **argv) {
    const int steps = argc > 1 ? atoi(argv[1]) : 256;
    const int only = argc > 2 ? atoi(argv[2]) : -1;  // one variant (the PMC passes), or all
    std::vector<float> h((size_t)8 << kLog);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)(i % 1000) * 1e-3f;
    float *d, *o;
    CHECK(hipMalloc(&d, h.size() * sizeof(float)));
    CHECK(hipMalloc(&o, sizeof(float)));
    CHECK(hipMemcpy(d, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice));
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int blocks = prop.multiProcessorCount * 2;  // 2 x 16 waves per CU = 8 waves per SIMD
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    void (*fn[V_COUNT])(int, const float *, int, float *) = {launch<0>, launch<1>, launch<2>,
                                                                launch<3>, launch<4>, launch<5>, launch<6>, launch<7>,
                                                                launch<8>, launch<9>, launch<10>};
    printf("{\"cus\": %d, \"blocks\": %d, \"steps\": %d, \"results\": [\n", prop.multiProcessorCount, blocks, steps);
    for (int v = 0; v < V_COUNT; ++v) {
        if (only >= 0 && v != only) continue;
        fn[v](blocks, d, 16, o);  // warm L2
        CHECK(hipEventRecord(a));
        fn[v](blocks, d, steps, o);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        CHECK(hipGetLastError());
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, a, b));
        const double lane_steps = (double)blocks * 1024 * steps;
        const double insts = lane_steps * kInsts[v] / 64;
        printf("%s{\"variant\": \"%s\", \"ms\": %.3f, \"lane_lookups_per_s\": %.4g, "
               "\"cu_cycles_per_wave_inst\": %.1f, \"cu_cycles_per_lane_lookup_x64\": %.1f}",
               (only < 0 ? v : 0) ? ",\n" : "", kNames[v], ms, lane_steps / (ms * 1e-3),
               (ms * 1e-3) * 2.4e9 * prop.multiProcessorCount / insts,
               (ms * 1e-3) * 2.4e9 * prop.multiProcessorCount / (lane_steps / 64));
    }
    printf("]}\n");
    return 0;
}
