// l2_mlp.hip -- does the per-lane gather's cost per L2 line depend on how many loads each wave keeps in
// flight? Same table and access pattern as l2_policy.hip (8 groups x 4 bands x 2^17 floats, group =
// block % 8, 64 distinct lines per instruction), with NL independent 8-byte loads issued per step before
// any is consumed (the Mo() gather issues 8: two points x four bands), at 16 or 32 waves per CU.
//
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/l2_mlp.hip -o tools/microbench/l2_mlp
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

constexpr int kLog = 17;
constexpr uint32_t kMask = (1u << kLog) - 2u;
struct __attribute__((aligned(4))) Pair {
    float a, b;
};

template <int NL>
__global__ __launch_bounds__(1024) void mlp_kernel(const float *__restrict__ tables, int steps, float *out) {
    const int grp = blockIdx.x & 7;
    const float *t = tables + ((size_t)grp * 4 << kLog);
    uint32_t s = (blockIdx.x * 1024u + threadIdx.x) * 2654435761u + 12345u;
    float acc = 0.f;
    for (int i = 0; i < steps; ++i) {
        Pair v[NL];
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            s = s * 1664525u + 1013904223u;
            const uint32_t o = (uint32_t)(j & 3) * (1u << kLog) + ((s >> (32 - kLog)) & kMask);
            v[j] = *reinterpret_cast<const Pair *>(t + o);
        }
#pragma unroll
        for (int j = 0; j < NL; ++j) acc += v[j].a * 0.5f + v[j].b;
    }
    if (acc == 12345.f) out[0] = acc;
}

template <int NL>
void run(const float *d, float *o, int blocks, int steps, const char *tag, bool &first) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL(mlp_kernel<NL>, dim3(blocks), dim3(1024), 0, 0, d, 8, o);  // warm
    CHECK(hipEventRecord(a));
    hipLaunchKernelGGL(mlp_kernel<NL>, dim3(blocks), dim3(1024), 0, 0, d, steps, o);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    CHECK(hipGetLastError());
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double loads = (double)blocks * 1024 * steps * NL;
    printf("%s{\"loads_in_flight\": %d, \"waves_per_cu\": \"%s\", \"ms\": %.3f, \"lines_per_s\": %.4g}", first ? "" : ",\n",
           NL, tag, ms, loads / (ms * 1e-3));
    first = false;
}

int main(int argc, char **argv) {
    const int steps0 = argc > 1 ? atoi(argv[1]) : 256;
    std::vector<float> h((size_t)8 * 4 << kLog);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)(i % 1000) * 1e-3f;
    float *d, *o;
    CHECK(hipMalloc(&d, h.size() * sizeof(float)));
    CHECK(hipMalloc(&o, sizeof(float)));
    CHECK(hipMemcpy(d, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice));
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    printf("{\"cus\": %d, \"results\": [\n", prop.multiProcessorCount);
    bool first = true;
    for (int wpc : {1, 2}) {  // 1024-thread blocks per CU: 16 or 32 waves per CU
        const int blocks = prop.multiProcessorCount * wpc;
        const char *tag = wpc == 1 ? "16" : "32";
        run<4>(d, o, blocks, steps0, tag, first);
        run<8>(d, o, blocks, steps0 / 2, tag, first);
        run<16>(d, o, blocks, steps0 / 4, tag, first);
        run<32>(d, o, blocks, steps0 / 8, tag, first);
    }
    printf("]}\n");
    return 0;
}
