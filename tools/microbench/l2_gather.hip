// l2_gather.hip -- L2 request ceiling of the Mo() gather's access pattern on MI355X (gfx950).
//
// Each lane performs 8-byte loads (an Rd lerp pair) at per-lane random offsets into one of 8
// band-group tables of 4 x L floats (1.9 MB for L = 119,766: the skin profile), group = block %
// 8, i.e. one XCD's L2 holds one group's tables -- the mo_band_kernel mapping. Four independent
// loads (the 4 bands) are issued per step and consumed together, 1024-thread workgroups at 8
// waves per SIMD. `spread` lanes share one offset (1 = every lane its own line). Reports lane
// loads/s and, for spread 1, L2 requests/s (one request per lane load: the lines are distinct).
//
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/l2_gather.hip -o /tmp/l2_gather && /tmp/l2_gather
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

struct __attribute__((aligned(4))) Pair {
    float a, b;
};

__device__ __forceinline__ uint32_t mix(uint32_t h) {
    h ^= h >> 16;
    h *= 0x7feb352du;
    h ^= h >> 15;
    h *= 0x846ca68bu;
    h ^= h >> 16;
    return h;
}

__global__ __launch_bounds__(1024) void gather_kernel(const float *__restrict__ tables, int L, int steps, int spread,
                                                      float *out) {
    const int grp = blockIdx.x & 7;
    const float *t = tables + (size_t)grp * 4 * L;
    const uint32_t lane_key = (blockIdx.x * 1024u + threadIdx.x) / (uint32_t)spread;
    float acc = 0.f;
    for (int i = 0; i < steps; ++i) {
        Pair v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t s = mix(lane_key * 2654435761u + (uint32_t)(i * 4 + j)) % (uint32_t)(L - 1);
            v[j] = *reinterpret_cast<const Pair *>(t + (size_t)j * L + s);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) acc += v[j].a * 0.5f + v[j].b;
    }
    if (acc == 12345.f) out[0] = acc;  // keep the loads
}

int main(int argc, char **argv) {
    const int L = 119766, steps = argc > 1 ? atoi(argv[1]) : 256;
    std::vector<float> h((size_t)8 * 4 * L);
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
    printf("{\"cus\": %d, \"blocks\": %d, \"steps\": %d, \"results\": [", prop.multiProcessorCount, blocks, steps);
    const int spreads[] = {1, 2, 4, 8, 16, 64};
    for (int k = 0; k < 6; ++k) {
        const int sp = spreads[k];
        hipLaunchKernelGGL(gather_kernel, dim3(blocks), dim3(1024), 0, 0, d, L, 16, sp, o);  // warm L2
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL(gather_kernel, dim3(blocks), dim3(1024), 0, 0, d, L, steps, sp, o);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, a, b));
        const double loads = (double)blocks * 1024 * steps * 4;
        printf("%s{\"spread\": %d, \"ms\": %.3f, \"lane_loads_per_s\": %.4g}", k ? ", " : "", sp, ms,
               loads / (ms * 1e-3));
    }
    printf("]}\n");
    return 0;
}
