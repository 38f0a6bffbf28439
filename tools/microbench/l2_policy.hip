// l2_policy.hip -- what a per-lane 8-byte table gather costs on MI355X (gfx950), by load form and
// cache policy: the question is whether any form moves more lane lookups per second through the
// vector L1 / L2 request path than the plain global_load_dwordx2 the Mo() gather issues.
//
// Table: 8 band groups x 4 bands x 2^17 floats (2 MB per group, the skin profile's footprint),
// group = block % 8 (one XCD's L2 per group, as in the gather). Each step issues 4 independent
// loads (the 4 bands) and consumes them together. Offsets come from a per-lane LCG (a few VALU
// per load, so the floor is the memory path, not the address arithmetic). `spread` lanes share an
// offset (1 = every lane its own line).
//
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/l2_policy.hip -o tools/microbench/l2_policy
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
constexpr uint32_t kMask = (1u << kLog) - 2u;  // even offsets (8-byte aligned) for the even variants
constexpr int kLdsFloats = 8192;                // 32 KB LDS table for the LDS variants

typedef float f2 __attribute__((ext_vector_type(2)));
struct __attribute__((aligned(4))) Pair {
    float a, b;
};

enum {
    V_PLAIN = 0,     // compiler global_load_dwordx2 (4-byte aligned pair, as the gather)
    V_ASM,           // asm global_load_dwordx2
    V_NT,            // ... nt
    V_SC0,           // ... sc0
    V_SC1,           // ... sc1
    V_SC01,          // ... sc0 sc1
    V_SC01NT,        // ... sc0 sc1 nt
    V_DWORD,         // one global_load_dword (4 B)
    V_FLAT,          // flat_load_dwordx2, global address
    V_FLAT_LDS,      // flat_load_dwordx2, LDS address (every lane)
    V_DS,            // ds_read_b64
    V_BUFFER,        // buffer_load_dwordx2 offen
    V_ODD,           // plain pair at odd (4-byte, not 8-byte aligned) offsets
    V_HALF,          // plain pair, odd lanes exec-masked off (32 distinct lines per instruction)
    V_MIX,           // flat_load_dwordx2, even lanes' addresses in LDS, odd lanes' in the table
    V_COUNT
};
static const char *kNames[V_COUNT] = {"plain", "asm", "nt", "sc0", "sc1", "sc0sc1", "sc0sc1nt", "dword",
                                      "flat", "flat_lds", "ds_read_b64", "buffer", "odd", "half", "mix"};

__device__ __forceinline__ uint32_t lcg(uint32_t &s) {
    s = s * 1664525u + 1013904223u;
    return s;
}


template <int V>
__global__ __launch_bounds__(1024) void gather_kernel(const float *__restrict__ tables, int steps, int spread,
                                                      float *out) {
    extern __shared__ float lds[];
    const int grp = blockIdx.x & 7;
    const float *t = tables + ((size_t)grp * 4 << kLog);
    uint32_t s = ((blockIdx.x * 1024u + threadIdx.x) / (uint32_t)spread) * 2654435761u + 12345u;
    if (V == V_FLAT_LDS || V == V_DS || V == V_MIX) {
        for (int i = threadIdx.x; i < kLdsFloats; i += blockDim.x) lds[i] = (float)i * 1e-3f;
        __syncthreads();
    }
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)t, 0, 0x7fffffff, 0x00020000);
    f2 acc = {0.f, 0.f};
    for (int i = 0; i < steps; ++i) {
        f2 v[4];
        uint32_t o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t r = lcg(s) >> (32 - kLog);
            if (V == V_FLAT_LDS || V == V_DS || (V == V_MIX && !(threadIdx.x & 1)))
                o[j] = (r & (kLdsFloats - 2)) ;
            else if (V == V_ODD)
                o[j] = (uint32_t)j * (1u << kLog) + ((r & (kMask - 2u)) | 1u)  /* pair ends at 2^17 - 2 */;
            else
                o[j] = (uint32_t)j * (1u << kLog) + (r & kMask);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float *p = t + o[j];
            if (V == V_HALF) {
                if (threadIdx.x & 1) {
                    v[j] = f2{0.f, 0.f};
                } else {
                    const Pair q = *reinterpret_cast<const Pair *>(p);
                    v[j] = f2{q.a, q.b};
                }
            } else if (V == V_MIX) {
                const float *q = (threadIdx.x & 1) ? p : lds + o[j];
                asm volatile("flat_load_dwordx2 %0, %1" : "=v"(v[j]) : "v"(q));
            } else if (V == V_PLAIN || V == V_ODD) {
                const Pair q = *reinterpret_cast<const Pair *>(p);
                v[j] = f2{q.a, q.b};
            } else if (V == V_ASM) {
                asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v[j]) : "v"(p));
            } else if (V == V_NT) {
                asm volatile("global_load_dwordx2 %0, %1, off nt" : "=v"(v[j]) : "v"(p));
            } else if (V == V_SC0) {
                asm volatile("global_load_dwordx2 %0, %1, off sc0" : "=v"(v[j]) : "v"(p));
            } else if (V == V_SC1) {
                asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=v"(v[j]) : "v"(p));
            } else if (V == V_SC01) {
                asm volatile("global_load_dwordx2 %0, %1, off sc0 sc1" : "=v"(v[j]) : "v"(p));
            } else if (V == V_SC01NT) {
                asm volatile("global_load_dwordx2 %0, %1, off sc0 sc1 nt" : "=v"(v[j]) : "v"(p));
            } else if (V == V_DWORD) {
                float a;
                asm volatile("global_load_dword %0, %1, off" : "=v"(a) : "v"(p));
                v[j] = f2{a, a};
            } else if (V == V_FLAT) {
                asm volatile("flat_load_dwordx2 %0, %1" : "=v"(v[j]) : "v"(p));
            } else if (V == V_FLAT_LDS) {
                const float *q = lds + o[j];  // generic pointer into the LDS aperture
                asm volatile("flat_load_dwordx2 %0, %1" : "=v"(v[j]) : "v"(q));
            } else if (V == V_DS) {
                const uint32_t a = (uint32_t)(o[j] * 4u);
                asm volatile("ds_read_b64 %0, %1" : "=v"(v[j]) : "v"(a));
            } else if (V == V_BUFFER) {
                typedef unsigned u2 __attribute__((ext_vector_type(2)));
                const u2 r = __builtin_amdgcn_raw_buffer_load_b64(rsrc, o[j] * 4u, 0, 0);
                v[j] = f2{__uint_as_float(r.x), __uint_as_float(r.y)};
            }
        }
        if (V != V_PLAIN && V != V_ODD && V != V_HALF) {
            if (V == V_DS)
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
            else if (V == V_FLAT || V == V_FLAT_LDS || V == V_MIX)
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
            else
                asm volatile("s_waitcnt vmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) acc += v[j];
    }
    if (acc.x == 12345.f) out[0] = acc.y;  // keep the loads
}

typedef void (*kfn)(const float *, int, int, float *);
template <int V>
void launch(int blocks, const float *d, int steps, int sp, float *o) {
    const size_t sh = (V == V_FLAT_LDS || V == V_DS || V == V_MIX) ? kLdsFloats * sizeof(float) : 0;
    hipLaunchKernelGGL(gather_kernel<V>, dim3(blocks), dim3(1024), sh, 0, d, steps, sp, o);
}
template <int... Vs>
struct Table {
    static constexpr void (*fn[])(int, const float *, int, int, float *) = {launch<Vs>...};
};

int main(int argc, char **argv) {
    const int steps = argc > 1 ? atoi(argv[1]) : 256;
    std::vector<float> h((size_t)8 * 4 << kLog);
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
    using T = Table<0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14>;
    const int spreads[] = {1, 4};
    printf("{\"cus\": %d, \"blocks\": %d, \"steps\": %d, \"results\": [\n", prop.multiProcessorCount, blocks, steps);
    bool first = true;
    for (int v = 0; v < V_COUNT; ++v)
        for (int sp : spreads) {
            T::fn[v](blocks, d, 16, sp, o);  // warm L2
            CHECK(hipEventRecord(a));
            T::fn[v](blocks, d, steps, sp, o);
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            CHECK(hipGetLastError());
            float ms = 0.f;
            CHECK(hipEventElapsedTime(&ms, a, b));
            const double loads = (double)blocks * 1024 * steps * 4;
            const double insts = loads / 64;
            printf("%s{\"variant\": \"%s\", \"spread\": %d, \"ms\": %.3f, \"lane_loads_per_s\": %.4g, "
                   "\"cu_cycles_per_inst_at_2.4GHz\": %.1f}",
                   first ? "" : ",\n", kNames[v], sp, ms, loads / (ms * 1e-3),
                   (ms * 1e-3) * 2.4e9 * prop.multiProcessorCount / insts);
            first = false;
        }
    printf("]}\n");
    return 0;
}
