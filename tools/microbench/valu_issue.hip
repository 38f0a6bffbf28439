// valu_issue.hip -- how many wave64 vector instructions per second one MI355X (gfx950) SIMD issues,
// by instruction and by waves per SIMD: the ceiling the Mo() gather's VALU count is priced against
// (MI355X_MICROARCH.md gives 2 cycles per v_fma_f32 on a SIMD-32 with several
// waves and 4 for one wave alone, but nothing for the packed f32 and conversion instructions the
// gather's record loop is made of).
//
// Each variant is one instruction repeated over 8 independent register chains (so no dependency
// wait), 32 per loop step, in inline asm (the compiler neither folds nor reorders it); "gather mix"
// is the instruction mix of one common-grid point record of mo_band_wave_kernel<false,5088,true>
// (counted from its ISA: hipcc -S of mo_wave_cg.hip) with its SALU beside it. Every wave stamps
// s_memtime at its start and end, so cycles are the shader clock's, not an assumed 2.4 GHz.
//
// Launch: W waves per SIMD as the gather runs them -- one workgroup of 64 x 4 x W threads per CU for
// W = 1, 2, 4, and two 1024-thread workgroups per CU for W = 8 (mo_band_wave_kernel's shape); each
// workgroup holds enough dynamic LDS that no third fits, so every wave of a CU is resident at once.
//
// Printed per (variant, W): wave64 instructions per second over the chip; the shader clock the waves
// ran at (s_memtime ticks over s_memrealtime's 100 MHz); and SIMD cycles per wave instruction = the
// launch time at that clock / (W x instructions per wave). (A SIMD issues its waves oldest first:
// with W > 1 a wave's own span is shorter than the launch -- span_over_launch -- so it is not the
// SIMD's busy time.)
//
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/valu_issue.hip -o tools/microbench/valu_issue
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

enum {
    V_FMA = 0,  // v_fma_f32
    V_ADD,      // v_add_f32
    V_PKMUL,    // v_pk_mul_f32
    V_PKADD,    // v_pk_add_f32
    V_PKFMA,    // v_pk_fma_f32
    V_CVT,      // v_cvt_u32_f32
    V_FRACT,    // v_fract_f32
    V_CND,      // v_cndmask_b32 (e64, SGPR-pair mask)
    V_LSHLADD,  // v_lshl_add_u32
    V_MIX,      // the gather's point-record mix (VALU only)
    V_MIXS,     // the same plus its SALU
    V_ADDU,     // v_add_u32
    V_MINU,     // v_min_u32
    V_MINF,     // v_min_f32
    V_MOV,      // v_mov_b32
    V_CMP,      // v_cmp_gt_f32 (e64, to an SGPR pair)
    V_MUL,      // v_mul_f32
    V_MAX3,     // v_max3_f32
    V_RCP,      // v_rcp_f32
    V_MIX5,     // the round-5 fused record (one group-row lookup + one LDS lookup), VALU + SALU
    V_MIX6,     // the round-6 record (one group-row lookup + one LDS lookup), VALU + SALU
    V_COUNT
};
static const char *kNames[V_COUNT] = {"v_fma_f32",      "v_add_f32",    "v_pk_mul_f32",   "v_pk_add_f32",
                                      "v_pk_fma_f32",   "v_cvt_u32_f32", "v_fract_f32",   "v_cndmask_b32",
                                      "v_lshl_add_u32", "gather mix (VALU)", "gather mix (VALU + SALU)",
                                      "v_add_u32",      "v_min_u32",    "v_min_f32",      "v_mov_b32",
                                      "v_cmp_gt_f32 (e64)", "v_mul_f32", "v_max3_f32",   "v_rcp_f32",
                                      "gather mix r05 (fused: row + LDS record, VALU + SALU)",
                                      "gather mix r06 (row + LDS record, VALU + SALU)"};
// wave64 VALU instructions per loop step, and SALU
static const int kValu[V_COUNT] = {32, 32, 32, 32, 32, 32, 32, 32, 32, 94, 94,  // mix: 2 records x 47
                                   32, 32, 32, 32, 32, 32, 32, 32, 64, 68};
static const int kSalu[V_COUNT] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 48, 0, 0, 0, 0, 0, 0, 0, 0, 24, 24};

#define R8(X) X X X X X X X X
#define R4(X) X X X X

// 8 chains a0..a7 (f32 or packed pairs p0..p7), operands x (VGPR), s (SGPR pair)
template <int V>
__device__ __forceinline__ void step(float (&a)[8], float x, float y) {
    if (V == V_FMA) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int k = 0; k < 8; ++k) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(x), "v"(y));
    } else if (V == V_ADD) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int k = 0; k < 8; ++k) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[k]) : "v"(x));
    } else if (V == V_CVT) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int k = 0; k < 8; ++k) asm volatile("v_cvt_u32_f32 %0, %0" : "+v"(a[k]));
    } else if (V == V_FRACT) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int k = 0; k < 8; ++k) asm volatile("v_fract_f32 %0, %0" : "+v"(a[k]));
    } else if (V == V_LSHLADD) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int k = 0; k < 8; ++k) asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(a[k]) : "v"(x));
    } else if (V == V_ADDU || V == V_MINU || V == V_MINF || V == V_MOV || V == V_MUL || V == V_MAX3 || V == V_RCP) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (V == V_ADDU) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[k]) : "v"(x));
                if (V == V_MINU) asm volatile("v_min_u32 %0, %0, %1" : "+v"(a[k]) : "v"(x));
                if (V == V_MINF) asm volatile("v_min_f32 %0, %0, %1" : "+v"(a[k]) : "v"(x));
                if (V == V_MOV) asm volatile("v_mov_b32 %0, %1" : "=v"(a[k]) : "v"(a[(k + 1) & 7]));
                if (V == V_MUL) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[k]) : "v"(x));
                if (V == V_MAX3) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(x), "v"(y));
                if (V == V_RCP) asm volatile("v_rcp_f32 %0, %0" : "+v"(a[k]));
            }
    } else if (V == V_CMP) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                uint64_t m;
                asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(m) : "v"(a[k]), "v"(x));
                asm volatile("" ::"s"(m));
            }
    } else if (V == V_CND) {
        uint64_t m;
        asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(m) : "v"(x), "v"(y));
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int k = 0; k < 8; ++k) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[k]) : "v"(x), "s"(m));
    }
}

typedef float f2v __attribute__((ext_vector_type(2)));

template <int V>
__device__ __forceinline__ void step_pk(f2v (&p)[8], f2v x) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (V == V_PKMUL) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p[k]) : "v"(x));
            if (V == V_PKADD) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p[k]) : "v"(x));
            if (V == V_PKFMA) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p[k]) : "v"(x));
        }
}

// One point record of the common-grid gather (mo_band_wave_kernel<false,5088,true>, point-pair loop
// per point): d2 (3 sub, 3 mul, 2 add as v_subrev/v_pk_add + v_mul/v_pk_mul + v_add), u and f (1 mul, 2
// pk_mul), 5 cvt, 1 cmp + 1 lshl-add (row offset), 4 lshl-add (LDS addresses), 2 cmp + 2 cndmask + 1 cmp
// (path), the lerp (4 fract, 4 sub, 4 pk_mul, 4 add), the tau test (1 cmp), products (4 pk_mul, 1
// pk_add) -- 47 VALU with 24 SALU (exec-mask saves/restores, branches' scalar compares, the pair's
// address increments). Two records interleaved (independent registers), as the pair loop runs them.
template <bool SALU>
__device__ __forceinline__ void step_mix(float (&a)[8], f2v (&p)[8], float x, f2v xv, uint32_t &s0, uint32_t &s1) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        float &d = a[4 * h], &u = a[4 * h + 1], &t = a[4 * h + 2], &w = a[4 * h + 3];
        f2v &pa = p[4 * h], &pb = p[4 * h + 1], &pc = p[4 * h + 2], &pd = p[4 * h + 3];
        uint64_t m;
        // d2
        asm volatile("v_subrev_f32 %0, %1, %0" : "+v"(d) : "v"(x));
        asm volatile("v_pk_add_f32 %0, %0, %1 neg_lo:[0,1] neg_hi:[0,1]" : "+v"(pa) : "v"(xv));
        asm volatile("v_mul_f32 %0, %0, %0" : "+v"(d));
        asm volatile("v_pk_mul_f32 %0, %0, %0" : "+v"(pa));
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(d) : "v"(x));
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(d) : "v"(x));
        // u, f
        asm volatile("v_mul_f32 %0, %1, %0" : "+v"(u) : "v"(x));
        asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(pb) : "v"(xv));
        asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(pc) : "v"(xv));
        R4(asm volatile("v_cvt_u32_f32 %0, %0" : "+v"(t));)
        asm volatile("v_cvt_u32_f32 %0, %0" : "+v"(w));
        asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(m) : "v"(x), "v"(u));
        asm volatile("v_lshl_add_u32 %0, %0, 5, %1" : "+v"(w) : "v"(x));
        R4(asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(t) : "v"(x));)
        // path
        asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(m) : "v"(x), "v"(u));
        asm volatile("v_cmp_le_f32_e64 %0, %1, %2" : "=s"(m) : "v"(x), "v"(u));
        asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(w) : "v"(x), "s"(m));
        asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(w) : "v"(x), "s"(m));
        asm volatile("v_cmp_lt_i32_e64 %0, 1, %1" : "=s"(m) : "v"(w));
        // lerp
        R4(asm volatile("v_fract_f32 %0, %0" : "+v"(u));)
        R4(asm volatile("v_sub_f32 %0, 1.0, %0" : "+v"(u));)
        asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(pd) : "v"(xv));
        asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(pd) : "v"(xv));
        asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(pb) : "v"(xv));
        asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(pc) : "v"(xv));
        R4(asm volatile("v_add_f32 %0, %0, %1" : "+v"(d) : "v"(x));)
        asm volatile("v_cmp_ge_f32_e64 %0, %1, %2" : "=s"(m) : "v"(x), "v"(d));
        // products
        asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(pa) : "v"(xv));
        asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(pb) : "v"(xv));
        asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(pc) : "v"(xv));
        asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(pd) : "v"(xv));
        asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(pa) : "v"(pb));
        if (SALU) {
            R4(asm volatile("s_add_u32 %0, %0, 32\n s_addc_u32 %1, %1, 0" : "+s"(s0), "+s"(s1) ::"scc");)
            R4(asm volatile("s_cmp_ge_i32 %0, %1\n s_cselect_b32 %0, %0, %1" : "+s"(s0) : "s"(s1) : "scc");)
            R4(asm volatile("s_mov_b32 %0, %1\n s_or_b32 %1, %1, %0" : "+s"(s0), "+s"(s1) ::"scc");)
        }
    }
}

// The round-5 fused common-grid record (mo_band.h cg_fetch / cg_combine with MPSS_MO_FUSED, TPATH,
// LAZYF; counted from the hipcc -S of mo_wave_cg.hip): a group-row record -- d2 (4 plain + 2 packed),
// u, its cvt, the LDS-path compare, the row offset, the two path compares, fract(u) and three moves,
// the lerp (4 sub + 4 fma), the tau compare, two packed FMAs (27 VALU) -- and an LDS record -- the same
// head, then 2 packed muls, 4 cvt, 4 LDS addresses, 4 fract, the compares, lerp, tau, products (37
// VALU); with the exec-mask SALU of the three path steps (12 per record).
__device__ __forceinline__ void step_mix5(float (&a)[8], f2v (&p)[8], float x, f2v xv, uint32_t &s0, uint32_t &s1) {
    float &d = a[0], &u = a[1], &t = a[2], &w = a[3], &e = a[4], &g = a[5], &h = a[6], &k = a[7];
    f2v &pa = p[0], &pb = p[1], &pc = p[2], &pd = p[3];
    uint64_t m;
#pragma unroll
    for (int rec = 0; rec < 2; ++rec) {
        asm volatile("v_subrev_f32 %0, %1, %0" : "+v"(d) : "v"(x));
        asm volatile("v_pk_add_f32 %0, %0, %1 neg_lo:[0,1] neg_hi:[0,1]" : "+v"(pa) : "v"(xv));
        asm volatile("v_mul_f32 %0, %0, %0" : "+v"(d));
        asm volatile("v_pk_mul_f32 %0, %0, %0" : "+v"(pa));
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(d) : "v"(x));
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(d) : "v"(x));
        asm volatile("v_mul_f32 %0, %1, %0" : "+v"(u) : "v"(x));
        asm volatile("v_cvt_u32_f32 %0, %0" : "+v"(w));
        asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(m) : "v"(x), "v"(u));
        asm volatile("v_add_lshl_u32 %0, %0, %1, 5" : "+v"(w) : "v"(x));
        asm volatile("v_cmp_le_f32_e64 %0, %1, %2" : "=s"(m) : "v"(x), "v"(u));
        asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(m) : "v"(x), "v"(u));
        if (rec == 0) {  // group rows
            asm volatile("v_fract_f32 %0, %0" : "+v"(t));
            asm volatile("v_mov_b32 %0, %1" : "=v"(e) : "v"(t));
            asm volatile("v_mov_b32 %0, %1" : "=v"(g) : "v"(t));
            asm volatile("v_mov_b32 %0, %1" : "=v"(h) : "v"(t));
        } else {  // LDS
            asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(pb) : "v"(xv));
            asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(pc) : "v"(xv));
            R4(asm volatile("v_cvt_u32_f32 %0, %0" : "+v"(k));)
            R4(asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(k) : "v"(x));)
            R4(asm volatile("v_fract_f32 %0, %0" : "+v"(t));)
        }
        R4(asm volatile("v_sub_f32 %0, %0, %1" : "+v"(e) : "v"(x));)
        R4(asm volatile("v_fma_f32 %0, %1, %0, %2" : "+v"(g) : "v"(t), "v"(x));)
        asm volatile("v_cmp_ge_f32_e64 %0, %1, %2" : "=s"(m) : "v"(x), "v"(d));
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(pd) : "v"(pb), "v"(xv));
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(pa) : "v"(pc), "v"(xv));
        R4(asm volatile("s_add_u32 %0, %0, 32\n s_addc_u32 %1, %1, 0" : "+s"(s0), "+s"(s1) ::"scc");)
        R4(asm volatile("s_mov_b32 %0, %1\n s_or_b32 %1, %1, %0" : "+s"(s0), "+s"(s1) ::"scc");)
        R4(asm volatile("s_cmp_ge_i32 %0, %1\n s_cselect_b32 %0, %0, %1" : "+s"(s0) : "s"(s1) : "scc");)
    }
}

// The round-6 record (mo_band.h cg_fetch / cg_fix / cg_combine, counted from the hipcc -S of
// mo_wave_cg.hip): the common head -- d2 (4 plain + 2 packed), u, the row coordinate v (fma, min), its
// cvt and row offset, the three path compares (14 VALU) -- then a group-row record: fract(v) and three
// moves, the flagged-cell compare, the lerp (4 sub + 4 fma), two packed FMAs (29 VALU); and an LDS
// record: 2 packed muls, 4 cvt, 4 LDS addresses, 4 fract, the flagged-cell compare, lerp, products (39
// VALU); with the exec-mask SALU of the path steps (12 per record).
__device__ __forceinline__ void step_mix6(float (&a)[8], f2v (&p)[8], float x, f2v xv, uint32_t &s0, uint32_t &s1) {
    float &d = a[0], &u = a[1], &t = a[2], &w = a[3], &e = a[4], &g = a[5], &h = a[6], &k = a[7];
    f2v &pa = p[0], &pb = p[1], &pc = p[2], &pd = p[3];
    uint64_t m;
#pragma unroll
    for (int rec = 0; rec < 2; ++rec) {
        asm volatile("v_subrev_f32 %0, %1, %0" : "+v"(d) : "v"(x));
        asm volatile("v_pk_add_f32 %0, %0, %1 neg_lo:[0,1] neg_hi:[0,1]" : "+v"(pa) : "v"(xv));
        asm volatile("v_mul_f32 %0, %0, %0" : "+v"(d));
        asm volatile("v_pk_mul_f32 %0, %0, %0" : "+v"(pa));
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(d) : "v"(x));
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(d) : "v"(x));
        asm volatile("v_mul_f32 %0, %1, %0" : "+v"(u) : "v"(x));
        asm volatile("v_fma_f32 %0, %1, %0, %2" : "+v"(g) : "v"(u), "v"(x));
        asm volatile("v_min_f32 %0, %0, %1" : "+v"(g) : "v"(u));
        asm volatile("v_cvt_u32_f32 %0, %0" : "+v"(w));
        asm volatile("v_add_lshl_u32 %0, %0, %1, 5" : "+v"(w) : "v"(x));
        asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(m) : "v"(x), "v"(u));
        asm volatile("v_cmp_le_f32_e64 %0, %1, %2" : "=s"(m) : "v"(x), "v"(u));
        asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(m) : "v"(x), "v"(u));
        if (rec == 0) {  // group rows
            asm volatile("v_fract_f32 %0, %0" : "+v"(t));
            asm volatile("v_mov_b32 %0, %1" : "=v"(e) : "v"(t));
            asm volatile("v_mov_b32 %0, %1" : "=v"(g) : "v"(t));
            asm volatile("v_mov_b32 %0, %1" : "=v"(h) : "v"(t));
        } else {  // LDS
            asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(pb) : "v"(xv));
            asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(pc) : "v"(xv));
            R4(asm volatile("v_cvt_u32_f32 %0, %0" : "+v"(k));)
            R4(asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(k) : "v"(x));)
            R4(asm volatile("v_fract_f32 %0, %0" : "+v"(t));)
        }
        asm volatile("v_cmp_u_f32_e64 %0, %1, %2" : "=s"(m) : "v"(e), "v"(e));
        R4(asm volatile("v_sub_f32 %0, %0, %1" : "+v"(e) : "v"(x));)
        R4(asm volatile("v_fma_f32 %0, %1, %0, %2" : "+v"(g) : "v"(t), "v"(x));)
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(pd) : "v"(pb), "v"(xv));
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(pa) : "v"(pc), "v"(xv));
        R4(asm volatile("s_add_u32 %0, %0, 32\n s_addc_u32 %1, %1, 0" : "+s"(s0), "+s"(s1) ::"scc");)
        R4(asm volatile("s_mov_b32 %0, %1\n s_or_b32 %1, %1, %0" : "+s"(s0), "+s"(s1) ::"scc");)
        R4(asm volatile("s_cmp_ge_i32 %0, %1\n s_cselect_b32 %0, %0, %1" : "+s"(s0) : "s"(s1) : "scc");)
    }
}

template <int V>
__global__ __launch_bounds__(1024) void issue_kernel(int steps, float *out, unsigned long long *span) {
    const float x = 1.0f + threadIdx.x * 1e-7f, y = 1e-3f;
    float a[8];
    f2v p[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        a[k] = 0.5f + k * 0.01f;
        p[k] = f2v{a[k], a[k] + 1.f};
    }
    const f2v xv = f2v{x, y};
    uint32_t s0 = blockIdx.x, s1 = steps;
    unsigned long long t0, r0;
    asm volatile("s_memtime %0\n s_memrealtime %1\n s_waitcnt lgkmcnt(0)" : "=s"(t0), "=s"(r0));
    for (int i = 0; i < steps; ++i) {
        if (V == V_PKMUL || V == V_PKADD || V == V_PKFMA)
            step_pk<V>(p, xv);
        else if (V == V_MIX)
            step_mix<false>(a, p, x, xv, s0, s1);
        else if (V == V_MIXS)
            step_mix<true>(a, p, x, xv, s0, s1);
        else if (V == V_MIX5)
            step_mix5(a, p, x, xv, s0, s1);
        else if (V == V_MIX6)
            step_mix6(a, p, x, xv, s0, s1);
        else
            step<V>(a, x, y);
    }
    unsigned long long t1, r1;
    asm volatile("s_memtime %0\n s_memrealtime %1\n s_waitcnt lgkmcnt(0)" : "=s"(t1), "=s"(r1));
    float r = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) r += a[k] + p[k].x + p[k].y;
    if (r == 12345.f) out[0] = r + (float)(s0 + s1);  // keep the chains
    if ((threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        span[2 * w] = t1 - t0;
        span[2 * w + 1] = r1 - r0;
    }
}

template <int V>
void launch(int blocks, int threads, size_t lds, int steps, float *o, unsigned long long *sp) {
    static bool attr = false;
    if (!attr) {
        CHECK(hipFuncSetAttribute((const void *)issue_kernel<V>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr = true;
    }
    hipLaunchKernelGGL(issue_kernel<V>, dim3(blocks), dim3(threads), lds, 0, steps, o, sp);
}

int main(int argc, char **argv) {
    const int steps = argc > 1 ? atoi(argv[1]) : 4096;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const int wmax = 8;
    float *o;
    unsigned long long *sp;
    CHECK(hipMalloc(&o, sizeof(float)));
    CHECK(hipMalloc(&sp, sizeof(unsigned long long) * 2 * 4 * cus * wmax));
    std::vector<unsigned long long> hs(2 * 4 * cus * wmax);  // (wave span, real-time span) per wave
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    void (*fn[V_COUNT])(int, int, size_t, int, float *, unsigned long long *) = {
        launch<0>,  launch<1>,  launch<2>,  launch<3>,  launch<4>,  launch<5>,  launch<6>,
        launch<7>,  launch<8>,  launch<9>,  launch<10>, launch<11>, launch<12>, launch<13>,
        launch<14>, launch<15>, launch<16>, launch<17>, launch<18>, launch<19>, launch<20>};
    const int ws[4] = {1, 2, 4, 8};
    printf("{\"cus\": %d, \"clock_khz\": %d, \"steps\": %d, \"results\": [\n", cus, prop.clockRate, steps);
    bool first = true;
    for (int v = 0; v < V_COUNT; ++v) {
        for (int wi = 0; wi < 4; ++wi) {
            const int W = ws[wi];
            // W <= 4: one workgroup of 4 W waves per CU; W = 8: two of 16 (the gather's shape). The LDS
            // keeps a further workgroup off the CU.
            const int threads = W <= 4 ? 256 * W : 1024, per_cu = W <= 4 ? 1 : 2, blocks = cus * per_cu;
            const size_t lds = per_cu == 1 ? 96 * 1024 : 64 * 1024;
            fn[v](blocks, threads, lds, 64, o, sp);  // warm-up (code, clocks)
            CHECK(hipEventRecord(a));
            fn[v](blocks, threads, lds, steps, o, sp);
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            CHECK(hipGetLastError());
            float ms = 0.f;
            CHECK(hipEventElapsedTime(&ms, a, b));
            const int waves_n = blocks * threads / 64;
            CHECK(hipMemcpy(hs.data(), sp, sizeof(unsigned long long) * 2 * waves_n, hipMemcpyDeviceToHost));
            // each wave's own span on the shader clock (s_memtime) and on the 100 MHz real-time clock;
            // every wave of a CU is resident from the start, so the mean span is the SIMDs' busy time
            double mean_span = 0.0, mean_real = 0.0;
            for (int w = 0; w < waves_n; ++w) {
                mean_span += (double)hs[2 * w];
                mean_real += (double)hs[2 * w + 1];
            }
            mean_span /= waves_n;
            mean_real /= waves_n;
            const double waves = waves_n;
            const double vinsts = waves * steps * kValu[v];
            // per SIMD: W waves, each issuing steps * kValu VALU, over the launch (the SIMD issues its
            // waves oldest first, so one wave's own span is shorter than the SIMD's busy time): the
            // launch time at the waves' clock
            const double clk = mean_span / (mean_real * 10.0);  // GHz
            const double cyc_per_inst = (ms * 1e-3) * clk * 1e9 / ((double)W * steps * kValu[v]);
            printf("%s{\"variant\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"valu_wave_insts_per_s\": %.4g, "
                   "\"salu_per_valu\": %.2f, \"simd_cycles_per_valu_inst\": %.3f, \"clock_ghz\": %.3f, "
                   "\"span_over_launch\": %.3f}",
                   first ? "" : ",\n", kNames[v], W, ms, vinsts / (ms * 1e-3), (double)kSalu[v] / kValu[v],
                   cyc_per_inst, clk, mean_real * 1e-8 / (ms * 1e-3));
            first = false;
        }
    }
    printf("\n]}\n");
    return 0;
}
