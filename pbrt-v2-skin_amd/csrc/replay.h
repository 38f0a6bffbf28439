// replay.h -- the reference sampler, replayed (mpss_config.sampler = MPSS_SAMPLER_REFERENCE).
//
// pbrt-v2 draws every sample value of a render from per-task MT19937 streams, so an image is a
// function of the task decomposition, which is a function of the reference run's core count:
//
//   SamplerRenderer::Render (renderers/samplerrenderer.cpp:191-225)
//       nTasks = RoundUpPow2(max(32 * NumSystemCores(), xres * yres / 256)); task n renders the
//       sub-window ComputeSubWindow(n, nTasks) (core/sampler.cpp:55-78) of the film's sample
//       extent [0, xres + 1) x [0, yres + 1) (ImageFilm::GetSampleExtent, film/image.cpp:150-166
//       with the 0.5-wide box filter) pixel by pixel in row order with RNG(n) (:60-74);
//   LDSampler::GetMoreSamples -> LDPixelSample (samplers/lowdiscrepancy.cpp:69-82,
//       core/montecarlo.cpp:200-250): per pixel, scrambled (0,2) sequences for the image, lens,
//       time and each 1D / 2D array the integrators requested, shuffled with the same RNG
//       (LDShuffleScrambled1D/2D, montecarlo.h:314-333; Shuffle, :183-189);
//   then, for every sample of the pixel whose camera ray hits the scene, Li draws 6 more values
//       (SpecularReflect + SpecularTransmit each build a BSDFSample(rng), integrator.cpp:177-185,
//       reflection.h:137-141) when ray.depth < maxdepth and irradiance points are not shown.
//
// The arrays, in request order (Sample::Sample, core/sampler.cpp:79-84): per light i (in scene
// order) LightSampleOffsets(n_i) = 1D comp + 2D pos (core/light.cpp:64-68), BSDFSampleOffsets(n_i)
// = 1D comp + 2D dir (core/reflection.cpp:655-659) with n_i = RoundUpPow2(nSamples); then the
// default "emission" volume integrator's two 1D(1) arrays (integrators/emission.cpp:39-43).
// LDPixelSample fills all 1D arrays, then all 2D arrays.
//
// IrradianceTask (integrators/multipolesubsurface.cpp:72-152, 186-210): RoundUpPow2(max(32 *
// NumSystemCores(), N / 4096)) tasks over point slices [k N / T, (k + 1) N / T), RNG(47 k), three
// draws per (point, light): the Sample02 scrambles and the component scramble.
//
// The product replays these streams on the GPU (replay_gen.hip: one wave per render task, per
// render batch into a table of the batch's window; render.hip replay_irradiance_kernel: one lane
// per irradiance task); oracle/render.c restates the same loop on the CPU.
#pragma once
#include "pbrt_math.h"

namespace mpss {

// Floats per camera sample in the replay table: image (u, v), then per light and light sample j:
// light position (2), BSDF component (1), BSDF direction (2). Lens, time, light components and
// the volume integrator's arrays are drawn (the stream must advance) but not consumed here.
constexpr int kReplayImage = 2, kReplayPerLightSample = 5;
constexpr int kReplayLiDraws = 6;
// the largest (power-of-two) spp the replay generator takes: one pixel's index arrays live in LDS,
// so the binding limit is kReplayMaxLds per generator wave (replay_check_lds: 1,024 spp fit with one
// light of 4 samples -- 94 KB -- and 2,048 do not; more or larger light-sample arrays fit fewer)
constexpr int kReplayMaxSpp = 4096;
constexpr size_t kReplayMaxLds = 160 * 1024;
// the largest window table of one render batch (floats: 8 GiB of the 288 GB); render_tiles closes a
// batch before it. (Larger windows replay more tasks at once: one wave per task is the unit.)
constexpr int64_t kReplayWindowFloats = (int64_t)1 << 31;

MPSS_HD int replay_round_up_pow2(int v) {
    int r = 1;
    while (r < v) r <<= 1;
    return r;
}

// RoundUpPow2(max(32 * cores, nPixels / 256)) (samplerrenderer.cpp:207-208)
MPSS_HD int replay_render_tasks(int xres, int yres, int cores) {
    const int a = 32 * cores, b = (int)(((int64_t)xres * yres) / (16 * 16));
    return replay_round_up_pow2(a > b ? a : b);
}

// RoundUpPow2(max(32 * cores, nPoints / 4096)) (multipolesubsurface.cpp:197-199)
MPSS_HD int replay_irradiance_tasks(int npoints, int cores) {
    const int a = 32 * cores, b = npoints / 4096;
    return replay_round_up_pow2(a > b ? a : b);
}

// Sampler::ComputeSubWindow (core/sampler.cpp:55-78) over [xs, xe) x [ys, ye)
MPSS_HD void replay_sub_window(int num, int count, int xs, int xe, int ys, int ye, int &x0, int &x1, int &y0,
                               int &y1) {
    const int dx = xe - xs, dy = ye - ys;
    int nx = count, ny = 1;
    while ((nx & 0x1) == 0 && 2 * dx * ny < dy * nx) {
        nx >>= 1;
        ny <<= 1;
    }
    const int xo = num % nx, yo = num / nx;
    const float tx0 = (float)xo / (float)nx, tx1 = (float)(xo + 1) / (float)nx;
    const float ty0 = (float)yo / (float)ny, ty1 = (float)(yo + 1) / (float)ny;
    // Floor2Int(Lerp(t, a, b)), Lerp = (1 - t) * a + t * b (pbrt.h)
    x0 = (int)floorf((1.f - tx0) * (float)xs + tx0 * (float)xe);
    x1 = (int)floorf((1.f - tx1) * (float)xs + tx1 * (float)xe);
    y0 = (int)floorf((1.f - ty0) * (float)ys + ty0 * (float)ye);
    y1 = (int)floorf((1.f - ty1) * (float)ys + ty1 * (float)ye);
}

// MT19937 (core/rng.cpp) with its 624-word state in memory at stride `st` (the device keeps
// the states of all tasks interleaved, word k of task t at k * ntasks + t, so a wave's lanes
// touch consecutive words).
struct Mt19937 {
    uint32_t *s;
    int st, i;
    MPSS_HD void seed(uint32_t v) {
        s[0] = v;
        for (int k = 1; k < 624; ++k) {
            v = 1812433253u * (v ^ (v >> 30)) + (uint32_t)k;
            s[(size_t)k * st] = v;
        }
        i = 624;
    }
    MPSS_HD uint32_t w(int k) const { return s[(size_t)k * st]; }
    MPSS_HD void twist() {
        for (int k = 0; k < 624; ++k) {
            const uint32_t y = (w(k) & 0x80000000u) | (w(k + 1 < 624 ? k + 1 : 0) & 0x7fffffffu);
            const int m = k + 397 < 624 ? k + 397 : k + 397 - 624;
            s[(size_t)k * st] = w(m) ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        i = 0;
    }
    MPSS_HD uint32_t next() {  // RNG::RandomUInt
        if (i >= 624) twist();
        uint32_t y = w(i++);
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= y >> 18;
        return y;
    }
    MPSS_HD void skip(int64_t n) {  // n draws whose values are not needed (no tempering)
        while (n > 0) {
            if (i >= 624) twist();
            const int64_t take = n < 624 - i ? n : 624 - i;
            i += (int)take;
            n -= take;
        }
    }
};

}  // namespace mpss
