// render.h -- device-side scene, sample records and the kernels of the per-pixel path
// (render.hip), plus the host driver that uploads a SceneData and runs Preprocess / tiles.
#pragma once
#include <vector>

#include "common.h"
#include "geom.h"
#include "mo_kernel.h"
#include "mo_band.h"
#include "replay.h"
#include "scene.h"
#include "texture.h"

namespace mpss {

struct RenderMesh {
    MeshView view;  // device pointers
    uint32_t material;
};

struct RenderLight {
    SphereView s;
    float Lemit[NB];
    int nsamples_pow2;   // RoundUpPow2(nSamples): IrradianceTask (file line 196)
    int nsamples_round;  // LDSampler::RoundSize(nSamples): RequestSamples (file line 248)
    // kind 1 (LightSource "infinite"): LightToWorld / WorldToLight, level 0 of the radiance
    // MIPMap (tw x th RGB texels) and the Distribution2D over the image (nu x nv): conditional
    // func / cdf rows, their funcInts (= the marginal's func), the marginal cdf and funcInt
    // (envmap.h). A light without "mapname" is the 1x1 map L.ToRGBSpectrum().
    int kind;
    int tw, th, nu, nv;
    const float *tex, *func, *cdf, *rint, *mcdf;
    float mint;
    float l2w[9], w2l[9];
    int replay_off;      // first float of this light's samples in a replay-table row (replay.h)
};

struct RenderMaterial {
    float R[NB];          // Kr (Microfacet reflectance), layeredskin.cpp:154-158
    float T[NB];          // Kt (MicrofacetTransmission), layeredskin.cpp:159-161
    float alb_mix[NB];    // Pow(albedo, mix)      (IrradianceTask, file line 224)
    float alb_1mmix[NB];  // Pow(albedo, 1 - mix)  (Li, file line 371)
    Microfacet mf;
    const float *rho;     // device rho_hd table
    int n_rho, has_bssrdf, has_refl, has_trans, is_mc;
    // ImageTexture "albedo" (replaces alb_mix / alb_1mmix: Pow(FromRGB(lookup), mix) per point)
    // and "bumpmap" (Material::Bump of the shading geometry), textures/imagemap.cpp
    int has_alb_tex, has_bump;
    float mix;
    TexView alb_tex, bump_tex;
    int band_pos[NB];     // band c's float offset in a hit's Mo() row (this profile's BandGroups::pos)
    // R's range for direct_combine's per-term quotient guard: every R[c] >= 0 (r_nonneg), the least
    // nonzero R[c] and the largest (0, 0 when R is black)
    float r_lo, r_hi;
    int r_nonneg;
};

struct RenderScene {
    const BvhNode *bvh;
    // the same nodes threaded for stackless any-hit walks: an interior node's offset is the end of
    // its pre-order subtree (render_host.hip upload_scene); nbvh nodes
    const BvhNode *bvh_thread;
    int nbvh;
    const TriRec *tris;
    const int32_t *tri_mesh, *tri_local;
    const RenderMesh *meshes;
    const RenderLight *lights;
    const RenderMaterial *materials;
    int nlights, nmaterials, xres, yres;
    int have_octree;  // Preprocess built an octree: BSSRDF hits evaluate Mo()
    int n_infinite;   // lights of kind 1: camera rays that miss everything see their Le
    int any_tex;      // some material has an albedo texture or a bump map: shade_tex_kernel runs
    float raster_to_camera[16], camera_to_world[16];
    float dx_camera[3], dy_camera[3];  // PerspectiveCamera dxCamera / dyCamera (perspective.cpp:47-48)
    // reference-sampler replay (replay.h); null: the counter-hash sampler. The sample values of one
    // render batch's window [replay_x0, replay_x0 + replay_w) x [replay_y0, ...) (replay_gen.hip),
    // column-major: value k of camera sample s of window pixel p at [(k * replay_npix + p) *
    // replay_spp + s] (a wave's lanes, consecutive samples of one pixel, read consecutive floats)
    const float *replay;
    int replay_k, replay_spp, replay_x0, replay_y0, replay_w;
    int64_t replay_npix;
    const uint32_t *irr_scr;  // [point][light][2] IrradianceTask Sample02 scrambles
};

// The GPU replay of the reference's render-task streams for one window of the sample extent
// (replay_gen.hip): one wave per SamplerRendererTask whose sub-window meets the window, resuming
// the task's MT19937 stream from its cursor (the next pixel of its sub-window, in row order) or
// from RNG(task) when the window lies behind it. The cursors persist between windows, so a frame
// rendered in row order replays every stream once. mt: [ntasks][624] states; cur_pix: the next
// pixel ordinal per task (-1: not seeded); cur_mti: the state's word index.
struct ReplayCursors {
    uint32_t *mt;
    int *cur_pix, *cur_mti;
};
struct ReplayWindow {
    int ntasks, nx;            // the task grid (ComputeSubWindow: nx x (ntasks / nx))
    int xo0, nxr, yo0, nyr;    // the tasks meeting the window: columns xo0.., rows yo0..
    int x0, y0, w, h;          // the window (pixels of the sample extent)
    int spp, K, li_draws, nmax;  // nmax: the largest light-sample count (array length)
    int nlights, arr_draws;      // arr_draws: the draws of a pixel's read light arrays, sum over
                                 // lights of 3 (spp n + spp) + 5
    ReplayCursors cur;
    float *out;                // the window table (RenderScene::replay layout)
    // the camera rays' candidate triangles per pixel of the sample extent (scene.h CameraBins)
    const uint32_t *bin_off;   // [bin_w * (yres + 1) + 1]
    const int32_t *bin_tri, *bin_all;
    int bin_w, bin_nall;
    // 1: every sample's light-sample values (replay_samples: the whole table); 0: only those of
    // samples whose camera ray hits (a render: the others are never shaded)
    int all_values;
};
// Launches the generation on `stream` (the host picks the task ranges: replay_window_tasks).
void launch_replay_window(const RenderScene &sc, const ReplayWindow &w, hipStream_t stream);
// Throws (naming `who` and the LDS a generator wave would need) when spp pixel samples with lights of
// these sample counts do not fit the generator's LDS (kReplayMaxLds).
void replay_check_lds(int spp, const int *light_samples, int nlights, const char *who);
// The task grid and the task columns / rows meeting [x0, x1) x [y0, y1) of the (xres + 1) x
// (yres + 1) sample extent.
void replay_window_tasks(int xres, int yres, int ntasks, int x0, int x1, int y0, int y1, ReplayWindow &w);
// IrradianceTask streams: scr[(i * nlights + l) * 2 + {0, 1}] for points i < n
__global__ void replay_irradiance_kernel(int n, int nlights, int ntasks, uint32_t *mt, uint32_t *scr);

// A tile [x0,x1) x [y0,y1) extended by one pixel on every side that exists (origin ex0, ey0;
// ew x eh pixels): a sample whose float image coordinate rounds onto a pixel edge also lands
// in the neighbouring pixel (film_kernel).
struct TileBatch {
    int x0, x1, y0, y1, ex0, ey0, ew, eh, spp;
    uint32_t seed;
    int64_t nsamples;  // ew * eh * spp
};

// Up to kMaxPieces tile pieces of one batch in ONE launch of primary_kernel / film_kernel (a
// launch per piece left most of the chip idle: a 128 x 128 tile's film pass is 64 workgroups).
// Piece k owns blocks [block0[k], block0[k + 1]); its camera samples start at record off[k] of
// the batch; out[k] / out_stride[k]: its film rectangle (film_kernel).
constexpr int kMaxPieces = 16;
struct PieceList {
    int n;
    int block0[kMaxPieces + 1];
    int out_stride[kMaxPieces];
    int64_t off[kMaxPieces];
    float *out[kMaxPieces];
    TileBatch tb[kMaxPieces];
};

// The piece of this block (wave-uniform: kernel-argument reads, <= kMaxPieces steps).
__device__ __forceinline__ int piece_of(const PieceList &pl, int block) {
    int k = 0;
    while (k + 1 < pl.n && block >= pl.block0[k + 1]) ++k;
    return k;
}

enum : uint32_t {
    REC_LIVE = 1u,
    REC_SURF = 2u,  // hit a mesh: Ld valid
    REC_SSS = 4u,   // material has a MultipoleBSSRDF: pq valid
    REC_LE = 8u,    // hit an area light's front face, or (light field 0xff) missed with infinite lights
    // the sample's float image position rounds onto a pixel edge, so the box filter also
    // carries it into the neighbour: left (x-1), right (x+1), up (y-1), down (y+1)
    REC_XLO = 16u, REC_XHI = 32u, REC_YLO = 64u, REC_YHI = 128u,
    REC_LIGHT_SHIFT = 8,
    REC_MAT_SHIFT = 16,
    REC_LSURF = 1u << 24  // hit an area light's sphere: its surface is shaded (default matte), Ld valid
};

// hit_s of a compacted slot: sample index (bits 0-15) | material, or light index for HS_LIGHT records
// (bits 16-23; 0xff = a miss with infinite lights) | flags
enum : uint32_t {
    HS_LE = 1u << 28,     // HS_LIGHT: the light sphere faces the camera ray (Le(wo) counts)
    HS_LSURF = 1u << 29,  // HS_LIGHT: a light sphere's surface, shaded with the default matte material
    HS_LIGHT = 1u << 30,  // a light seen directly (no mesh surface, no Mo())
    HS_SSS = 1u << 31     // a mesh surface whose material has a MultipoleBSSRDF
};

// Per camera sample: flags and the slot of its surface hit; per surface hit (compacted, one
// slot per REC_SURF sample of the whole batch): direct light, Mo() query, Mo().
struct SampleRecs {
    uint32_t *flags;
    uint32_t *spill;  // per extended-tile pixel: OR of its samples' REC_XLO..REC_YHI bits
    int32_t *slot;   // hit slot of a REC_SURF sample, else -1
    float *ld;       // [hits][ROW] UniformSampleAllLights result
    float4 *hit_a;   // [hits] t, b1, b2, triangle id (bits)            (primary_kernel)
    float4 *hit_b;   // [hits] ray direction, pixel index (bits)
    uint32_t *hit_s; // [hits] sample index (bits 0-15) | material (16-23) | needs Mo() (bit 31)
    float4 *hit_q;   // [hits] Mo() query p.xyz, cos(theta_o); w = -1 when the hit needs no Mo()
    int *hit_count;  // device counter of hit slots (shared by every tile of a batch)
    float4 *mo4;     // [hits][kGroups] Mo() per band group (mo_band.h layout)
    float4 *xyz;     // [hits] the sample's filtered XYZ (assemble_kernel)
    float4 *hit_alb; // [hits] albedo texture lookup (RGB) of a textured BSSRDF hit (shade_tex_kernel)
    float4 *hit_frame; // [hits][2] bump-mapped shading normal nn and dpdu direction sn (shade_tex_kernel)
};

// SurfacePointTask's random-walk paths (usepoissonpointfinder): one lane per path, candidates of
// path i at out[i * kPoissonCand ...], their count in count[i] (render.hip).
constexpr int kPoissonDepth = 30, kPoissonCand = kPoissonDepth - 3;
struct PoissonWalk {
    V3 origin;        // pCamera
    SphereView bound; // the scene's bounding sphere (ReverseOrientation sphere at its centre)
    uint32_t seed, path0;
    int npaths;
};
__global__ void poisson_walk_kernel(RenderScene sc, PoissonWalk w, SurfacePoint *out, int *count);
template <bool EMIT, bool INCENTER>
__global__ void tess_kernel(RenderScene sc, int mesh, int ntri, int64_t base, float min_dist, int64_t *counts,
                            const int64_t *offs, SurfacePoint *out);

__global__ void irradiance_kernel(RenderScene sc, const float *sp_p, const float *sp_n, const float *sp_eps,
                                  const uint32_t *sp_mat, const float *sp_uv, int n, uint32_t seed, float *E_out);

__global__ void primary_kernel(RenderScene sc, PieceList pl, SampleRecs rec0);
struct DirectTerms;
// inf_st (null without infinite lights): per lane, the radiance-map lookup coordinates (s, t)
// of the light-sampled and the BSDF-sampled direction of an infinite light's EstimateDirect
__global__ void shade_direct_kernel(RenderScene sc, SampleRecs rec, int spp, uint32_t seed, int max_hits, int ns_max,
                                    DirectTerms *terms, float4 *inf_st);
// Per surface hit of a material with textures: the camera ray's differentials (scaled by
// 1/sqrt(spp)), ComputeDifferentials, the albedo lookup (-> hit_alb) and the bumped shading frame
// (-> hit_frame), before shade_direct_kernel reads them.
__global__ void shade_tex_kernel(RenderScene sc, SampleRecs rec, int spp, uint32_t seed, int max_hits);
__global__ void shade_nolight_kernel(RenderScene sc, SampleRecs rec, int max_hits);
template <bool kInf>
__global__ void direct_combine_kernel(RenderScene sc, SampleRecs rec, int max_hits, int ns_max,
                                      const DirectTerms *terms, const float4 *inf_st);
// Li assembly per slot (L = Le + SSS + Ld, sample filter, ToXYZ), then the box-filtered film.
__global__ void assemble_kernel(RenderScene sc, SampleRecs rec, int max_hits);
// Tile-cost probe: one camera ray through the centre of every pixel of [x0, x1) x [y0, y1);
// cls[i] = 0 miss or light, 1 mesh surface, 2 BSSRDF surface (render_host.hip tile_costs).
__global__ void probe_kernel(RenderScene sc, int x0, int x1, int y0, int y1, uint8_t *cls);
__global__ void sky_kernel(RenderScene sc, SampleRecs rec, int max_hits);
__global__ void film_kernel(RenderScene sc, PieceList pl, SampleRecs rec0);

}  // namespace mpss
