/*
 * oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, single precision where the reference is single
 * precision, double where it is double) of pbrt-v2-skin's multipole
 * subsurface-scattering hot path.  It is the parity checker for the HIP product
 * in pbrt-v2-skin_amd/; nothing outside tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.
 *
 * Parity status: the reference ships no golden vectors for this path and its
 * binary cannot be built or run here (SURVEY.md section 8c records the denial),
 * so this restatement is "parity unpinned" against reference outputs.  It is
 * pinned instead by the reference's own physics self-checks, restated as tests:
 *   - kissfft vs brute-force DFT   (libkissfft/test/test_vs_dft.c)
 *   - MPC profile integral vs totalReflectance (src/multipole/test/test.cpp:74-75)
 *   - Mo() at maxError -> 0 equals the brute-force point sum (diffusionutil.h:175-210)
 *   - the analytic single dipole DiffusionReflectance (diffusionutil.h:38-83, o_diffusion_*
 *     below) as a closed-form Rd: its TotalReflectance against Jensen's closed-form total
 *     diffuse reflectance, and Mo() with it against the brute-force point sum
 * Every function cites the reference file:line it follows.
 *
 * Build: make -C oracle  (gcc -O2 -ffp-contract=off, no -ffast-math)
 */
#ifndef MPSS_ORACLE_H
#define MPSS_ORACLE_H
#include <stdint.h>

#define O_NB 30 /* nSpectralSamples, src/core/spectrum.h:46 */

#ifdef __cplusplus
extern "C" {
#endif

/* ---- spectrum (src/core/spectrum.h:291-393, spectrum.cpp:60-193) ---- */
float o_average_spectrum_samples(const float *lambda, const float *vals, int n, float l0, float l1);
void o_from_sampled(const float *lambda, const float *vals, int n, float out[O_NB]);
void o_from_rgb(const float rgb[3], int illuminant, float out[O_NB]);
/* SampledSpectrum::ToRGB = ToXYZ + XYZToRGB (spectrum.h:51-55, 374-398) */
void o_to_rgb(const float s[O_NB], float rgb[3]);
float o_y(const float s[O_NB]);
void o_to_xyz(const float s[O_NB], float xyz[3]);

/* ---- skin coefficients (materials/skincoeffs.h:38-158, layeredskin.cpp:39-89) ---- */
typedef struct {
    float roughness, nmperunit;
    float f_mel, f_eu, f_blood, f_ohg;
    float layer_thickness_nm[2];
    float layer_ior[2];
} o_skin_params;
void o_skin_layers(const o_skin_params *p, float mua[2][O_NB], float musp[2][O_NB],
                   float thickness[2], float eta[2]);

/* ---- kissfft v1.3.0 restated, kiss_fft_scalar = double ---- */
typedef struct { double r, i; } o_cpx;
void o_kiss_fft(int nfft, int inverse, const o_cpx *fin, o_cpx *fout);
void o_kiss_fftndr2(int rows, int cols, const double *in, o_cpx *out);   /* forward */
void o_kiss_fftndri2(int rows, int cols, const o_cpx *in, double *out);  /* inverse (unscaled) */

/* ---- MPC (MultipoleProfileCalculator.cpp:151-426, DipoleCalculator.cpp:38-91) ---- */
typedef struct { float ior, thickness, mua, musp; } o_layer_spec;
/* Returns number of (dsq, R, T) entries written before resampling; caller frees *out arrays via o_free. */
int o_mpc_profile(int nlayers, const o_layer_spec *specs, float step, int desired_length,
                  int lerp_on_thin_slab, int resample, float **dsq, float **refl, float **trans,
                  float *total_r, float *total_t);
void o_free(void *p);
/* MPC_ResampleDistribution (:429-448) of an unresampled o_mpc_profile output at distances points[] */
void o_mpc_resample(int len, const float *d, const float *R, const float *T, int n, const float *points, float *r,
                    float *t);
/* MPC_ResampleForUniformDistanceSquaredDistribution (:404-426) to `target` entries */
void o_mpc_resample_uniform(int len, const float *d, const float *R, int target, float *out);
float o_dipole_rd(float eta0, float etad, float d, float mua, float musp, int zi, int lerp, float dsq);

/* Per-channel profile (multipole.cpp:241-295). table: [O_NB][*len] floats (channel-major). */
int o_compute_profile(const float mua[2][O_NB], const float musp[2][O_NB], const float eta[2],
                      const float thickness[2], int desired_length, int lerp_on_thin_slab,
                      int nthreads, float **table, float rcp[O_NB], float spacing[O_NB],
                      float total_r[O_NB]);
/* sampleProfile (multipole.cpp:60-73) for one channel */
float o_sample_profile(const float *data, int len, float rcp, float dsq);

/* ---- rho table (multipole.cpp:466-549; reflection.cpp:132-153,228-240,391-403,548-580,623-652) ---- */
void o_rho_table(float roughness, float eta, int n_entries /*1025*/, int sqrt_samples /*256*/,
                 int nthreads, float *hd, float *hh);
/* doublerefsslf: fixed != 0 -> FixedFresnelDielectric (reflection.h:315-324) in the Microfacet */
void o_rho_table_ex(float roughness, float eta, int fixed, int n_entries, int sqrt_samples, int nthreads, float *hd,
                    float *hh);
uint32_t o_mt_first(uint32_t seed, int n, uint32_t *out); /* MT19937 stream check */
/* MT19937, core/rng.cpp (RNG::Seed, RNG::RandomUInt) */
typedef struct { uint32_t mt[624]; int mti; } o_mt;
void o_mt_seed(o_mt *r, uint32_t seed);
uint32_t o_mt_u32(o_mt *r);

/* ---- octree + Mo (diffusionutil.h:86-234; multipolesubsurface.cpp:301-321) ---- */
typedef struct o_octree o_octree;
o_octree *o_octree_build(int n, const float *p /*n*3*/, const float *n_ /*n*3*/, const float *E /*n*O_NB*/,
                         const float *area /*n*/);
void o_octree_free(o_octree *t);
int o_octree_num_nodes(const o_octree *t);
/* Mo for q queries; rd_table channel-major [O_NB][len]; counters (nullable): per query nodes, points */
void o_mo_batch(const o_octree *t, int q, const float *pts /*q*3*/, const float *rd_table, int len,
                const float rcp[O_NB], float max_error, float *mo /*q*O_NB*/, int32_t *n_nodes,
                int32_t *n_points, int nthreads);
/* Mo with an rgbprofile material: rd_table rows 0..2 = R, G, B profiles [3][len], rcp[3];
   Rd = SampledSpectrum::FromRGB(reflectance) of the three lookups (multipole.cpp:85-107) */
void o_mo_batch_rgb(const o_octree *t, int q, const float *pts, const float *rd_table, int len, const float rcp[3],
                    float max_error, float *mo, int32_t *n_nodes, int32_t *n_points, int nthreads);
/* DiffusionReflectance (diffusionutil.h:38-83): the single-dipole Rd functor */
typedef struct {
    float zpos[O_NB], zneg[O_NB], sigmap_t[O_NB], sigma_tr[O_NB], alphap[O_NB];
    float A;
} o_diffusion;
void o_diffusion_init(const float sigma_a[O_NB], const float sigmap_s[O_NB], float eta, o_diffusion *d);
void o_diffusion_eval(const o_diffusion *d, float d2, float out[O_NB]);
void o_diffusion_total(const o_diffusion *d, float out[O_NB]);
/* Mo with DiffusionReflectance as the Rd functor (dipolesubsurface.cpp:171-172) */
void o_mo_batch_diffusion(const o_octree *t, int q, const float *pts, const o_diffusion *d, float max_error,
                          float *mo, int32_t *nn, int32_t *np, int nthreads);
/* Flatten for inspection: pre-order nodes (same order as the product's layout contract) */
int o_octree_export(const o_octree *t, float *node_p /*N*3*/, float *node_area, float *node_et /*N*O_NB*/,
                    float *bmin /*N*3*/, float *bmax /*N*3*/, int32_t *depth, int32_t *skip,
                    int32_t *leaf_first, int32_t *leaf_count, int32_t *point_order);
void o_octree_bounds(const o_octree *t, float bmin[3], float bmax[3]);

/* ---- per-pixel path (render.c): tessellation, irradiance, Li, film ---- */
typedef struct {  /* SurfacePoint, renderers/surfacepoints.h:45-55 (44-byte record) */
    float p[3], n[3], u, v;
    uint32_t material;
    float area, ray_eps;
} o_surface_point;
typedef struct o_scene o_scene;
/* ImageTexture with UVMapping2D (texture.c): MIPMap levels of the converted texels */
typedef struct {
    int nch, nlevels, wrap, trilinear; /* wrap: 0 repeat, 1 black, 2 clamp */
    float max_aniso, su, sv, du, dv;
    int w[16], h[16];
    float *lv[16];
} o_tex;
int o_tex_build(o_tex *t, int W, int H, const float *texels, int is_float, float shift, float scale, float gamma,
                int wrap, int trilinear, float max_aniso, float su, float sv, float du, float dv);
void o_tex_free(o_tex *t);
void o_tex_eval(const o_tex *t, float u, float v, float dudx, float dvdx, float dudy, float dvdy, float out[3]);
int o_imagemap_lookup(int W, int H, const float *texels, int is_float, float shift, float scale, float gamma,
                      int wrap, int trilinear, float max_aniso, float su, float sv, float du, float dv, int n,
                      const float *uvd, float *out);

o_scene *o_scene_create(int xres, int yres, const float *raster_to_camera, const float *camera_to_world);
int o_scene_add_material(o_scene *s, const float *R, const float *T /* nullable: black */, const float *albedo,
                         float mix, float roughness, float eta, int fixed_fresnel, const float *rho, int n_rho,
                         int is_mc, const float *rd_table, int L, const float *rcp);
int o_scene_add_mesh(o_scene *s, int nv, const float *P, const float *N, const float *S, const float *uv, int nt,
                     const int32_t *idx, const float *o2w, const float *w2o, int flip, int material);
int o_scene_add_sphere_light(o_scene *s, const float *c, float r, const float *Le, int nsamples);
/* texels: W x H RGB as ReadImage returns them, or NULL for a light without "mapname" */
int o_scene_add_infinite_light(o_scene *s, const float *L, int nsamples, const float *l2w, const float *w2l, int W,
                               int H, const float *texels);

/* FindPoissonPointDistribution with one task (replay-mode random numbers); returns the number of
 * points written to out (<= cap), -1 if cap is too small, -2 if no BSSRDF surface was found */
long o_poisson_points(o_scene *s, float min_dist, int quick, uint32_t seed, o_surface_point *out, long cap);

/* envmap.c: InfiniteAreaLight's radiance MIPMap level 0 and Distribution2D */
typedef struct {
    int tw, th, nu, nv;
    float *tex, *func, *cdf, *rint, *mcdf;
    float mint;
} o_envmap;
int o_envmap_build(int W, int H, const float *texels, o_envmap *m);
void o_envmap_free(o_envmap *m);
void o_envmap_lookup(const o_envmap *m, float s, float t, float out[3]);
void o_envmap_sample(const o_envmap *m, float u0, float u1, float uv[2], float *pdf);
float o_envmap_pdf(const o_envmap *m, float u, float v);
long o_tessellate(const o_scene *s, float min_dist, int incenter, o_surface_point *out, long cap);

/* ---- the reference sampler (samplerrenderer.cpp:60-225, lowdiscrepancy.cpp:40-93,
 *      montecarlo.{h:254-333, cpp:200-250}, multipolesubsurface.cpp:72-152) ----
 * Sample values of the film's whole sample extent ((xres+1) x (yres+1) pixels, spp a power of two)
 * as the reference's render tasks draw them with `cores` = NumSystemCores(); one row of K floats
 * per camera sample (pixel-major, then sample): image u, v, then per light (scene order) and light
 * sample j: light pos u0, u1, BSDF component, BSDF dir u0, u1. li_draws: RNG values Li draws per
 * camera-ray hit (6 with maxdepth > 0). Returns K; vals may be NULL to query it. */
int o_replay_render_table(o_scene *s, int spp, int cores, int li_draws, int nthreads, float *vals);
/* The same for the pixels [vx0, vx1) x [vy0, vy1) of the sample extent only: row of pixel (x, y),
 * sample i at vals[(((y - vy0) * (vx1 - vx0) + x - vx0) * spp + i) * K]; tasks whose sub-window
 * misses the window are not run. */
int o_replay_render_table_window(o_scene *s, int spp, int cores, int li_draws, int nthreads, int vx0, int vx1,
                                 int vy0, int vy1, float *vals);
/* IrradianceTask's RNG(47 k) scrambles: scr[(i * nlights + l) * 2 + {0, 1}] */
void o_replay_irradiance_scr(int n, int nlights, int cores, uint32_t *scr);
/* o_irradiance / o_render_tile with the reference sampler's values instead of counter hashes */
void o_irradiance_replay(o_scene *s, int n, const o_surface_point *pts, const uint32_t *scr, int nthreads, float *E);
void o_render_tile_replay(o_scene *s, int spp, const float *vals, int K, int x0, int x1, int y0, int y1,
                          int nthreads, float *xyzw);
/* o_render_tile_replay with a windowed table (o_replay_render_table_window's window) */
void o_render_tile_replay_window(o_scene *s, int spp, const float *vals, int K, int vx0, int vx1, int vy0, int vy1,
                                 int x0, int x1, int y0, int y1, int nthreads, float *xyzw);
/* CPU baseline: SamplerRenderer::Render's task loop -- the sub-windows order[0..norder) of
 * nTasks = norder tasks (o_render_task_count) taken from one shared counter by nthreads workers
 * until `seconds` pass; hash sampler. Returns pixels rendered; *tasks_done, *elapsed (s). */
long o_cpu_baseline(o_scene *s, int spp, uint32_t seed, int cores, int nthreads, double seconds, const int *order,
                    int norder, long *tasks_done, double *elapsed);
/* RoundUpPow2(max(32 * cores, xres * yres / 256)) (samplerrenderer.cpp:206-207) */
int o_render_task_count(int xres, int yres, int cores);
/* Sampler::ComputeSubWindow (sampler.cpp:55-78): out = x0, x1, y0, y1 */
void o_sub_window(int num, int count, int xs, int xe, int ys, int ye, int *out);
void o_irradiance(o_scene *s, int n, const o_surface_point *pts, uint32_t seed, int nthreads, float *E);
void o_scene_set_octree(o_scene *s, int n, const float *p, const float *nrm, const float *E, const float *area,
                        float max_error);
void o_render_tile(o_scene *s, int spp, uint32_t seed, int x0, int x1, int y0, int y1, int nthreads, float *xyzw);
void o_scene_free(o_scene *s);
/* LayeredSkin "albedo" (which = 0, a spectrum imagemap) or "bumpmap" (which = 1, a float imagemap) */
/* rgbprofile material: its rd table's rows 0..2 are the R, G, B profiles (o_mo_batch_rgb) */
int o_scene_set_material_rgb(o_scene *s, int material, int rgb);
int o_scene_set_material_no_bssrdf(o_scene *s, int material, int no_bssrdf);
int o_scene_set_material_texture(o_scene *s, int material, int which, int W, int H, const float *texels,
                                 float shift, float scale, float gamma, int wrap, int trilinear, float max_aniso,
                                 float su, float sv, float du, float dv);

/* ---- Monte-Carlo layered profile (mc.c; src/renderers/mcprofile.cpp:120-341,443-498) ---- */
typedef struct { float mua, musp, ior, thickness; } o_mc_layer;
/* Traces photons [photon_begin, photon_end) of nphotons and ADDS un-normalised ring tallies to
 * raw_r / raw_t [nseg]; extent_out = mfp_range * mean mfp. */
int o_mc_profile(const o_mc_layer *layers, int n, float mfp_range, int nseg, uint64_t nphotons, uint64_t seed,
                 uint64_t photon_begin, uint64_t photon_end, double *raw_r, double *raw_t, double *extent_out);

#ifdef __cplusplus
}
#endif
#endif
