/*
 * mpss.h -- C ABI of libmpss, the MI355X-native multipole subsurface-scattering path for
 * pbrt-v2-skin (Thomi6York/pbrt-v2-skin).  Plain C: no C++ or torch types cross it.
 *
 * It replaces, one for one, the pieces of pbrt's SurfaceIntegrator plugin surface for
 * "multipolesubsurface" + "layeredskin" (reference paths relative to /root/reference):
 *
 *   mpss_create / mpss_destroy      CreateMultipoleSubsurfaceIntegrator + dtor
 *                                   (src/integrators/multipolesubsurface.cpp:306-320 [file 390-404],
 *                                    src/integrators/multipolesubsurface.h:46-63)
 *   mpss_add_layeredskin            CreateLayeredSkinMaterial + LayeredSkin::LayeredSkin parse-time
 *                                   precompute (src/materials/layeredskin.cpp:39-123, 222-262;
 *                                   src/core/multipole.cpp:241-295, 371-406, 466-549)
 *   mpss_set_material_tables        MultipoleBSSRDFData(pData, rhoData) for externally built tables
 *                                   (src/core/multipole.h:44-59)
 *   mpss_get_material_tables        read back Profile::data / rcpDsqSpacing / RhoData::hd
 *   mpss_set_irradiance_points      the octree build at the end of Preprocess
 *                                   (multipolesubsurface.cpp:301-321 [file], diffusionutil.h:94-173)
 *   mpss_mo_batch                   SubsurfaceOctreeNode::Mo over a batch of shading points
 *                                   (diffusionutil.h:175-210 via multipolesubsurface.cpp:364)
 *
 * Error convention: every entry point returns MPSS_OK (0) or a negative MPSS_ERR_* code and
 * records a message retrievable with mpss_last_error() (thread-local). No exception ever
 * crosses the boundary; the reference's Severe()/abort() paths become error returns.
 * Thread safety (SamplerRendererTask calls Li from every worker thread, parallel.cpp:800-878):
 * mpss_mo_batch, mpss_render_tile(s) and the query functions may be called concurrently from
 * several host threads, each with its own stream; every call takes its own device workspace.
 * Calls that change the context (materials, meshes, lights, camera, points, preprocess) are
 * serialized against each other. Those that replace device state a render reads (the octree via
 * mpss_set_irradiance_points / mpss_preprocess, the scene buffers, the replay table) first wait
 * until every render / mo_batch call in flight has queued its kernels, then for those kernels; a
 * render started after such a call sees the new state. Which of two racing calls goes first is
 * the caller's to order.
 * Pointers named *_dev are HIP device pointers (e.g. torch CUDA tensors' data_ptr());
 * all other arrays are caller-owned host memory that is copied in.
 * stream: a hipStream_t (NULL = legacy default stream).
 */
#ifndef MPSS_H
#define MPSS_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPSS_NBANDS 30 /* nSpectralSamples, src/core/spectrum.h:46 */

enum {
    MPSS_OK = 0,
    MPSS_ERR_INVALID = -1,   /* bad argument / state */
    MPSS_ERR_INTERNAL = -2,  /* algorithmic failure (e.g. degenerate point cloud) */
    MPSS_ERR_HIP = -3,       /* HIP runtime error */
    MPSS_ERR_NOMEM = -4
};

typedef struct mpss_ctx mpss_ctx;

/* Integrator parameters, defaults as CreateMultipoleSubsurfaceIntegrator (file lines 393-401). */
typedef struct {
    int device;                /* HIP device ordinal */
    int max_depth;             /* "maxdepth" = 5 */
    float max_error;           /* "maxerror" = .05 */
    float min_sample_distance; /* "minsampledistance" = .25 */
    float mix;                 /* "mix" = .5 */
    int show_irradiance_points;/* "showirradiancepoints" = false */
    int incenter;              /* "incenter" = false */
    int quick_render;          /* PbrtOptions.quickRender: maxError *= 4, minDist *= 4 */
    int exact_mo;              /* Mo gather kernel. 1: sums in the reference recursion order
                                  (bit-exact, slower); 0 (default): spectrally sharded kernel (band
                                  groups pinned to XCDs); 2: packet kernel. 0 and 2 evaluate the same
                                  terms with one running sum per band and agree bit for bit */
    int kernel_timing;         /* 1: time every render kernel with HIP events (mpss_get_render_stats) */
    int count_traversal;       /* 1: the Mo() gather counts the octree nodes / points it reads (slower);
                                  2: the same with the exact-zero reach pruning off, so every band
                                  group walks exactly the records of the reference's Mo() recursion
                                  (SURVEY 8d algorithmic bytes; results unchanged) */
    int profile_on_host;       /* 1: build LayeredSkin profiles and rho_hd tables on the host CPU
                                  (threads); 0 (default): on the GPU (profile_gpu.hip, rho_gpu.hip) */
    int64_t max_batch_samples; /* camera samples per render batch (default 1 << 26: a whole C2 frame
                                  in two batches, one Mo() launch each); the workspace grows to the
                                  largest batch rendered, sized for the worst case (every sample a
                                  hit): ~280 B/sample, 18.8 GB for a full 2^26 batch of the 288 GB;
                                  at least 2^10. The reference sampler also closes a batch before
                                  its pieces' bounding box x spp x 22 floats (skin.pbrt) passes 2^31
                                  floats, and generates its values for windows of as many
                                  consecutive batches as that holds */
    int use_poisson_point_finder; /* "usepoissonpointfinder" = false: SurfacePoints by random-walk
                                  dart throwing (FindPoissonPointDistribution) instead of tessellation */
    int sampler;               /* MPSS_SAMPLER_HASH (default): counter-hash scrambled (0,2) sequences, a
                                  sample's values depend only on (seed, pixel, index) -- any tiling,
                                  any GPU count; MPSS_SAMPLER_REFERENCE: the reference's own streams
                                  replayed -- LDSampler's per-task MT19937 (RNG(task)) scrambles and
                                  shuffles, Li's 6 draws per camera hit, IrradianceTask's RNG(47 k)
                                  (samplerrenderer.cpp:60-225, montecarlo.cpp:200-250,
                                  multipolesubsurface.cpp:72-152); seeds are then ignored and spp is
                                  rounded up to a power of two as LDSampler does */
    int replay_cores;          /* NumSystemCores() of the reference run being replayed (its task
                                  counts, samplerrenderer.cpp:207, multipolesubsurface.cpp:198) = 8 */
    int octree_on_host;        /* 1: build the irradiance octree on the host (serial Insert in point
                                  order, octree.cpp); 0 (default): level-synchronous build on the GPU
                                  (octree_gpu.hip), the same tree bit for bit */
    /* Choices of the spectrally sharded gather (exact_mo = 0). None of these three changes a result bit
       (mo_common_grid, below, does within its stated bound). */
    int mo_band_dealing;       /* 0 (default): the 30 bands dealt into 8 groups of adjacent profile
                                  reach; 1: snake rounds (every group one of the 8 longest reaches) */
    int mo_work_stealing;      /* 1 (default): a workgroup whose band group runs dry moves on to the
                                  next group with work left; 0: each stays on its own group (XCD) */
    int mo_near_field;         /* profile entries per band kept in LDS: 5088 (default; two 1024-thread
                                  workgroups per CU, 8 waves per SIMD) or 10236 (one workgroup per CU
                                  holds the whole 160 KB, 4 waves per SIMD). With the common grid the
                                  gather waits on memory latency more than on the L2 request rate, and
                                  8 waves hide more of it (C2, round 4's first grid: 59.4 vs 68.8 ms
                                  per frame) */
    int tessellate_on_host;    /* 1: Preprocess tessellates on the host (threads over triangles,
                                  scene.cpp); 0 (default): one GPU thread per triangle (render.hip
                                  tess_kernel), the same points bit for bit (tessellate.h) */
    int mo_common_grid;        /* 1 (default): the sharded gather reads a band group's lookups past
                                  the exact LDS near field, as far as the resampling stays within 2e-6
                                  of each band's own value or 1e-13 of the band's peak (measured at
                                  every band knot when the material is added; at most 65,536 rows per
                                  group), from ONE table of the group's bands resampled onto its
                                  coarsest d^2 grid: two 16-byte loads from one 32-byte sector per
                                  lookup instead of four 8-byte lerp pairs; farther lookups read the
                                  bands' own tables. Results differ from the per-band gather by at most
                                  that error per term (mpss_get_gather_info; C2 full frame vs the
                                  oracle: 4.3e-6 relative). 0: per-band tables everywhere
                                  (bit-identical to the packet kernel) */
} mpss_config;

enum { MPSS_SAMPLER_HASH = 0, MPSS_SAMPLER_REFERENCE = 1 };

void mpss_config_defaults(mpss_config *cfg);
int mpss_create(const mpss_config *cfg, mpss_ctx **out);
void mpss_destroy(mpss_ctx *ctx);
const char *mpss_last_error(void);
int mpss_abi_version(void);

/* LayeredSkin parameters, defaults as CreateLayeredSkinMaterial (layeredskin.cpp:234-257). */
typedef struct {
    float roughness;      /* 0.4 */
    float nmperunit;      /* 100e6 */
    float f_mel, f_eu, f_blood, f_ohg;  /* 0.15, 1, 0.002, 0.3 */
    float ga_epi, ga_derm, b_derm;      /* 0.9, 0.8, 0.4 (carried, unused by the multipole path) */
    float layer_thickness_nm[2];        /* "skinlayer layers" thickness (nm) */
    float layer_ior[2];                 /* "skinlayer layers" ior */
    float albedo[MPSS_NBANDS];          /* constant "albedo" texture value (default Spectrum(1)) */
    float Kr[MPSS_NBANDS];              /* "Kr" (default Spectrum(1)): Microfacet reflection */
    float Kt[MPSS_NBANDS];              /* "Kt" (default Spectrum(1)): MicrofacetTransmission */
    int desired_length;   /* "desiredlength" = 512 */
    int lerp_on_thin_slab;/* "lerponthinslab" = true */
    int double_ref_sslf;  /* "doublerefsslf" = false (FixedFresnelDielectric) */
    int use_monte_carlo;  /* "usemontecarlo" = false: the profile is a Monte-Carlo random walk per band
                             (ComputeMonteCarloProfile, multipole.cpp:298-368) on this context's GPU,
                             and Li uses Ft = 1 (multipolesubsurface.cpp:283-286) */
    uint64_t photons;     /* "photons" = 10000000 (per band) */
    int rgb_profile;      /* "rgbprofile" = false: ComputeRGBMultipoleProfile (multipole.cpp:408-451) --
                             the layers' 30-band mua / musp reduced to RGB (ToRGBSpectrum), three
                             profiles, Rd(d^2) = FromRGB(reflectance) of the three lookups
                             (multipole.cpp:85-107); the exported table then holds the R, G, B
                             profiles in rows c % 3. Mo(): the sharded gather reads the three
                             profiles in every band group (its common grid built over them) and
                             takes FromRGB per record into the group's bands; exact_mo = 1 runs the
                             reference-order gather */
    int gen_profile;      /* "genprofile" = true. false: no profile is prepared (preparedBSSRDFData =
                             NULL, layeredskin.cpp:70,120-122) and the material carries no subsurface
                             term: its surfaces get no Mo() term and its irradiance points are lit as
                             a point without a MultipoleBSSRDF (Ft = 1, no albedo^mix:
                             multipolesubsurface.cpp:100-107,139-140). (The reference would read the
                             NULL profile through MultipoleBSSRDF::rho / reflectance,
                             reflection.cpp:833-843; this is the no-BSSRDF branch it has for that.) */
    int show_irradiance_points;   /* "showirradiancepoints" = false: the material's profile is
                             ComputeIrradiancePointsProfile (multipole.cpp:551-567) -- every band a
                             disc of radius irradiance_point_size, Rd = 1 / (pi r^2) for d < r -- and
                             its rho table ComputeRoughRhoData's two zeros (:569-572, Ft = 1):
                             each irradiance point shows as a disc of its irradiance */
    float irradiance_point_size;  /* "irradiancepointsize" = 0.002 (world units) */
} mpss_layeredskin;

void mpss_layeredskin_defaults(mpss_layeredskin *m);
/* Builds the 30-band multipole profile and the 1025-entry rho_hd table; returns a material id. */
int mpss_add_layeredskin(mpss_ctx *ctx, const mpss_layeredskin *m, uint32_t *material_id);
/* Install precomputed tables: rd_table is channel-major [30][length]; rcp[30] = rcpDsqSpacing;
 * rho_hd[n_rho] (scalar, replicated over bands); albedo[30]. */
int mpss_set_material_tables(mpss_ctx *ctx, const float *rd_table, uint32_t length, const float *rcp,
                             const float *rho_hd, uint32_t n_rho, const float *albedo, int is_monte_carlo,
                             uint32_t *material_id);
/* The dipolesubsurface integrator's Rd functor, DiffusionReflectance(sigma_a, sigmap_s, eta)
 * (integrators/diffusionutil.h:38-83, built per hit at dipolesubsurface.cpp:171): a material whose
 * mpss_mo_batch evaluates the closed-form single dipole per band inside the reference-order gather
 * (SubsurfaceOctreeNode::Mo, diffusionutil.h:175-210; nothing pruned). sigma_a / sigmap_s: [30].
 * It is not a surface material: mpss_add_mesh rejects it (the dipole integrator's Li is not part of
 * this library). */
int mpss_add_dipole_material(mpss_ctx *ctx, const float *sigma_a, const float *sigmap_s, float eta,
                             uint32_t *material_id);
/* Query sizes first with NULL buffers: *length and *n_rho are always written. */
int mpss_get_material_tables(mpss_ctx *ctx, uint32_t material_id, float *rd_table, uint32_t *length, float *rcp,
                             float *rho_hd, uint32_t *n_rho, float *total_reflectance);
/* How the sharded gather evaluates material `id` (mpss_config.mo_common_grid): *common_grid = 1 when
 * its far field is read from the resampled group tables, 0 for per-band tables (or a material the
 * sharded gather does not run: dipole). rel_err / l1_err (nullable, 30 floats): the measured
 * resampling error per band (see mo_common_grid; rgbprofile: entries 0..2, its R, G, B profiles),
 * 0 without a common grid. */
int mpss_get_gather_info(mpss_ctx *ctx, uint32_t id, int *common_grid, float *rel_err, float *l1_err);

/* Texture "imagemap" (CreateImageSpectrumTexture / CreateImageFloatTexture, textures/imagemap.cpp:
 * 110-180) with the default "uv" mapping (UVMapping2D, core/texture.cpp:88-98). texels = the image
 * ReadImage returns (width x height RGB triples, row-major, row t = 0 first); they pass through
 * convertIn (RGB: scale * (pow(c, gamma) + shift); float: scale * (pow(y(c), gamma) + shift)) and
 * build the MIPMap (Lanczos resampling to powers of two, box-filtered levels; core/mipmap.h).
 * width = 0 or texels = NULL: the file could not be read; the reference then uses a one-valued
 * 1x1 map of powf(scale * (1 + shift), gamma) (imagemap.cpp:76-81). Lookups filter with EWA
 * (mipmap.h:272-363), or trilinearly with "trilinear". */
typedef struct {
    int width, height;
    const float *texels;
    int is_float;          /* 1: a "float" texture (bumpmap), 0: "color"/"spectrum" (albedo) */
    float shift, scale, gamma;   /* "shift" = 0, "scale" = 1, "gamma" = 1 (this fork's convertIn) */
    int wrap;              /* "wrap": 0 repeat (default), 1 black, 2 clamp */
    int trilinear;         /* "trilinear" = false */
    float max_anisotropy;  /* "maxanisotropy" = 8 */
    float uscale, vscale, udelta, vdelta;  /* "uscale" = "vscale" = 1, "udelta" = "vdelta" = 0 */
} mpss_imagemap;
void mpss_imagemap_defaults(mpss_imagemap *t);
int mpss_add_imagemap(mpss_ctx *ctx, const mpss_imagemap *t, uint32_t *texture_id);
/* LayeredSkin's texture parameters (CreateLayeredSkinMaterial, layeredskin.cpp:246-249): "albedo"
 * (a spectrum imagemap; the constant albedo[] of mpss_layeredskin applies when -1) and "bumpmap"
 * (a float imagemap, Material::Bump on the shading geometry; -1: none). The albedo texture is
 * evaluated per irradiance point (no differentials) and per camera hit (ray differentials). */
int mpss_set_material_textures(mpss_ctx *ctx, uint32_t material_id, int32_t albedo_texture, int32_t bump_texture);

/* Irradiance points (IrradiancePoint p, n, E, area; irradiancepoint.h:36-45) -> device octree. */
int mpss_set_irradiance_points(mpss_ctx *ctx, uint32_t n, const float *p, const float *nrm, const float *E,
                               const float *area);
/* Octree statistics: node count, max depth, point count. */
int mpss_octree_info(mpss_ctx *ctx, uint32_t *n_nodes, uint32_t *max_depth, uint32_t *n_points);
/* The context's device octree as the gather reads it (any pointer may be null): nodes n_nodes x 64 B
 * (pre-order NodeHdr records: centroid, sumArea, box, skip, leaf range, depth, flags, live point
 * count), node_et n_nodes x 32 floats (30 bands + 2 zero pads), pt_hdr n_points x 4 floats {p, area;
 * sign bit: black E}, pt_e n_points x 32 floats, pt_index n_points original point indices (each
 * leaf's non-black points first). Sizes from mpss_octree_info. Synchronous. */
int mpss_octree_export(mpss_ctx *ctx, void *nodes, float *node_et, float *pt_hdr, float *pt_e, int32_t *pt_index);

/* Mo for q shading points (p_dev: q*3 floats) with material's Rd profile; mo_dev: q*30 floats.
 * 0 <= q <= 2^30 (q = 0: nothing is launched; larger: MPSS_ERR_INVALID).
 * counters_dev (nullable): q*4 int32 {nodes entered, leaf points evaluated} by the reference
 * recursion (exact_mo = 1 only; else 0), then the same two counts for the kernel's pruned traversal. */
int mpss_mo_batch(mpss_ctx *ctx, uint32_t material_id, uint32_t q, const float *p_dev, float *mo_dev,
                  int32_t *counters_dev, void *stream);

/* ---- scene slice of the per-pixel path (the renderer feeds pbrt's parsed scene through these) ---- */
/* TriangleMesh (shapes/trianglemesh.cpp:43-73): P already in world space (the ctor's ObjectToWorld),
 * N / S in object space (nullable), uv (nullable), o2w / w2o = ObjectToWorld and its inverse
 * (row-major 4x4). */
int mpss_add_mesh(mpss_ctx *ctx, uint32_t nverts, const float *P, const float *N, const float *S, const float *uv,
                  uint32_t ntris, const int32_t *indices, const float *obj_to_world, const float *world_to_obj,
                  int reverse_orientation, uint32_t material_id);
/* AreaLightSource "area" + Shape "sphere" placed by a translation (lights/diffuse.cpp:45-67). */
int mpss_add_sphere_light(mpss_ctx *ctx, const float *center, float radius, const float *Lemit, int nsamples);
/* LightSource "infinite" without "mapname" (CreateInfiniteLight, lights/infinite.cpp:180-188): L is
 * the 30-band L * scale; the light keeps L.ToRGBSpectrum() as its 1x1 radiance map and returns
 * Spectrum(map lookup, SPECTRUM_ILLUMINANT) for Le / Sample_L (infinite.cpp:66-234).
 * light_to_world / world_to_light: row-major 4x4 (only the rotation part is used). Lights join
 * scene->lights in call order, mixed with sphere lights; at most 254 lights. */
int mpss_add_infinite_light(mpss_ctx *ctx, const float *L, int nsamples, const float *light_to_world,
                            const float *world_to_light);
/* LightSource "infinite" with "mapname": texels = the image ReadImage returns (width x height RGB
 * triples, row-major, top row first), before the light multiplies them by L.ToRGBSpectrum(). The
 * MIPMap (Lanczos resampling to powers of two) and the Distribution2D over img(u, v) * sin(theta)
 * are built here (infinite.cpp:66-106, mipmap.h:147-220, montecarlo.h:54-175). */
int mpss_add_infinite_light_map(mpss_ctx *ctx, const float *L, int nsamples, const float *light_to_world,
                                const float *world_to_light, int width, int height, const float *texels);
/* PerspectiveCamera (cameras/perspective.cpp): RasterToCamera and CameraToWorld, row-major 4x4. */
int mpss_set_camera(mpss_ctx *ctx, const float *raster_to_camera, const float *camera_to_world, int xres, int yres);
/* SurfacePoint records (44 B: p[3] n[3] u v materialId area rayEpsilon, renderers/surfacepoints.h:45-55),
 * the "pointsfile" format; set before mpss_preprocess to skip tessellation. */
int mpss_set_surface_points(mpss_ctx *ctx, uint32_t n, const void *records);
int mpss_get_surface_points(mpss_ctx *ctx, void *records, uint32_t *n);
/* The "pointsfile" on disk: a raw array of the 44-byte records in native byte order, as
 * TessellateSurfacePointsRenderer writes it (surfacepoints.cpp:335-347) and Preprocess reads it
 * (multipolesubsurface.cpp:176-181 via ReadBinaryFile, floatfile.h:45-63; a trailing partial
 * record is ignored). load = set_surface_points from the file; save = the current points. */
int mpss_load_pointsfile(mpss_ctx *ctx, const char *path);
int mpss_save_pointsfile(mpss_ctx *ctx, const char *path);
/* Irradiance E[n][30] of the last Preprocess. */
int mpss_get_irradiance(mpss_ctx *ctx, float *E, uint32_t *n);
/* The reference sampler's sample values (mpss_config.sampler = MPSS_SAMPLER_REFERENCE) for the
 * film's whole sample extent at spp (rounded up to a power of two): (yres + 1) x (xres + 1)
 * pixels x spp samples x *k floats -- image u, v, then per light and light sample: light
 * position u0, u1, BSDF component, BSDF direction u0, u1. Query *k and *n_floats with out NULL. */
int mpss_replay_samples(mpss_ctx *ctx, int spp, float *out, uint64_t *n_floats, int *k);
/* MultipoleSubsurfaceIntegrator::Preprocess: tessellation, irradiance (GPU), octree. */
int mpss_preprocess(mpss_ctx *ctx, uint32_t seed);
/* Render pixels [x0,x1) x [y0,y1) at spp samples per pixel; xyzw_dev receives
 * (y1-y0)*(x1-x0) float4 {sum X, sum Y, sum Z, sum of filter weights} (ImageFilm::Pixel). */
int mpss_render_tile(mpss_ctx *ctx, int spp, uint32_t seed, int x0, int x1, int y0, int y1, float *xyzw_dev,
                     void *stream);
/* Render n rectangles (rects[4*i..] = x0, x1, y0, y1) into xyzw_dev[i] in as few kernel batches
 * as the workspace allows (mpss_config.max_batch_samples): one Mo() gather launch covers the
 * shading points of every tile in a batch, which is what fills the GPU. Same results as n
 * mpss_render_tile calls. */
int mpss_render_tiles(mpss_ctx *ctx, int spp, uint32_t seed, int n, const int32_t *rects, float *const *xyzw_dev,
                      void *stream);

/* Cost probe for dealing tiles to GPUs (the bench's multi-GPU path; not a reference entry point):
 * one camera ray through the centre of every pixel, counted per rectangle (rects[4*i..] = x0, x1,
 * y0, y1): sss_hits[i] = rays that hit a surface with a MultipoleBSSRDF (they will run the Mo()
 * gather), surf_hits[i] = rays that hit any mesh. Synchronous; identical counts on every device. */
int mpss_tile_costs(mpss_ctx *ctx, int n, const int32_t *rects, int64_t *sss_hits, int64_t *surf_hits);

/* Accumulated per-kernel statistics of mpss_render_tile / mpss_preprocess since the last reset.
 * Kernel times need kernel_timing = 1; traversal counts need count_traversal = 1. Synchronizes. */
typedef struct {
    double ms_irradiance, ms_camera, ms_shade, ms_film;  /* summed kernel durations */
    int64_t n_irradiance, n_camera, n_shade, n_film;     /* launches */
    int64_t samples;      /* camera samples traced (incl. the tile's one-pixel border) */
    int64_t sss_samples;  /* samples with a surface hit (the Mo() query list; count_traversal only) */
    int64_t mo_nodes;     /* octree node visits of the Mo() gather, summed over band groups */
    int64_t mo_points;    /* leaf point evaluations, summed over band groups */
    int64_t group_nodes[8], group_points[8];  /* the same per band group (8 groups <= 4 bands) */
    int32_t group_bands[8][4];                /* band indices of each group (-1: empty slot) */
    double ms_direct;     /* shading + direct lighting kernel (ms_camera: primary rays only) */
    int64_t n_direct;
    /* count_traversal: iterations of the gather's node loop and leaf-point loop summed over waves
     * (one wave = 64 queries x one band group); 64 x iterations / visits = 1 / lane efficiency */
    int64_t mo_wave_node_iters, mo_wave_point_iters;
    /* count_traversal: Rd table lookups inside the profile (lane x band), and how many of them
     * fall in the first 4096 / 8192 / 16384 entries of their band */
    int64_t mo_lookups, mo_lookups_near[3];
    /* count_traversal with the common grid: lane-records (one record's lookups of one lane) read from
     * the group rows (two 16-byte loads), from the LDS near field, from the bands' own tables (four
     * 8-byte loads) */
    int64_t mo_row_lane_records, mo_lds_lane_records, mo_table_lane_records;
    double ms_tex;        /* texture lookups at the camera hits (albedo / bump imagemaps; shade_tex) */
    int64_t n_tex;
    double ms_replay;     /* the reference sampler's values of each batch's window (replay_window) */
    int64_t n_replay;
    /* count_traversal with the common grid, per band group: lane-records by path (group rows, LDS,
     * own tables), and the L2 footprint of the row / own-table fetches -- distinct 32-byte sectors and
     * 128-byte lines the active lanes' loads touch, summed over wave fetches -- and the wave fetches */
    int64_t group_path_records[8][3];
    int64_t group_path_sectors[8][2], group_path_lines[8][2], group_path_fetches[8][2];
} mpss_render_stats;
int mpss_get_render_stats(mpss_ctx *ctx, mpss_render_stats *out);
/* Switch kernel_timing / count_traversal (0, 1 or 2, as mpss_config) after creation
 * (instrumented passes). */
int mpss_set_instrumentation(mpss_ctx *ctx, int kernel_timing, int count_traversal);
int mpss_reset_render_stats(mpss_ctx *ctx);

/* ---- Monte-Carlo layered profile (renderer "mcprofile", src/renderers/mcprofile.cpp) ---- */
typedef struct { float mua, musp, ior, thickness; } mpss_layer; /* core/layer.h:35-46, "layer layers" order */
/* MonteCarloProfileRenderer::Render (mcprofile.cpp:443-533) on the ctx's GPU: nphotons random walks
 * (FP64), rings of width extent/nsegments with extent = mfp_range * mean_l 1/(mua+musp). Outputs
 * are normalised per photon and ring area; totals per photon. seed selects the photon streams.
 * events (nullable) = free-flight events simulated. Synchronous on stream. */
int mpss_mc_profile(mpss_ctx *ctx, const mpss_layer *layers, int nlayers, float mfp_range, int nsegments,
                    uint64_t nphotons, uint64_t seed, double *reflectance, double *transmittance, double *total_r,
                    double *total_t, uint64_t *events, void *stream);

/* MultipoleReferenceTask (mcprofile.cpp:356-425): the multipole model of the same layers (MPC at
 * desiredLength 1024, step extent * 1.01 / 1024, lerp on thin slabs or not) sampled at the ring
 * centres (i + .5) * extent / nsegments, extent = mfp_range * mean_l 1/(mua + musp); host code,
 * no device needed. Outputs per ring (double) and the MPC totals. */
int mpss_mc_reference(const mpss_layer *layers, int nlayers, float mfp_range, int nsegments, int lerp_on_thin_slab,
                      double *reflectance, double *transmittance, double *total_r, double *total_t);

/* ---- host-side utilities (no HIP device needed): the product's own parse-time builders,
 * exposed so their results can be checked on a CPU-only machine. ---- */
/* SampledSpectrum::FromRGB (spectrum.cpp:103-187); pbrt's "color"/"rgb" parameters use
 * illuminant = 0 (ParamSet::AddRGBSpectrum, paramset.cpp:97-105). */
int mpss_host_from_rgb(const float *rgb, int illuminant, float *out);
/* TessellateSurfacePoints of one triangle mesh (trianglemesh.cpp:187-351); flip =
 * ReverseOrientation ^ ObjectToWorld.SwapsHandedness(). Sizes first with records NULL. */
int mpss_host_tessellate(uint32_t nverts, const float *P, const float *N, const float *S, const float *uv,
                         uint32_t ntris, const int32_t *indices, const float *obj_to_world, const float *world_to_obj,
                         int flip, uint32_t material_id, float min_dist, int incenter, void *records, uint32_t *n);
/* The same with a "bumpmap" float imagemap applied to every point's normal (BumpMapping::Bump,
 * trianglemesh.cpp:240-245); bump NULL = mpss_host_tessellate. */
int mpss_host_tessellate_bumped(uint32_t nverts, const float *P, const float *N, const float *S, const float *uv,
                                uint32_t ntris, const int32_t *indices, const float *obj_to_world,
                                const float *world_to_obj, int flip, uint32_t material_id, float min_dist,
                                int incenter, const mpss_imagemap *bump, void *records, uint32_t *n);
/* ImageTexture::Evaluate of an imagemap at n points: uvd[6 i ..] = u, v, dudx, dvdx, dudy, dvdy;
 * out[3 i ..] = the MIPMap value (RGB; a float texture fills out[3 i] and zeroes the rest). */
int mpss_host_imagemap_lookup(const mpss_imagemap *t, uint32_t n, const float *uvd, float *out);
/* LayeredSkin -> per-layer 30-band mua/musp [2][30], thickness[2], eta[2] (layeredskin.cpp:47-89). */
int mpss_host_skin_layers(const mpss_layeredskin *m, float *mua, float *musp, float *thickness, float *eta);
/* Multipole profile from layer params; rd_table: [30][*length] (query *length with rd_table NULL). */
int mpss_host_build_profile(const float *mua, const float *musp, const float *thickness, const float *eta,
                            int desired_length, int lerp_on_thin_slab, float *rd_table, uint32_t *length,
                            float *rcp, float *total_reflectance);
/* DiffusionReflectance::operator() at n squared distances (rd: n x 30) and, if total is not NULL,
 * TotalReflectance() (diffusionutil.h:69-77, a 1024-step sum in d^2 over (4 mfp)^2). */
int mpss_host_dipole_rd(const float *sigma_a, const float *sigmap_s, float eta, uint32_t n, const float *d2,
                        float *rd, float *total);
/* rho_hd table (n entries, sqrt_samples^2 samples each) and rho_hh. */
int mpss_host_rho_table(float roughness, float eta, int double_ref_sslf, int n, int sqrt_samples, float *hd,
                        float *hh);
/* The common grid the sharded gather builds for a profile (mpss_config.mo_common_grid), on the host:
 * table [30][L], rcp [30]; snake as mpss_config.mo_band_dealing (0, 1), or 2: an rgbprofile table
 * (rows 0..2 = R, G, B, read in slots 0..2 of every group); near_field as mpss_config.mo_near_field
 * (5088 or 10236: the LDS split the grid is built for). Outputs (each nullable): rows
 * [n_rows][8] (the groups' pair rows: group g's row for row coordinate v = u below ua[g], ua + (u - ua)
 * hinv above it, is row0[g] + floor(v) - ubase[g], holding R_j(u_k), R_j(u_k+1) for slots j = 0..3, u_k
 * the row's position; a NaN first value flags a cell whose lanes read the exact tables);
 * *n_rows (call with rows NULL to size it); bands [8][4] (band of each group slot, -1 empty); rg [8]
 * (each group's grid: u = d2 * rg); u0lim / u1lim / u1start [8] (lanes with u < u0lim read the exact
 * LDS near field, u0lim <= u < u1lim the rows, any other u the bands' own tables; the rows' cells below
 * u1start are flagged); row0 / ubase [8]; rel_err / l1_err [30] (the measured resampling error over the
 * knots each band reads from the rows); ua / hinv [8]; *ok = 1 when some group has rows. */
int mpss_host_common_grid(const float *table, uint32_t L, const float *rcp, int snake, int near_field, float *rows,
                          uint32_t *n_rows, int32_t *bands, float *rg, float *u0lim, float *u1lim, float *u1start,
                          uint32_t *row0, uint32_t *ubase, float *rel_err, float *l1_err, float *ua, float *hinv,
                          int *ok);
/* Octree build + pre-order export (sizes first with NULL outputs). */
int mpss_host_octree_export(uint32_t n, const float *p, const float *nrm, const float *E, const float *area,
                            uint32_t *n_nodes, float *node_p, float *node_area, float *node_et, int32_t *depth,
                            int32_t *skip, int32_t *leaf_first, int32_t *leaf_count, int32_t *point_order);

#ifdef __cplusplus
}
#endif
#endif
