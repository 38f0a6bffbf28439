// scene.h -- the scene slice the multipole path needs (host side): triangle meshes in world
// space, sphere area lights and constant infinite lights, perspective camera, the BVH over triangles, and the tessellated
// SurfacePoint set (reference: shapes/trianglemesh.{cpp,inl}, shapes/sphere.cpp,
// lights/diffuse.cpp, cameras/perspective.cpp, accelerators/bvh.cpp,
// renderers/surfacepoints.cpp:301-369).
#pragma once
#include <vector>

#include "common.h"
#include "pbrt_math.h"

namespace mpss {

struct Mesh {
    // world-space positions (TriangleMesh ctor applies ObjectToWorld, trianglemesh.cpp:43-73)
    std::vector<float> P;        // nv*3
    std::vector<float> N, S, uv; // object-space normals / tangents (nv*3), uv (nv*2); may be empty
    std::vector<int32_t> idx;    // nt*3
    float o2w[16], w2o[16];      // ObjectToWorld and its inverse (row-major)
    uint32_t material = 0;
    bool reverse_orientation = false, swaps_handedness = false;
};

// scene->lights in declaration order. kind 0: AreaLightSource "area" on Shape "sphere"
// (translation-only placement, lights/diffuse.cpp); kind 1: LightSource "infinite" with a
// constant radiance map (lights/infinite.cpp:66-106, the 1x1 map of a light without "mapname").
struct SceneLight {
    int kind = 0;
    float center[3], radius;
    float Lemit[NB];      // kind 0: DiffuseAreaLight::Lemit
    float l2w[9], w2l[9]; // kind 1: LightToWorld / WorldToLight (upper 3x3, row-major)
    int map_w = 0, map_h = 0;
    std::vector<float> map;  // kind 1: texels * (L * scale).ToRGBSpectrum(), or 1x1 without a map
    int nsamples;
};

struct Camera {
    float raster_to_camera[16], camera_to_world[16];
    int xres = 0, yres = 0;
};

// Linear BVH node (accelerators/bvh.cpp:113-123 layout): 32 B.
struct alignas(16) BvhNode {
    float bmin[3];
    int32_t offset;  // leaf: first primitive; interior: second child index
    float bmax[3];
    uint16_t nprims;  // 0 for interior
    uint16_t axis;
};
static_assert(sizeof(BvhNode) == 32, "BvhNode is 32 B");

// Flattened triangle for the GPU: p1, e1 = p2-p1, e2 = p3-p1 (trianglemesh.inl:57-60) and its
// global triangle id; 48 B.
struct alignas(16) TriRec {
    float p1[3];
    int32_t tri;
    float e1[3];
    int32_t mesh;
    float e2[3];
    int32_t pad;
};

struct SceneData {
    std::vector<Mesh> meshes;
    std::vector<SceneLight> lights;
    Camera camera;
    // flattened (all meshes)
    std::vector<int32_t> tri_mesh, tri_local;  // global tri -> mesh, local index
    std::vector<BvhNode> bvh;
    std::vector<TriRec> tris;  // in BVH leaf order
};

void build_bvh(SceneData &s);

// Candidate triangles per pixel for the reference sampler's camera rays (replay_gen.hip: whether a
// camera ray hits anything decides how many Li draws its sample consumes). For each pixel of the
// (xres + 1) x (yres + 1) sample extent (a sample's raster point lies in [x, x + 1) x [y, y + 1)):
// the triangles (indices into SceneData::tris) whose raster projection, widened by kCamBinMargin
// pixels, meets it (its box, then its edges) -- a ray through a point of the pixel can hit no other
// triangle in front of the camera -- largest projected area first. Triangles with a vertex near or behind the camera plane, or whose box spans
// more than kCamBinMaxArea pixels, go to `all` (tested for every pixel); triangles entirely behind
// the camera or off the extent to neither list.
struct CameraBins {
    int w = 0, h = 0;            // xres + 1, yres + 1
    std::vector<uint32_t> off;   // [w * h + 1]: pixel p's triangles are tri[off[p] .. off[p + 1])
    std::vector<int32_t> tri;
    std::vector<int32_t> all;
};
constexpr double kCamBinMargin = 1.0 / 64;
constexpr int kCamBinMaxArea = 4096;
void build_camera_bins(const SceneData &s, CameraBins &b);

// SurfacePoint (renderers/surfacepoints.h:45-55): p, n, u, v, materialId, area, rayEpsilon.
struct SurfacePoint {
    float p[3], n[3], u, v;
    uint32_t material;
    float area, ray_eps;
};
static_assert(sizeof(SurfacePoint) == 44, "SurfacePoint matches the reference's 44-B pointsfile record");

// TriangleMesh::TessellateSurfacePoints over every mesh in order (trianglemesh.cpp:187-257,
// tessellator 265-318, matching 321-351; driver surfacepoints.cpp:301-333).
// bump (nullable): per material id, its "bumpmap" ImageTexture (host view) or null; a bumped
// material's points carry the bump-mapped normal (BumpMapping::Bump, trianglemesh.cpp:240-245).
struct TexView;
void tessellate_surface_points(const SceneData &s, float min_dist, bool incenter, std::vector<SurfacePoint> &out,
                               int nthreads = 0, const TexView *const *bump = nullptr);

}  // namespace mpss
