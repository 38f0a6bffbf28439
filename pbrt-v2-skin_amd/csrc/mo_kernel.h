// mo_kernel.h -- device-resident octree / profile and the Mo() gather launchers.
#pragma once
#include <memory>
#include <vector>

#include "common.h"
#include "mo_band.h"
#include "octree.h"

namespace mpss {

// The group-major copy of the octree's E/Et rows for one band grouping (mo_band.h): et[g][node],
// e[g][point] = the 4 bands of group g as a float4.
struct BandLayout {
    BandGroups groups{};
    DevBuf<float4> et, e;
    DevBuf<float4> ew;  // e scaled by each point's area (the common-grid gather's products, mo_band.h)
};

struct DeviceOctree {
    DevBuf<NodeHdr> nodes;
    DevBuf<float> node_et;
    DevBuf<float4> pt_hdr;
    DevBuf<float> pt_e;
    DevBuf<int> pt_index;  // original point index of every point slot
    int n_nodes = 0, n_points = 0, max_depth = 0;
    float bmin[3] = {0.f, 0.f, 0.f}, bmax[3] = {0.f, 0.f, 0.f};  // root bounds (query sort keys)
    // one group-major layout per distinct band grouping in use; built eagerly and synchronously
    // (Context::set_irradiance_points / add material) so launches only read them
    std::vector<std::unique_ptr<BandLayout>> layouts;
    // per node: for a leaf, the square of a radius around its centroid that holds every point of the
    // leaf as seen from any query that opens it under max_error (DiffusionOctree Mo(): d^2 <= sumArea /
    // maxError, or the query inside the leaf's box): max(sqrt(sumArea / maxError), diag) + diag,
    // squared, rounded up; +inf for interior nodes and leaves without a finite centroid. Lets the
    // sharded gather prove a leaf's point lookups lie in its LDS near field. Valid for
    // leaf_r2_error == the gather's max_error. The gather reads it as a 16-bit code in the node's
    // header (NodeHdr::pad's high half, rounded up; ensure_leaf_r2 writes both).
    DevBuf<float> leaf_r2;
    float leaf_r2_error = -1.f;
    void ensure_leaf_r2(float max_error);  // synchronous
    void upload(const FlatOctree &t);
    const BandLayout *find_layout(const BandGroups &g) const;
    // builds the layout if it is missing (synchronizes the device); the caller serializes calls
    const BandLayout &ensure_layout(const BandGroups &g);
};

// SubsurfaceOctreeNode::Insert + InitHierarchy on the device (octree_gpu.hip): the tree of the host
// build (octree.cpp) + DeviceOctree::upload, bit for bit. P, N: n x 3, E: n x NB, A: n device floats;
// bmin / bmax: the points' bounds (Union of the points in index order). Synchronous.
void build_octree_device(int n, const float *P, const float *N, const float *E, const float *A, const float bmin[3],
                         const float bmax[3], DeviceOctree &t);

struct DeviceProfile {
    DevBuf<float> table;  // [NB][L] channel-major + 2 trailing zeros
    DevBuf<float> rcp;    // [NB]
    float rcp_min = 0.f;  // min over bands (exact subtree pruning, mo_kernel.hip)
    int L = 0;
    float host_rcp[NB];
    BandGroups groups{};   // band -> XCD group assignment for this profile
    // The common grid of each band group (mo_band.h CommonGrid), built by upload() for each LDS layout
    // (the 10236-entry near field: cg; the 5088-entry one, the default: cg_half): ctab / ctab_half hold
    // the groups' pair rows (two float4 per row); on = 1 when some group has an accurate row range.
    DevBuf<float4> ctab, ctab_half;
    CommonGrid cg{}, cg_half{};  // for the 10236 and 5088 LDS layouts
    // per band and layout: max |R - T| / |T| over its knots read from the group rows, and the sum of
    // |R - T| over those knots / the sum of |T| over the table ([0]: 10236 layout, [1]: 5088)
    float cg_rel_err[2][NB] = {};
    float cg_l1_err[2][NB] = {};
    // snake: deal the bands to groups in snake rounds instead of runs of adjacent reach (mo_band.h)
    void upload(const float *table, int L, const float *rcp, bool snake = false);
    // (upload calls it with groups, set_rgb with rows 0..2 in every group; host table [NB][L])
    // lds_reserve: floats at the end of the LDS near field the grid's split leaves free
    // rgb: the slots are the rgbprofile's R, G, B (build_common_grid)
    void build_common(const float *table, const BandGroups &slots, int lds_reserve, bool rgb);
    // rgbprofile material: rows 0..2 of the table are its R, G, B profiles; the sharded gather looks
    // up those three for every group and converts them with FromRGB (rgb_refl: the device copy of
    // the rgbRefl2Spect tables, [7][NB]; set_rgb after upload)
    DevBuf<float> rgb_refl;
    void set_rgb(const float *table);
};

// The common grid's bound on the resampling error of a lookup: kCgRelTol of the band's own value
// there, or kCgAbsTol of the band's peak where that is larger (the far tails, whose values fall to
// 1e-11 of the peak and carry under 1 % of a band's mass on C2's profile: there the bound is
// absolute). DeviceProfile::build_common; a group row (cell) holding a knot off by more is flagged and
// its lanes read the exact tables. The floor is chosen on the full C2 frame against the oracle, same
// box (profiles/r06_grid_ab.txt, rows H steps apart with flagged cells): 1e-13: gather 43.4 ms,
// unfloored image error 3.3e-5; 1e-14: 43.9 ms, 1.5e-6; 1e-15: 45.1 ms, 1.1e-6 -- the worst values at
// 1e-16 of the frame's peak, far below the film's resolution (round 4, one stretch of rows per group,
// profiles/r04p_abstol.txt: none 60.4 ms, 1.1e-6; 1e-13 48.6 ms, 4.3e-6; 1e-10 47.1 ms, 9.0e-5).
constexpr double kCgRelTol = 2e-6;
#ifndef MPSS_CG_ABS_TOL  // (A/B builds of the floor only)
#define MPSS_CG_ABS_TOL 1e-14
#endif
constexpr double kCgAbsTol = MPSS_CG_ABS_TOL;

// The host half of DeviceProfile::build_common: the layout (cg, without tab), the pair rows h (two
// float4 per row, group by group from cg.row0) and the per-band errors; true (cg.on) when some group
// has rows. rgb: the slots are the rgbprofile's R, G, B, whose knots' errors are relative to the
// largest of the three at that distance (the scale of FromRGB's outputs) instead of their own value.
bool build_common_grid(const float *tab, int L, const float *rcp, const BandGroups &groups, CommonGrid &cg,
                       std::vector<float4> &h, float rel_err[NB], float l1_err[NB], int near_field = 10236,
                       int lds_reserve = 0, bool rgb = false);

// Choices of the sharded gather (mpss_config.mo_near_field / mo_work_stealing; count_noprune =
// mpss_config.count_traversal == 2, instrumented passes only).
struct GatherOpts {
    int near_field = 10236;
    bool steal = true;
    bool count_noprune = false;
    bool common_grid = true;  // mpss_config.mo_common_grid (the layout's grid: cg for 10236, cg_half for 5088)
};

// queries/out/counters are device pointers. out[q * out_stride + c], c < 30.
// counters (nullable, q*4 int32): per query {reference-traversal nodes entered, points evaluated,
// pruned-kernel nodes entered, points evaluated}. The packet kernel reports only
// the last two (the first two are 0); mode 1 follows the reference summation order.
// mode: 0 spectrally sharded (default; needs `layout` for p.groups), 1 exact reference order, 2 packet.
// work: kGroups ints of device scratch for mode 0 (the persistent grid's chunk counters); perm:
// >= nq rounded up to 1024 ints of device scratch for mode 0 (the sorted query permutation).
void launch_mo_gather(const DeviceOctree &t, const BandLayout *layout, const DeviceProfile &p, float max_error, int nq,
                      const float *queries, float *out, int out_stride, int32_t *counters, int *work, int *perm,
                      int mode, const GatherOpts &opts, hipStream_t stream);

// Mo with the closed-form single dipole (dipole.h) as Rd, in the reference summation order.
// dipole_dev: [4][NB] device floats zpos, zneg, sigma_tr, k. Nothing is pruned.
void launch_mo_dipole(const DeviceOctree &t, const float *dipole_dev, float max_error, int nq, const float *queries,
                      float *out, int out_stride, int32_t *counters, hipStream_t stream);

// Mo with an rgbprofile material (multipole.cpp:85-107): table3 [3][L] R, G, B profiles (device),
// rcp3 their rcpDsqSpacing (device and host copies), in the reference summation order. Queries
// either queries (q x 3) or the render path's queries4 / count_dev / hit_s + mat (see
// launch_mo_band); out[i * out_stride + c].
void launch_mo_rgb(const DeviceOctree &t, const float *table3, const float *rcp3_dev, const float rcp3[3], int L,
                   float max_error, int nq, const float *queries, const float4 *queries4, const int *count_dev,
                   const uint32_t *hit_s, int mat, float *out, int out_stride, int32_t *counters, hipStream_t stream);

// Traversal statistics of the sharded gather (count variant): per group g, counts[kStatStride*g + k]
// for k = 0 node visits, 1 point visits (summed over queries), 2 wave node iterations, 3 wave
// point iterations (summed over waves; 64 x these / the visits = 1 / lane efficiency), 4 table
// lookups inside the profile (lane x band), 5..7 those at entries < 4096, 8192, 16384; common grid
// only: 8 lane-records read from the group rows (two 16-byte loads each), 9 from the LDS near field,
// 10 from the bands' own tables (four 8-byte loads); 11..16 the L2 footprint of the row and own-table
// fetches (mo_band.h kHist 7..12: distinct 32-B sectors, 128-B lines, wave fetches).
constexpr int kStatStride = 4 + 13;

// Spectrally sharded gather for the render path: queries4[i] = {p, *}, i < *count_dev (<= nq_max);
// out4[i * 8 + g] = the 4 bands of group g (BandGroups::pos gives a band's float offset).
// hit_s / mat (hit_s nullable): only queries whose hit_s material field equals mat are evaluated
// (scenes with several BSSRDF materials run one launch per material). counts: see kStatStride.
// work: kGroups ints of device scratch (the chunk counters of the persistent grid); perm: >= nq_max
// rounded up to 1024 ints of device scratch.
void launch_mo_band(const DeviceOctree &t, const BandLayout &layout, const DeviceProfile &p, float max_error,
                    int nq_max, const float4 *queries4, const int *count_dev, float4 *out4,
                    const uint32_t *hit_s, int mat, unsigned long long *counts, int *work, int *perm,
                    const GatherOpts &opts, hipStream_t stream);

}  // namespace mpss
