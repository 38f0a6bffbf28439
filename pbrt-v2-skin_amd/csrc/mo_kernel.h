// mo_kernel.h -- device-resident octree / profile and the Mo() gather launcher.
#pragma once
#include "common.h"
#include "mo_band.h"
#include "octree.h"

namespace mpss {

struct DeviceOctree {
    DevBuf<NodeHdr> nodes;
    DevBuf<float> node_et;
    DevBuf<float4> pt_hdr;
    DevBuf<float> pt_e;
    int n_nodes = 0, n_points = 0, max_depth = 0;
    // group-major copies for the spectrally sharded gather (mo_band.h), built on demand
    DevBuf<float4> band_et, band_e;
    BandGroups band_groups{};
    bool band_valid = false;
    void upload(const FlatOctree &t);
    void ensure_band_layout(const BandGroups &g, hipStream_t stream);
};

struct DeviceProfile {
    DevBuf<float> table;  // [NB][L] channel-major
    DevBuf<float> rcp;    // [NB]
    float rcp_min = 0.f;  // min over bands (exact subtree pruning, mo_kernel.hip)
    int L = 0;
    float host_rcp[NB];
    BandGroups groups{};   // band -> XCD group assignment for this profile
    void upload(const float *table, int L, const float *rcp);
};

// queries/out/counters are device pointers. out[q * out_stride + c], c < 30.
// counters (nullable, q*4 int32): per query {reference-traversal nodes entered, points evaluated,
// pruned-kernel nodes entered, points evaluated}. The packet kernel (exact=false)
// reports only the last two (the first two are 0); exact=true follows the reference summation order.
// mode: 0 spectrally sharded (default), 1 exact reference order, 2 packet.
void launch_mo_gather(const DeviceOctree &t, const DeviceProfile &p, float max_error, int nq, const float *queries,
                      float *out, int out_stride, int32_t *counters, hipStream_t stream, int mode);

// Spectrally sharded gather for the render path: queries4[i] = {p, *}, i < *count_dev (<= nq_max);
// out4[i * 8 + g] = the 4 bands of group g (BandGroups::pos gives a band's float offset).
// counts (nullable): [2 * kGroups] nodes / points visited per group (atomics).
void launch_mo_band(DeviceOctree &t, const DeviceProfile &p, float max_error, int nq_max, const float4 *queries4,
                    const int *count_dev, float4 *out4, unsigned long long *counts, hipStream_t stream);

}  // namespace mpss
