// mo_kernel.h -- device-resident octree / profile and the Mo() gather launcher.
#pragma once
#include "common.h"
#include "octree.h"

namespace mpss {

struct DeviceOctree {
    DevBuf<NodeHdr> nodes;
    DevBuf<float> node_et;
    DevBuf<float4> pt_hdr;
    DevBuf<float> pt_e;
    int n_nodes = 0, n_points = 0, max_depth = 0;
    void upload(const FlatOctree &t);
};

struct DeviceProfile {
    DevBuf<float> table;  // [NB][L] channel-major
    DevBuf<float> rcp;    // [NB]
    float rcp_min = 0.f;  // min over bands (exact subtree pruning, mo_kernel.hip)
    int L = 0;
    void upload(const float *table, int L, const float *rcp);
};

// queries/out/counters are device pointers. out[q * out_stride + c], c < 30.
// counters (nullable, q*4 int32): per query {reference-traversal nodes entered, points evaluated,
// pruned-kernel nodes entered, points evaluated}. The packet kernel (exact=false)
// reports only the last two (the first two are 0); exact=true follows the reference summation order.
void launch_mo_gather(const DeviceOctree &t, const DeviceProfile &p, float max_error, int nq, const float *queries,
                      float *out, int out_stride, int32_t *counters, hipStream_t stream, bool exact);

}  // namespace mpss
