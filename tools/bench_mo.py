#!/usr/bin/env python3
"""Mo() gather microbenchmark (product path only; no oracle).

Workload (synthetic stand-in until the tessellated head is used):
an ellipsoid point cloud at minsampledistance-like density, S007 LayeredSkin profile,
Q surface queries in spatially sorted order. Reports kernel time (HIP events on the
launch stream), queries/s and algorithmic bytes/s = 136 B x (nodes entered + points
evaluated) / t.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pbrt-v2-skin_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=600000)
    ap.add_argument("--queries", type=int, default=4 << 20)
    ap.add_argument("--max-error", type=float, default=0.1)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--desired-length", type=int, default=512)
    ap.add_argument("--exact", action="store_true", help="reference-order kernel instead of the packet kernel")
    args = ap.parse_args()
    import torch
    import mpss
    import synth

    radii = (0.25, 0.3, 0.35)
    t0 = time.time()
    ctx = mpss.Context(max_error=args.max_error, exact_mo=int(args.exact))
    skin = mpss.default_skin(roughness=0.3, nmperunit=40e6, f_mel=0.5, f_eu=0.5, f_blood=0.5, f_ohg=0.5, Kt=[0.0] * 30,
                             desired_length=args.desired_length)
    mid = ctx.add_layeredskin(skin)
    t1 = time.time()
    cloud = synth.ellipsoid_cloud(args.points, radii=radii, seed=7, black_frac=0.0)
    ctx.set_irradiance_points(*cloud)
    t2 = time.time()
    q = synth.surface_queries(args.queries, radii=radii, seed=13)
    qd = torch.from_numpy(q).cuda()
    out = torch.empty((len(q), 30), dtype=torch.float32, device="cuda")
    cnt = torch.zeros((len(q), 4), dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    ctx.mo_batch(mid, len(q), qd.data_ptr(), out.data_ptr(), cnt.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    visits = cnt.sum(0).cpu().numpy().astype(np.int64)
    times = []
    for _ in range(args.iters):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(s)
        ctx.mo_batch(mid, len(q), qd.data_ptr(), out.data_ptr(), None, s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1) / 1e3)
    t = float(np.median(times))
    algo = 136.0 * float(visits[2] + visits[3])      # pruned kernel traversal
    algo_ref = 136.0 * float(visits[0] + visits[1])  # reference recursion (same result)
    res = dict(mode="exact" if args.exact else "packet", points=args.points, queries=args.queries, info=ctx.octree_info(),
               ref_nodes_per_query=float(visits[0]) / len(q), ref_points_per_query=float(visits[1]) / len(q),
               nodes_per_query=float(visits[2]) / len(q), points_per_query=float(visits[3]) / len(q),
               ref_equiv_GBps=algo_ref / t / 1e9,
               kernel_s=t, all_s=times, mqueries_per_s=len(q) / t / 1e6, algo_GBps=algo / t / 1e9,
               frac_of_8TBps=algo / t / 8e12, profile_build_s=t1 - t0, octree_build_s=t2 - t1,
               mo_mean=float(out.mean().item()))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
