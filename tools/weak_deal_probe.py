"""One GPU's share of a C2 weak-scaling step at N = 8, two ways (tools/gpu.sh has no step for it):
the tiles rank 0 got when the 8 frames' tiles were dealt by cost (tiles of up to 8 frames: one
mpss_render_tiles call per frame), and one whole frame (bench.py's deal since round 3). Prints
ms per step for both; same number of pixels and samples.

    python tools/weak_deal_probe.py [--world 8] [--steps 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "pbrt-v2-skin_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from mpss import tiles as tl
    ba = bench.parse(["--config", "c2"])
    sc, ctx, *_ = bench.build_scene(ba, "c2", 0)
    T = ba.tile
    tiles = tl.tile_grid(sc.xres, sc.yres, T)
    sss, surf = ctx.tile_costs(tiles)
    px = np.array([(x1 - x0) * (y1 - y0) for x0, x1, y0, y1 in tiles])
    cost1 = tl.tile_cost_model(sss, surf, px)
    items_all = [(f, t) for f in range(a.world) for t in range(len(tiles))]
    by_rank = tl.deal_balanced([cost1[t] for _, t in items_all], a.world)
    variants = {"cost_dealt_over_frames": [items_all[i] for i in by_rank[0]],
                "whole_frame": [(0, t) for t in range(len(tiles))]}
    seeds = [ba.seed + f for f in range(a.world)]
    res = {}
    for name, items in variants.items():
        out = torch.zeros((len(items), T * T * 4), dtype=torch.float32, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream
        tl.render_items(ctx, items, tiles, sc.spp, seeds, out, T, stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            tl.render_items(ctx, items, tiles, sc.spp, seeds, out, T, stream)
        torch.cuda.synchronize()
        res[name] = {"ms_per_step": round((time.perf_counter() - t0) / a.steps * 1e3, 3), "tiles": len(items),
                     "frames_touched": len({f for f, _ in items})}
    print(json.dumps({"world": a.world, "config": "c2", "rank": 0, **res}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
