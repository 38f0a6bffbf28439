"""Child process of test_rccl_gpu.py (started before it touches the GPU): bench.py's multi-GPU data
path -- torch.distributed over RCCL ("nccl"), bench.deal + bench.timed_steps (render the dealt tiles,
one dist.gather of the film tiles per step) and tiles.assemble -- at world size 1 on cuda:0, on a
256x256 16-spp skin.pbrt frame. Exit 0 iff the assembled film equals one mpss_render_tile call of
the whole frame bit for bit. Prints one JSON line with what ran."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "pbrt-v2-skin_amd"))


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    import bench
    from mpss import pbrtscene
    from mpss import tiles as tl

    port = int(sys.argv[1])
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    backend = dist.get_backend()
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin.pbrt"), xres=256, yres=256, spp=16)
    ctx = pbrtscene.build_context(sc)
    ctx.preprocess(seed=1)
    T = 64
    tiles, items_by_rank, _, skin_tiles = bench.deal(ctx, sc, T, 1, 1)
    a = argparse.Namespace(seed=5)
    dt, gath, out = bench.timed_steps(a, ctx, sc, tiles, items_by_rank, 1, T, 0, 1, 2, 1)
    assert gath is not None and len(gath) == 1  # the gather ran (world size 1 keeps the collective)
    img = np.zeros((1, sc.yres, sc.xres, 4), np.float32)
    tl.assemble(img, [g.cpu().numpy() for g in gath], items_by_rank, tiles, T)
    full = torch.zeros((sc.yres * sc.xres * 4,), dtype=torch.float32, device="cuda")
    ctx.render_tile(sc.spp, 5, 0, sc.xres, 0, sc.yres, full.data_ptr())
    torch.cuda.synchronize()
    ref = full.cpu().numpy().reshape(sc.yres, sc.xres, 4)
    t = torch.tensor([dt], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ok = bool(np.array_equal(img[0], ref) and (ref[..., 1] > 0).any())
    print(json.dumps({"backend": backend, "world": dist.get_world_size(), "tiles": len(tiles),
                      "skin_tiles": int(skin_tiles), "step_s": float(t.item()) / 2, "film_equal": ok}), flush=True)
    ctx.close()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
