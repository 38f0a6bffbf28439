"""Multi-rank tile sharding + film gather (the bench's N>1 data path) on CPU with gloo:
tiles dealt over ranks and frames, one gather to rank 0, reassembly into full films. A
deterministic per-pixel "renderer" stands in for mpss_render_tile (which needs a GPU); the
assertions are that every pixel of every frame arrives exactly once, from the rank that owned
its tile, and that the cost dealer (deal_balanced) spreads the skin evenly on the real C2/C3
geometry (tile costs estimated here by projecting the head mesh into the image: the GPU's
mpss_tile_costs counts camera-ray hits instead)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def fake_pixels(f, x0, x1, y0, y1):
    ys, xs = np.mgrid[y0:y1, x0:x1]
    v = np.stack([xs + 1000 * ys, ys, np.full_like(xs, f), np.full_like(xs, 7)], -1).astype(np.float32)
    return v


def _worker(rank, world, port, W, H, T, q, dealer="round_robin"):
    sys.path.insert(0, os.path.join(ROOT, "pbrt-v2-skin_amd"))
    from mpss import tiles as tl
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    frames = world
    tiles = tl.tile_grid(W, H, T)
    items_all = [(f, t) for f in range(frames) for t in range(len(tiles))]
    if dealer == "balanced":  # every rank derives the deal from the same cost estimates on its own
        cx, cy = W / 2.0, H / 2.0
        cost1 = [max(0.0, 1.0 - (((x0 + x1) / 2 - cx) ** 2 + ((y0 + y1) / 2 - cy) ** 2) / (0.3 * W * H))
                 for x0, x1, y0, y1 in tiles]
        idx = tl.deal_balanced([cost1[t] for _, t in items_all], world)
        check = torch.tensor([hash(tuple(map(tuple, idx))) % (1 << 31)], dtype=torch.int64)
        allc = [torch.zeros_like(check) for _ in range(world)]
        dist.all_gather(allc, check)
        assert all(int(c) == int(check) for c in allc), "ranks derived different deals"
        by_rank = [[items_all[i] for i in d] for d in idx]
    else:
        by_rank = [[items_all[i] for i in tl.rank_items(len(items_all), r, world)] for r in range(world)]
    slots = max(len(x) for x in by_rank)
    out = torch.zeros((slots, T * T * 4), dtype=torch.float32)
    for i, (f, t) in enumerate(by_rank[rank]):
        x0, x1, y0, y1 = tiles[t]
        px = fake_pixels(f, x0, x1, y0, y1) + rank * 0  # owner-independent content
        out[i, : px.size] = torch.from_numpy(px.reshape(-1))
    gath = [torch.zeros_like(out) for _ in range(world)] if rank == 0 else None
    dist.gather(out, gath, dst=0)
    if rank == 0:
        img = np.zeros((frames, H, W, 4), np.float32)
        tl.assemble(img, [g.numpy() for g in gath], by_rank, tiles, T)
        ok = all(np.array_equal(img[f], fake_pixels(f, 0, W, 0, H)) for f in range(frames))
        q.put(bool(ok))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("W,H,T,dealer", [(100, 70, 32, "round_robin"), (64, 64, 64, "round_robin"),
                                          (100, 70, 16, "balanced"), (128, 96, 32, "balanced")])
def test_gloo_world2_tiles_gather(W, H, T, dealer):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, W, H, T, q, dealer)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True


class _FakeCtx:
    """Stands in for mpss.Context in bench.py's own multi-GPU code: tile_costs from a radial blob,
    render_tiles writing fake_pixels into CPU tensors."""

    def __init__(self, W, H):
        self.W, self.H = W, H

    def tile_costs(self, rects):
        cx, cy = self.W / 2.0, self.H / 2.0
        sss = [int(100 * max(0.0, 1.0 - (((x0 + x1) / 2 - cx) ** 2 + ((y0 + y1) / 2 - cy) ** 2) /
                                 (0.2 * self.W * self.H))) for x0, x1, y0, y1 in rects]
        return np.array(sss, np.int64), np.array([(x1 - x0) * (y1 - y0) for x0, x1, y0, y1 in rects], np.int64)

    def render_tiles(self, spp, seed, rects, ptrs, stream=None):
        for (x0, x1, y0, y1), ptr in zip(rects, ptrs):
            px = fake_pixels(seed, x0, x1, y0, y1).reshape(-1)
            dst = np.ctypeslib.as_array((__import__("ctypes").c_float * px.size).from_address(ptr))
            dst[:] = px

    def reset_render_stats(self):
        pass


def _bench_worker(rank, world, port, W, H, T, frames, q):
    """bench.py's deal + timed_steps (render, one dist.gather per step, max-over-ranks time) and
    tiles.assemble, over gloo with the stand-in renderer."""
    import argparse
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "pbrt-v2-skin_amd"))
    import bench
    from mpss import tiles as tl
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = _FakeCtx(W, H)
    sc = argparse.Namespace(xres=W, yres=H, spp=4)
    tiles, items_by_rank, bal, skin = bench.deal(ctx, sc, T, frames, world)
    dt, gath, out = bench.timed_steps(argparse.Namespace(seed=3), ctx, sc, tiles, items_by_rank, frames, T, rank,
                                      world, 2, 1, device="cpu")
    if rank == 0:
        img = np.zeros((frames, H, W, 4), np.float32)
        tl.assemble(img, [g.numpy() for g in gath], items_by_rank, tiles, T)
        ok = all(np.array_equal(img[f], fake_pixels(3 + f, 0, W, 0, H)) for f in range(frames))
        q.put((bool(ok), dt > 0, skin))
    dist.destroy_process_group()


@pytest.mark.parametrize("W,H,T,frames", [(100, 70, 32, 1), (128, 96, 32, 2)])
def test_gloo_world2_bench_timed_steps(W, H, T, frames):
    """The code bench.py runs at N > 1 (deal by tile cost, timed steps with the film gather, the
    MAX-over-ranks time, reassembly), at world size 2 over gloo."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, 2, port, W, H, T, frames, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs)
    ok, timed, skin = q.get(timeout=5)
    assert ok and timed and skin > 0


def test_rank_items_partition():
    sys.path.insert(0, os.path.join(ROOT, "pbrt-v2-skin_amd"))
    from mpss import tiles as tl
    for n in (1, 7, 64, 129):
        for world in (1, 2, 3, 8):
            got = sorted(i for r in range(world) for i in tl.rank_items(n, r, world))
            assert got == list(range(n))
            assert max(len(tl.rank_items(n, r, world)) for r in range(world)) == tl.slots_per_rank(n, world)


def _projected_head_costs(res, T):
    """Per-tile count of head-mesh vertices projected through skin.pbrt's camera at res x res:
    a CPU stand-in for mpss_tile_costs (which traces camera rays on the GPU)."""
    sys.path.insert(0, os.path.join(ROOT, "pbrt-v2-skin_amd"))
    from mpss import pbrtscene
    from mpss import tiles as tl
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin.pbrt"), xres=res, yres=res)
    r2c, c2w = sc.raster_to_camera()
    w2c = np.linalg.inv(c2w.astype(np.float64))
    c2r = np.linalg.inv(r2c.astype(np.float64))
    P = np.concatenate([me["P"] for me in sc.meshes]).astype(np.float64)
    cam = P @ w2c[:3, :3].T + w2c[:3, 3]
    # PerspectiveCamera: raster = CameraToRaster(camera point projected onto z = 1 plane)
    proj = np.concatenate([cam[:, :2] / cam[:, 2:3], np.ones((len(cam), 1))], 1)
    ras = proj @ c2r[:3, :3].T + c2r[:3, 3]
    tiles = tl.tile_grid(res, res, T)
    nx = (res + T - 1) // T
    cost = np.zeros(len(tiles))
    ok = (ras[:, 0] >= 0) & (ras[:, 0] < res) & (ras[:, 1] >= 0) & (ras[:, 1] < res)
    tx, ty = (ras[ok, 0] // T).astype(int), (ras[ok, 1] // T).astype(int)
    np.add.at(cost, ty * nx + tx, 1.0)
    return tiles, cost


@pytest.mark.parametrize("res,T,world", [(1024, 128, 2), (1024, 64, 8), (2048, 64, 8), (2048, 128, 8), (2048, 64, 4)])
def test_balanced_deal_spreads_the_face(res, T, world):
    sys.path.insert(0, os.path.join(ROOT, "pbrt-v2-skin_amd"))
    from mpss import tiles as tl
    tiles, cost = _projected_head_costs(res, T)
    head = cost > 0
    assert 0 < head.sum() < len(tiles)
    deal = tl.deal_balanced(cost, world)
    assert sorted(i for d in deal for i in d) == list(range(len(tiles)))
    per_rank_head = [int(head[d].sum()) for d in deal]
    assert max(per_rank_head) - min(per_rank_head) <= 1, per_rank_head
    assert tl.balance(cost, deal) <= 1.0 + cost.max() / max(cost.sum() / world, 1e-9) + 1e-9
    if head.sum() >= 8 * world:  # enough skin tiles per rank for the granularity not to dominate
        assert tl.balance(cost, deal) <= 1.10, tl.balance(cost, deal)
    # round-robin over a row-major grid whose width is a multiple of the rank count leaves whole
    # tile columns (and the face) to a few ranks
    rr = [tl.rank_items(len(tiles), r, world) for r in range(world)]
    if (res // T) % world == 0 and world >= 4:
        assert tl.balance(cost, rr) > 1.3 > tl.balance(cost, deal)


def test_deal_diagonal_partition():
    sys.path.insert(0, os.path.join(ROOT, "pbrt-v2-skin_amd"))
    from mpss import tiles as tl
    for nx, ny, world in ((16, 16, 8), (8, 8, 3), (5, 7, 4)):
        d = tl.deal_diagonal(nx, ny, world)
        assert sorted(i for x in d for i in x) == list(range(nx * ny))
        # a 4x4 block of tiles lands on every rank (world <= 8)
        blk = [ty * nx + tx for ty in range(min(4, ny)) for tx in range(min(4, nx))]
        owners = {r for r, x in enumerate(d) for i in x if i in blk}
        assert len(owners) == min(world, len(blk))


def test_bench_defaults_keep_the_metric_config():
    """BASELINE.json's metric is quoted on skin.pbrt 1024^2 at 1/2/4/8 GPUs: every N defaults to C2
    (weak scaling at N > 1, 128^2 tiles), so the driver's per-N values compare the same workload;
    C3's one-frame strong scaling runs as the secondary figure or with --config c3 (64^2 tiles)."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    for n in (1, 2, 8):
        a = bench.parse(["--gpus", str(n)])
        assert (a.config, a.tile) == ("c2", 128)
        assert bench.CONFIGS[a.config][3] == "weak"
    a = bench.parse(["--gpus", "8", "--config", "c3"])
    assert (a.config, a.tile) == ("c3", 64)
