"""Multi-rank tile sharding + film gather (the bench's N>1 data path) on CPU with gloo,
world size 2: tiles dealt round-robin over ranks and frames, one gather to rank 0,
reassembly into full films. A deterministic per-pixel "renderer" stands in for
mpss_render_tile (which needs a GPU); the assertion is that every pixel of every frame
arrives exactly once, from the rank that owned its tile."""
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


def _worker(rank, world, port, W, H, T, q):
    sys.path.insert(0, os.path.join(ROOT, "pbrt-v2-skin_amd"))
    from mpss import tiles as tl
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    frames = world
    tiles = tl.tile_grid(W, H, T)
    items_all = [(f, t) for f in range(frames) for t in range(len(tiles))]
    by_rank = [[items_all[i] for i in tl.rank_items(len(items_all), r, world)] for r in range(world)]
    slots = tl.slots_per_rank(len(items_all), world)
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


@pytest.mark.parametrize("W,H,T", [(100, 70, 32), (64, 64, 64)])
def test_gloo_world2_tiles_gather(W, H, T):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, W, H, T, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True


def test_rank_items_partition():
    sys.path.insert(0, os.path.join(ROOT, "pbrt-v2-skin_amd"))
    from mpss import tiles as tl
    for n in (1, 7, 64, 129):
        for world in (1, 2, 3, 8):
            got = sorted(i for r in range(world) for i in tl.rank_items(n, r, world))
            assert got == list(range(n))
            assert max(len(tl.rank_items(n, r, world)) for r in range(world)) == tl.slots_per_rank(n, world)
