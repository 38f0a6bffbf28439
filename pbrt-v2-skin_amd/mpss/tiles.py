"""Image-tile sharding of the pixel loop across ranks.

pbrt splits the film into RoundUpPow2(max(32*cores, W*H/256)) sampler tasks
(renderers/samplerrenderer.cpp:191-217; Sampler::ComputeSubWindow, core/sampler.cpp:55-78);
here the unit is a T x T pixel tile handed to one GPU, and each rank's film tiles reach rank 0
through one collective gather at the end of the frame.

Dealing. The skin sits in the middle of the frame and a tile's cost is dominated by its
subsurface (Mo() gather) hits, so round-robin over a row-major grid is not balanced: with a
grid 8, 16 or 32 tiles wide every rank owns whole tile columns. ``deal_balanced`` sorts the
tiles by an estimated cost (``mpss.Context.tile_costs``: one camera ray through every pixel
centre, hits counted per tile -- integer counts, identical on every rank, so every rank derives
the same deal without communicating) and deals them in rounds, one tile per rank per round,
the heaviest tile of a round to the least-loaded rank. Every prefix of that order -- in
particular "the tiles that contain skin" -- is split with per-rank counts differing by at most
one, and the costs balance as in longest-processing-time-first dealing.
``deal_diagonal`` is the geometry-free fallback: tile (tx, ty) goes to rank (tx + s * ty) mod N
with s coprime to N, so a compact blob is spread over all ranks instead of over column owners.
"""
import math

import numpy as np


def tile_grid(W, H, T):
    """Row-major list of (x0, x1, y0, y1) tiles covering a W x H film."""
    return [(x0, min(x0 + T, W), y0, min(y0 + T, H)) for y0 in range(0, H, T) for x0 in range(0, W, T)]


def rank_items(n_items, rank, world):
    """Work items of `rank` when n_items are dealt round-robin over `world` ranks."""
    return list(range(rank, n_items, world))


def slots_per_rank(n_items, world):
    return (n_items + world - 1) // world


def deal_balanced(costs, world):
    """Items dealt in rounds of `world`: items sorted by decreasing cost (ties: lower index
    first); in each round the round's heaviest item goes to the rank with the least cost so far,
    the next to the next-least, and so on (ties: lower rank). Every rank gets one item per round,
    so any prefix of the order -- e.g. "the tiles that contain skin" -- is split with per-rank
    counts differing by at most one, and costs stay balanced as in longest-processing-time-first
    dealing. Returns per rank its item indices in increasing order. Deterministic."""
    costs = np.asarray(costs, np.float64)
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    load = [0.0] * world
    out = [[] for _ in range(world)]
    for r0 in range(0, len(order), world):
        rnd = order[r0:r0 + world]
        ranks = sorted(range(world), key=lambda k: (load[k], k))
        for i, k in zip(rnd, ranks):
            out[k].append(i)
            load[k] += costs[i]
    return [sorted(x) for x in out]


def _coprime_shift(world):
    for s in (3, 5, 7, 11, 13, 2, 1):
        if s < max(world, 2) and math.gcd(s, world) == 1:
            return s
    return 1


def deal_diagonal(nx, ny, world):
    """Tile (tx, ty) of an nx x ny row-major grid -> rank (tx + s * ty) % world."""
    s = _coprime_shift(world)
    out = [[] for _ in range(world)]
    for ty in range(ny):
        for tx in range(nx):
            out[(tx + s * ty) % world].append(ty * nx + tx)
    return out


def tile_cost_model(sss_hits, surf_hits, pixels):
    """Relative cost of a tile from its probe counts (one camera ray per pixel centre): a
    subsurface hit runs the Mo() gather (~85 % of a C2 frame), a surface hit the direct
    lighting, every pixel its camera rays and film work."""
    return (np.asarray(sss_hits, np.float64) * 1.0 + np.asarray(surf_hits, np.float64) * 0.1
            + np.asarray(pixels, np.float64) * 0.004)


def balance(costs, deal):
    """max over ranks of the dealt cost / mean over ranks (1.0 = perfect)."""
    costs = np.asarray(costs, np.float64)
    per = np.array([costs[list(d)].sum() if len(d) else 0.0 for d in deal])
    return float(per.max() / max(per.mean(), 1e-30))


def render_items(ctx, items, tiles, spp, seeds, out, T, stream=None):
    """Render work items (frame, tile) into out[i] (a [n, T*T*4] float32 device tensor): one
    mpss_render_tiles call per frame, so the tiles of a frame share Mo() gather launches."""
    by_frame = {}
    for i, (f, t) in enumerate(items):
        by_frame.setdefault(f, []).append((i, t))
    for f, lst in by_frame.items():
        rects = [tiles[t] for _, t in lst]
        ctx.render_tiles(spp, seeds[f], rects, [out[i].data_ptr() for i, _ in lst], stream)


def assemble(frames_xyzw, gathered, items_by_rank, tiles, T):
    """Scatter gathered tile buffers (per rank: [slots, T*T*4]) into [F, H, W, 4] films."""
    for r, items in enumerate(items_by_rank):
        buf = gathered[r]
        for i, (f, t) in enumerate(items):
            x0, x1, y0, y1 = tiles[t]
            tw, th = x1 - x0, y1 - y0
            frames_xyzw[f, y0:y1, x0:x1] = np.asarray(buf[i][: tw * th * 4]).reshape(th, tw, 4)
    return frames_xyzw
