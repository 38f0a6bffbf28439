"""Image-tile sharding of the pixel loop across ranks.

pbrt splits the film into RoundUpPow2(max(32*cores, W*H/256)) sampler tasks
(renderers/samplerrenderer.cpp:177-199, Sampler::ComputeSubWindow in core/sampler.cpp:55-78);
here the unit is a T x T pixel tile handed to one GPU, tiles are dealt to ranks interleaved
(balancing the face in the middle of the frame against empty background), and each rank's
film tiles reach rank 0 through one collective gather at the end of the frame.
"""
import numpy as np


def tile_grid(W, H, T):
    """Row-major list of (x0, x1, y0, y1) tiles covering a W x H film."""
    return [(x0, min(x0 + T, W), y0, min(y0 + T, H)) for y0 in range(0, H, T) for x0 in range(0, W, T)]


def rank_items(n_items, rank, world):
    """Work items of `rank` when n_items are dealt round-robin over `world` ranks."""
    return list(range(rank, n_items, world))


def slots_per_rank(n_items, world):
    return (n_items + world - 1) // world


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
