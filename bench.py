"""bench.py -- headline benchmark of the MI355X multipole skin path (BASELINE.json metric).

A step = the pixel loop of one skin.pbrt frame (SamplerRenderer::Render's task loop,
samplerrenderer.cpp:191-217): every camera sample is traced, shaded (direct lighting + the
Mo() octree gather) and splatted into the film; at N > 1 the film tiles of every rank
reach rank 0 through one RCCL gather per step.

* Every N (default): config C2, skin.pbrt 1024x1024 at 64 spp -- BASELINE.json's metric is quoted on
  it "@ 1/2/4/8 MI355X", so `value` at every N is the same workload and the driver's per-N
  efficiency compares like with like. At N > 1 a step renders N independent C2 frames, one whole
  frame per GPU (seed + rank; weak scaling: no tile dealing, no load balancing), gathered on rank 0
  by one RCCL gather per step. At N = 1 there is no process group and no gather.
* N > 1 also reports, as `secondary.c3_strong`, north_star's tile scaling of ONE frame: config C3
  (2048x2048, 256 spp) split over the N GPUs as cost-dealt 64x64 tiles (strong scaling).
* --config c3 / c5 select BASELINE.json's other configurations explicitly (their own scaling).

Preprocess (tessellation, irradiance kernel, octree build) runs once before timing and is
reported separately, as SURVEY.md §8d prescribes.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c5]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...
  Without torchrun, --gpus N > 1 starts the N rank processes itself (before any GPU call).
"""
import argparse
import hashlib
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "pbrt-v2-skin_amd"))

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
# SURVEY.md §8d algorithmic bytes of the Mo() gather: per octree record a query needs, position
# 12 + area 4 + 4 bytes per band of E/Et (136 B for 30 bands). The sharded kernel visits
# records per band group, so a step's bytes = 4 B x (record, band) evaluations summed over
# groups + 16 B x the record visits of the busiest group (position/area counted once per
# query-record, as the reference reads them once). Re-reads the sharding adds are not counted.
REC_HDR_BYTES = 16
REF_RECORD_BYTES = 12 + 4 + 4 * 30  # position, area / sumArea, 30-band E / Et
# The L2 request ceiling of the gather's far lookups in the common grid's shape: one group row = two
# 16-byte loads from one 32-byte sector per lane, 64 distinct lines per instruction (the second load of a
# sector hits the vector L1): tools/microbench/l2_width.hip, profiles/r05a_l2_width.json (2.48e11 lane
# lookups/s, 158.6 CU cycles per 64 lane lookups; per-lane 8-byte gathers: 2.53e11, and 2.69e11 in
# their best load form, profiles/r03_l2_policy.json).
L2_GATHER_CEILING_REQ_S = 2.48e11
# The gather's other ceiling, VALU issue (the headline names whichever of the two runs at the larger
# fraction: bench.headline_bound; round 5 ended L2-request-bound, round 6 VALU-bound). It is measured, not
# assumed: tools/microbench/valu_issue.hip runs the record loop's instruction mix (with its SALU) at the
# gather's occupancy (two 1024-thread workgroups per CU, 8 waves per SIMD) and reports wave64 VALU
# instructions per second over the chip. Plain f32 add / mul / fma issue every ~2.3 cycles per SIMD there,
# packed f32, conversions, compares, selects and integer shifts every ~4.2, v_rcp every ~8.2
# (profiles/r05c_valu_issue.json, r05e_valu_issue.json, r06m_valu_issue.json), so the ceiling is the mix's, not a
# per-instruction constant: round 6's record (the row coordinate, the flagged-cell compare, no range test)
# issues at 6.19e11/s there.
VALU_CEILING_JSON = "profiles/r06m_valu_issue.json"
VALU_CEILING_VARIANT = "gather mix r06 (row + LDS record, VALU + SALU)"
# sources whose code the PMC summary's counters describe (profiles/*_pmc.json "source_hash")
KERNEL_SOURCES = ("pbrt-v2-skin_amd/csrc/mo_kernel.hip", "pbrt-v2-skin_amd/csrc/mo_band.h",
                  "pbrt-v2-skin_amd/csrc/mo_wave.h", "pbrt-v2-skin_amd/csrc/octree.h")


# BASELINE.json configs this bench runs: (label, resolution, spp, default scaling, mesh subdivision
# levels). C5's "synthetic 4M-triangle head mesh + 2M irradiance SurfacePoints": head.pbrt
# subdivided 1:4 four times (4.06 M triangles, the same surface) lit and shaded as skin.pbrt,
# with the 2.2 M points of the original mesh's tessellation handed over as a pointsfile would be.
CONFIGS = {
    "c2": ("C2: skin.pbrt 1024x1024 64 spp", 1024, 64, "weak", 0),
    "c3": ("C3: skin.pbrt 2048x2048 256 spp", 2048, 256, "strong", 0),
    "c5": ("C5: synthetic 4M-triangle head + 2.2M SurfacePoints, 4096x4096 512 spp", 4096, 512, "strong", 4),
}


def _code_only(src):
    """A C++ source without its comments and with whitespace runs collapsed: what the compiler sees,
    so that editing a comment does not orphan the PMC summaries of unchanged code (string and char
    literals are kept whole)."""
    out, i, n = [], 0, len(src)
    while i < n:
        c = src[i]
        if c in "\"'":
            j = i + 1
            while j < n and src[j] != c:
                j += 2 if src[j] == "\\" else 1
            out.append(src[i:j + 1])
            i = j + 1
        elif src.startswith("//", i):
            j = src.find("\n", i)
            i = n if j < 0 else j
        elif src.startswith("/*", i):
            j = src.find("*/", i + 2)
            i = n if j < 0 else j + 2
        else:
            out.append(c)
            i += 1
    return " ".join("".join(out).split())


def kernel_source_hash(read=None):
    """Hash of the gather's sources (KERNEL_SOURCES) as code, comments and layout aside. read: a
    function path -> text (default: the working tree)."""
    h = hashlib.sha256()
    for f in KERNEL_SOURCES:
        if read is None:
            with open(os.path.join(ROOT, f), encoding="utf-8") as fh:
                txt = fh.read()
        else:
            txt = read(f)
        h.update(_code_only(txt).encode())
    return h.hexdigest()[:16]


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", choices=sorted(CONFIGS), default=None,
                    help="BASELINE.json config (default c2, the metric's config, at every N: one frame per GPU "
                         "per step; several GPUs add the C3 strong-scaling figure as `secondary`)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default=None,
                    help="weak: one frame per GPU per step; strong: one frame per step split over the GPUs "
                         "(default: the config's)")
    ap.add_argument("--scene", default=os.path.join(ROOT, "scenes", "skin.pbrt"),
                    help="scene file (scenes/skin_textured.pbrt: C2 with imagemap albedo and bump)")
    ap.add_argument("--rgb-profile", action="store_true",
                    help="LayeredSkin \"rgbprofile\" on (ComputeRGBMultipoleProfile: three profiles, FromRGB)")
    ap.add_argument("--sampler", choices=("hash", "reference"), default="hash",
                    help="mpss_config.sampler: hash (default, counter-based (0,2) sequences) or reference (pbrt's "
                         "per-task MT19937 streams replayed, replay_cores emulated cores; the window tables are "
                         "generated per render batch inside the timed region)")
    ap.add_argument("--replay-cores", type=int, default=8)
    ap.add_argument("--res", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--tile", type=int, default=None, help="tile size (default 128; 64 for c3 on several GPUs)")
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--batch-log2", type=int, default=None,
                    help="camera samples per render batch, log2 (mpss_config.max_batch_samples; default 2^26)")
    ap.add_argument("--common-grid", type=int, choices=(0, 1), default=1,
                    help="mpss_config.mo_common_grid: 1 (default) the Mo() gather's far field from the band groups' "
                         "resampled common-grid tables; 0 the per-band tables")
    ap.add_argument("--near-field", type=int, choices=(10236, 5088), default=None,
                    help="mpss_config.mo_near_field (default: the library's)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary figures (C3 strong scaling at N > 1; the reference-sampler C2 frame at N = 1)")
    ap.add_argument("--out", default=None, help="write rank 0's first frame as .pfm/.exr")
    ap.add_argument("--pmc-json", default=None,
                    help="rocprofv3 PMC summary (tools/summarize_prof.py) of this bench command; default: the "
                         "newest profiles/*_pmc.json of this config whose source_hash matches the kernel sources")
    a = ap.parse_args(argv)
    if a.config is None:
        a.config = "c2"
    if a.tile is None:
        a.tile = 64 if a.config == "c3" and a.gpus > 1 else 128
    return a


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _spawned(local_rank, world, port, argv):
    os.environ.update(RANK=str(local_rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    main(parse(argv))


def launch(a, argv):
    """--gpus N > 1 without torchrun: one spawned process per GPU (the parent never touches the
    GPU), rendezvous on 127.0.0.1."""
    import torch.multiprocessing as mp
    mp.start_processes(_spawned, args=(a.gpus, _free_port(), argv), nprocs=a.gpus, join=True, start_method="spawn")


def build_scene(a, label_cfg, local):
    from mpss import pbrtscene
    label, res, spp, scaling, subdiv = CONFIGS[label_cfg]
    res = a.res or res
    spp = a.spp or spp
    sc = pbrtscene.load(a.scene, xres=res, yres=res, spp=spp)
    if a.rgb_profile:
        for m in sc.materials:
            m["rgb_profile"] = 1
    pts = None
    if subdiv:
        pts = pbrtscene.mesh_points(sc)
        sc.meshes = [pbrtscene.subdivide_mesh(me, subdiv) for me in sc.meshes]
    t0 = time.perf_counter()
    kw = {} if a.batch_log2 is None else {"max_batch_samples": 1 << a.batch_log2}
    kw["mo_common_grid"] = a.common_grid
    if a.near_field:
        kw["mo_near_field"] = a.near_field
    if a.sampler == "reference":
        import mpss
        kw["sampler"] = mpss.SAMPLER_REFERENCE
        kw["replay_cores"] = a.replay_cores
    ctx = pbrtscene.build_context(sc, device=local, **kw)
    t_mat = time.perf_counter() - t0
    if pts is not None:
        ctx.set_surface_points(pts)
    t0 = time.perf_counter()
    ctx.preprocess(seed=1)
    import torch
    torch.cuda.synchronize()
    t_pre = time.perf_counter() - t0
    return sc, ctx, label, scaling, subdiv, t_mat, t_pre


def deal(ctx, sc, T, frames, world):
    """Tiles of `frames` frames dealt over `world` ranks (identical on every rank). One frame per
    rank (weak scaling) gives each rank a whole frame: the frames cost the same, and one frame's
    tiles render in one mpss_render_tiles call, one Mo() gather launch per step -- tiles of several
    frames would cost one smaller launch per frame (one seed per call). Otherwise the tiles are
    dealt by estimated cost."""
    import numpy as np
    from mpss import tiles as tl
    tiles = tl.tile_grid(sc.xres, sc.yres, T)
    sss, surf = ctx.tile_costs(tiles)
    px = np.array([(x1 - x0) * (y1 - y0) for x0, x1, y0, y1 in tiles])
    cost1 = tl.tile_cost_model(sss, surf, px)
    items_all = [(f, t) for f in range(frames) for t in range(len(tiles))]
    costs = [cost1[t] for _, t in items_all]
    if frames == world and world > 1:
        nt = len(tiles)
        by_rank_idx = [list(range(r * nt, (r + 1) * nt)) for r in range(world)]
    else:
        by_rank_idx = tl.deal_balanced(costs, world)
    items_by_rank = [[items_all[i] for i in idx] for idx in by_rank_idx]
    return tiles, items_by_rank, tl.balance(costs, by_rank_idx), int((np.asarray(sss) > 0).sum())


def timed_steps(a, ctx, sc, tiles, items_by_rank, frames, T, rank, world, steps, warmup, device="cuda"):
    """Warmup + `steps` timed steps (barrier + synchronize on both sides); returns (max seconds
    over ranks, the gather buffers of rank 0 or None, this rank's output buffer). device: where the
    film tiles live ("cpu" only for the gloo tests' stand-in renderer, tests/test_tiles_dist.py)."""
    import torch
    import torch.distributed as dist
    from mpss import tiles as tl
    mine = items_by_rank[rank]
    slots = max(len(x) for x in items_by_rank)
    seeds = [a.seed + f for f in range(frames)]
    out = torch.zeros((max(slots, 1), T * T * 4), dtype=torch.float32, device=device)
    gath = [torch.zeros_like(out) for _ in range(world)] if (dist.is_initialized() and rank == 0) else None
    on_gpu = device == "cuda"
    stream = torch.cuda.current_stream().cuda_stream if on_gpu else None

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    collective = dist.is_available() and dist.is_initialized()  # any process group, world size 1 included

    def step():
        tl.render_items(ctx, mine, tiles, sc.spp, seeds, out, T, stream)
        if collective:
            dist.gather(out, gath if rank == 0 else None, dst=0)

    for _ in range(warmup):
        step()
    sync()
    ctx.reset_render_stats()  # per-kernel times cover exactly the timed steps
    if collective:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if collective:
        dist.barrier()
    dt = time.perf_counter() - t0
    if collective:
        tt = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    return dt, gath, out


def main(a):
    import numpy as np
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != a.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE %d" % (a.gpus, world))
    if local >= torch.cuda.device_count():
        raise SystemExit("bench.py: rank %d needs HIP device %d but only %d visible" % (rank, local,
                                                                                     torch.cuda.device_count()))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from mpss import tiles as tl

    sc, ctx, label, scaling, subdiv, t_materials, t_pre = build_scene(a, a.config, local)
    scaling = a.scaling or scaling
    n_points = ctx.octree_info()["n_points"] if ctx.surface_points().size else 0
    frames = world if scaling == "weak" else 1  # weak: one frame's worth of work per GPU
    T = a.tile
    t0 = time.perf_counter()
    tiles, items_by_rank, deal_balance, skin_tiles = deal(ctx, sc, T, frames, world)
    t_deal = time.perf_counter() - t0
    mine = items_by_rank[rank]
    seeds = [a.seed + f for f in range(frames)]
    stream = torch.cuda.current_stream().cuda_stream

    # traversal-count pass (untimed): octree records the Mo gather reads for this workload
    out_c = torch.zeros((max(1, len(mine)), T * T * 4), dtype=torch.float32, device="cuda")
    ctx.set_instrumentation(kernel_timing=False, count_traversal=True)
    ctx.reset_render_stats()
    tl.render_items(ctx, mine, tiles, sc.spp, seeds, out_c, T, stream)
    cnt = ctx.render_stats()
    # the reference traversal's record visits: the same pass with the reach pruning off
    ctx.set_instrumentation(kernel_timing=False, count_traversal=2)
    ctx.reset_render_stats()
    tl.render_items(ctx, mine, tiles, sc.spp, seeds, out_c, T, stream)
    cnt_ref = ctx.render_stats()
    del out_c
    ctx.set_instrumentation(kernel_timing=True, count_traversal=False)
    ctx.reset_render_stats()
    dt, gath, out = timed_steps(a, ctx, sc, tiles, items_by_rank, frames, T, rank, world, a.steps, a.warmup)
    st = ctx.render_stats()
    ctx.set_instrumentation(kernel_timing=False, count_traversal=False)

    samples_per_step = frames * sc.xres * sc.yres * sc.spp
    value = samples_per_step * a.steps / dt / 1e6
    # SSS-shaded samples (camera samples that run the Mo() gather): counted on every rank
    sss = torch.tensor([cnt["sss_samples"], cnt["samples"]], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(sss)
    sss_per_step, traced_per_step = float(sss[0].item()), float(sss[1].item())
    # dominant kernel + Mo gather roofline (per-launch averages over the timed region, this rank)
    kern = {"primary": (st["ms_camera"], st["n_camera"]), "shade_direct": (st["ms_direct"], st["n_direct"]),
            "shade_tex": (st["ms_tex"], st["n_tex"]), "replay": (st["ms_replay"], st["n_replay"]),
            "mo_band": (st["ms_shade"], st["n_shade"]),
            "film": (st["ms_film"], st["n_film"])}
    dom = max(kern, key=lambda k: kern[k][0])
    nbands = [sum(1 for c in grp if c >= 0) for grp in cnt["group_bands"]]
    gvis = [cnt["group_nodes"][g] + cnt["group_points"][g] for g in range(8)]
    # algorithmic bytes: 136 B (position, area, 30-band E) per record the reference's
    # Mo() recursion reads, counted by the no-pruning pass (every group walks the same records)
    ref_visits = cnt_ref["group_nodes"][0] + cnt_ref["group_points"][0]
    mo_bytes_step = REF_RECORD_BYTES * ref_visits  # this rank
    # the kernel's own evaluations (after the exact-zero reach pruning), the earlier definition
    kern_bytes_step = sum(gvis[g] * 4 * nbands[g] for g in range(8)) + REC_HDR_BYTES * max(gvis)
    shade_launch_ms = st["ms_shade"] / max(1, st["n_shade"])
    launches_per_step = max(1, st["n_shade"] // max(1, a.steps))
    mo_gbs = mo_bytes_step / launches_per_step / (shade_launch_ms * 1e-3) / 1e9 if shade_launch_ms > 0 else 0.0
    # The gather's roofline: its L2 request rate against the rate
    # tools/microbench/l2_width.hip sustains in the grid's load shape, and its VALU issue against the
    # rate tools/microbench/valu_issue.hip measures for its instruction mix (headline_bound: the larger
    # fraction leads). The counts come from the committed PMC pass of the same config and kernel
    # sources (TCP_TCC_READ_REQ, SQ_INSTS_VALU per launch), the duration from this run's HIP events.
    pt = pmc_traffic(a.pmc_json, shade_launch_ms, a.config)
    roofline = {"kernel": "mo_sort_kernel + mo_band_wave_kernel (Mo gather, spectrally sharded, wave queue)",
                "bound": "l2_requests", "achieved": None, "peak": L2_GATHER_CEILING_REQ_S / 1e9, "unit": "Greq/s",
                "frac": None, "traffic": None, "avg_launch_ms": round(shade_launch_ms, 4),
                "peak_source": "tools/microbench/l2_width.hip: per-lane group-row lookups (two 16-byte loads from "
                               "one 32-byte sector) from a per-XCD-resident table, 64 distinct lines per "
                               "instruction (profiles/r05a_l2_width.json); 0.99 L2 requests (TCP_TCC_READ_REQ) "
                               "per lookup under PMC (profiles/r05k_l2_width_pmc.json)",
                "algorithmic": {"achieved_gbs": round(mo_gbs, 1), "peak_gbs": HBM_PEAK_GBS,
                                "frac": round(mo_gbs / HBM_PEAK_GBS, 4),
                                "bytes_per_launch": mo_bytes_step / launches_per_step,
                                "note": "SURVEY 8d algorithmic throughput (136 B x record visits of the reference "
                                        "Mo() traversal, %.4g visits per SSS sample) / kernel time vs 8 TB/s; the "
                                        "kernel does not move these bytes (exact-zero subtrees pruned, tables in L2), "
                                        "so > 1 is possible -- not an HBM measurement"
                                        % (ref_visits / max(1, cnt["sss_samples"]))},
                "kernel_eval_bytes_per_launch": kern_bytes_step / launches_per_step,
                "dominant_kernel": dom,
                "kernel_ms_per_step": {k: round(v[0] / a.steps, 3) for k, v in kern.items()}}
    if pt:
        roofline["traffic"] = pt.get("traffic")
        roofline["traffic_source"] = pt["source"]
        if "l2" in pt:
            l2 = pt["l2"]
            roofline["achieved"] = round(l2["achieved_req_per_s"] / 1e9, 2)
            roofline["frac"] = round(l2["frac"], 4)
            roofline["l2_requests_per_launch"] = l2["requests_per_launch"]
            roofline["l2_requests_per_sss_sample"] = round(l2["requests_per_launch"] * launches_per_step /
                                                           max(1, cnt["sss_samples"]), 1)
            roofline["l2_hit_rate"] = l2["hit_rate"]
        if roofline["traffic"] is not None:
            roofline["hbm_gbs"] = round(roofline["traffic"] / (shade_launch_ms * 1e-3) / 1e9, 1)
            roofline["hbm_frac"] = round(roofline["hbm_gbs"] / HBM_PEAK_GBS, 4)
        headline_bound(roofline, pt, shade_launch_ms)

    secondary = None
    if world > 1 and a.config == "c2" and not a.no_secondary:
        secondary = c3_strong_secondary(a, rank, world, local)
    if world == 1 and a.config == "c2" and a.sampler == "hash" and not a.no_secondary:
        # pbrt's own sampler on the same frame, and C3's frame on this one GPU: the N = 1 anchor of the
        # c3_strong series the N > 1 lines carry
        secondary = reference_sampler_secondary(a, local)
        secondary.update(c3_strong_secondary(a, rank, world, local))

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(sc, ctx, a)

    if rank == 0:
        line = {"metric": "Msamples/s (%s pixel loop) + Mo()-gather roofline" % ("skin.pbrt C2" if a.config == "c2"
                                                                                 else a.config.upper()),
                "value": round(value, 3),
                "unit": "Msamples/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                "ms_per_step": round(dt / a.steps * 1e3, 3), "higher_is_better": True, "scaling": scaling,
                "vs_baseline": None, "dtype": "f32",
                "data": "synthetic (reconstructed %s, head.pbrt mesh%s%s)" % (
                    os.path.basename(a.scene), ", subdivided" if subdiv else "", ", rgbprofile" if a.rgb_profile else "")
                    + (", pbrt's sampler replayed" if a.sampler == "reference" else ""),
                "config": {"workload": "%s (%dx%d, %d spp%s), %dx%d tiles%s%s"
                           % (label, sc.xres, sc.yres, sc.spp, " per GPU" if scaling == "weak" else "", T, T,
                              ", independent whole frames, one per GPU" if frames == world and world > 1 else
                              (" dealt by cost" if world > 1 else ""),
                              ", one RCCL film gather per step" if world > 1 else ""),
                           "scene": os.path.basename(a.scene), "rgb_profile": bool(a.rgb_profile),
                           "sampler": a.sampler if a.sampler == "hash" else "reference (%d cores)" % a.replay_cores,
                           "frames_per_step": frames, "triangles": int(sum(len(me["indices"]) for me in sc.meshes)),
                           "irradiance_points": n_points, "preprocess_s": round(t_pre, 3),
                           "material_build_s": round(t_materials, 3), "tile_deal_s": round(t_deal, 3),
                           "tiles": len(tiles), "skin_tiles": skin_tiles, "deal_balance": round(deal_balance, 4),
                           "sss_hit_fraction": round(sss_per_step / max(1.0, traced_per_step), 4),
                           "sss_samples_per_s": round(sss_per_step * a.steps / dt, 1),
                           "mo_algorithmic_gbs": round(mo_gbs, 1), "mo_sss_samples": cnt["sss_samples"],
                           "mo_record_visits_per_sss_sample": round((cnt["mo_nodes"] + cnt["mo_points"]) /
                                                                    max(1, cnt["sss_samples"]), 2),
                           "mo_group_visits": [x + y for x, y in zip(cnt["group_nodes"], cnt["group_points"])],
                           "mo_lane_efficiency": round((cnt["mo_nodes"] + cnt["mo_points"]) /
                                                       max(1, 64 * (cnt["mo_wave_node_iters"] +
                                                                    cnt["mo_wave_point_iters"])), 4),
                           "mo_lookup_near_fraction": [round(x / max(1, cnt["mo_lookups"]), 4)
                                                       for x in cnt["mo_lookups_near"]],
                           "mo_wave_iters": {"node": cnt["mo_wave_node_iters"], "point": cnt["mo_wave_point_iters"]},
                           "mo_common_grid": bool(ctx.gather_info(0)["common_grid"]) if sc.materials else False,
                           "mo_lane_records": {"rows": cnt["mo_row_lane_records"], "lds": cnt["mo_lds_lane_records"],
                                                  "tables": cnt["mo_table_lane_records"]},
                           "mo_l2_footprint": l2_footprint(cnt),
                           "mo_visits": {"node": cnt["mo_nodes"], "point": cnt["mo_points"],
                                         "lookups_in_profile": cnt["mo_lookups"]}},
                "roofline": roofline, "cpu_baseline": cpu}
        if secondary:
            line["secondary"] = secondary
        print(json.dumps(line), flush=True)
    if a.out and rank == 0:
        from mpss import film
        img = np.zeros((frames, sc.yres, sc.xres, 4), np.float32)
        g = [x.cpu().numpy() for x in gath] if gath is not None else [out.cpu().numpy()]
        tl.assemble(img, g, items_by_rank, tiles, T)
        rgb = film.finalize(img[0])
        film.write_image(a.out, rgb)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def l2_footprint(cnt):
    """The count pass's L2 footprint of the gather's far lookups by path (mo_band.h kHist 7..12): per band
    group, lane-records on the group rows / LDS / own tables, and for the rows and own tables the distinct
    32-byte sectors and 128-byte lines their loads touch, summed over wave fetches (what the
    vector-memory path asks of L2), and the wave fetches. Per SSS sample in "per_sss_sample"."""
    ns = max(1, cnt["sss_samples"])
    rec = cnt["group_path_records"]
    out = {"per_group": [{"records": rec[g], "sectors": cnt["group_path_sectors"][g],
                          "lines": cnt["group_path_lines"][g], "fetches": cnt["group_path_fetches"][g]}
                         for g in range(8)]}
    tot = {}
    for i, path in enumerate(("rows", "tables")):
        tot[path] = {k: int(sum(cnt["group_path_" + k][g][i] for g in range(8)))
                     for k in ("sectors", "lines", "fetches")}
        tot[path]["records"] = int(sum(rec[g][0 if i == 0 else 2] for g in range(8)))
    tot["lds"] = {"records": int(sum(rec[g][1] for g in range(8)))}
    out["total"] = tot
    out["per_sss_sample"] = {p: {k: round(v / ns, 1) for k, v in d.items()} for p, d in tot.items()}
    return out


def c3_strong_secondary(a, rank, world, local):
    """C3 strong scaling beside the C2 line: ONE skin.pbrt 2048x2048 256-spp frame per step split
    over the N ranks as cost-dealt 64x64 tiles, gathered on rank 0 (north_star's tile scaling)."""
    import torch
    sc, ctx, _, _, _, _, _ = build_scene(a, "c3", local)
    T = 64
    tiles, items_by_rank, balance, _ = deal(ctx, sc, T, 1, world)
    torch.cuda.synchronize()
    steps = max(1, min(a.steps, 3))
    dt, _, _ = timed_steps(a, ctx, sc, tiles, items_by_rank, 1, T, rank, world, steps, 1)
    ctx.close()
    return {"c3_strong": {"value": round(sc.xres * sc.yres * sc.spp * steps / dt / 1e6, 3),
                          "unit": "Msamples/s", "ms_per_step": round(dt / steps * 1e3, 3), "frames_per_step": 1,
                          "tiles": len(tiles), "deal_balance": round(balance, 4), "scaling": "strong"}}


def valu_ceiling():
    """(wave64 VALU instructions / s over the chip, shader clock GHz, source) of the gather's record mix
    at 8 waves per SIMD, from the committed microbenchmark run (VALU_CEILING_JSON), or None."""
    try:
        d = json.load(open(os.path.join(ROOT, VALU_CEILING_JSON)))
    except (OSError, ValueError):
        return None
    for r in d.get("results", []):
        if r.get("variant") == VALU_CEILING_VARIANT and r.get("waves_per_simd") == 8:
            return (r["valu_wave_insts_per_s"], r.get("clock_ghz"),
                    "%s, variant \"%s\" at 8 waves per SIMD: %.4g wave64 VALU/s (%.2f SIMD cycles per instruction "
                    "at %.2f GHz)" % (VALU_CEILING_JSON, VALU_CEILING_VARIANT, r["valu_wave_insts_per_s"],
                                      r["simd_cycles_per_valu_inst"], r.get("clock_ghz") or 0.0))
    return None


def reference_sampler_secondary(a, local):
    """The same C2 frame with pbrt's own sampler replayed (mpss_config.sampler = MPSS_SAMPLER_REFERENCE,
    --replay-cores emulated cores: SamplerRendererTask's per-task MT19937 streams, samplerrenderer.cpp:
    60-167), timed like the headline: the replay window's generation (replay_window_kernel) is inside every
    step. This is the mode whose output is pbrt's own, sample for sample."""
    import argparse
    b = argparse.Namespace(**vars(a))
    b.sampler = "reference"
    sc, ctx, _, _, _, _, _ = build_scene(b, "c2", local)
    T = a.tile
    tiles, items_by_rank, _, _ = deal(ctx, sc, T, 1, 1)
    steps = max(1, min(a.steps, 5))
    ctx.set_instrumentation(kernel_timing=True, count_traversal=False)
    dt, _, _ = timed_steps(b, ctx, sc, tiles, items_by_rank, 1, T, 0, 1, steps, 1)
    st = ctx.render_stats()
    ctx.close()
    return {"reference_sampler": {
        "value": round(sc.xres * sc.yres * sc.spp * steps / dt / 1e6, 3), "unit": "Msamples/s",
        "ms_per_step": round(dt / steps * 1e3, 3), "replay_cores": a.replay_cores,
        "kernel_ms_per_step": {"replay": round(st["ms_replay"] / steps, 3), "mo_band": round(st["ms_shade"] / steps, 3),
                               "primary": round(st["ms_camera"] / steps, 3),
                               "shade_direct": round(st["ms_direct"] / steps, 3), "film": round(st["ms_film"] / steps, 3)},
        "note": "C2 with pbrt's per-task MT19937 sample streams replayed (the window generation timed in every step)"}}


def headline_bound(roofline, pt, launch_ms):
    """The headline names the resource that binds the gather hardest: the L2 request rate of its
    lookups (rounds 2-3) or VALU issue (round 4 on), whichever runs at the larger fraction of its
    measured ceiling; the other stays beside it (`roofline.l2_requests` / `roofline.valu_issue`). The
    VALU peak is the measured issue rate of the record loop's instruction mix at the kernel's
    occupancy (valu_ceiling), cross-checked by the counters' own VALU busy fraction
    (SQ_ACTIVE_INST_VALU over SQ_BUSY_CU_CYCLES: the SIMDs' cycles with a VALU instruction in flight,
    from the same PMC summary)."""
    v = pt.get("valu") if pt else None
    ceil = valu_ceiling()
    if not v or not ceil or launch_ms <= 0:
        return
    achieved = v["insts_per_launch"] / (launch_ms * 1e-3)
    frac = achieved / ceil[0]
    valu = {"achieved": round(achieved / 1e9, 1), "peak": round(ceil[0] / 1e9, 1),
            "unit": "G wave64 VALU instructions/s", "frac": round(frac, 4),
            "peak_source": ceil[2] + "; achieved = SQ_INSTS_VALU per launch (committed PMC summary) / this run's "
                                     "launch time"}
    if "busy" in v:
        valu["busy_pmc"] = round(v["busy"], 4)
        valu["busy_source"] = ("SQ_ACTIVE_INST_VALU / SQ_BUSY_CU_CYCLES per launch (quad-cycles with a VALU "
                               "instruction in flight per SIMD over the CUs' busy cycles / 4 SIMDs x 4)")
    if roofline.get("frac") is not None and frac <= roofline["frac"]:
        roofline["valu_issue"] = valu
        return
    if roofline.get("achieved") is not None:
        roofline["l2_requests"] = {"achieved": roofline["achieved"], "peak": roofline["peak"], "unit": "Greq/s",
                                   "frac": roofline["frac"], "peak_source": roofline.get("peak_source")}
    roofline["bound"] = "valu_issue"
    for k in ("achieved", "peak", "unit", "frac", "peak_source"):
        roofline[k] = valu[k]
    if "busy_pmc" in valu:
        roofline["valu_busy_pmc"] = valu["busy_pmc"]
        roofline["valu_busy_source"] = valu["busy_source"]


def pmc_traffic(path, launch_ms, config):
    """Counters of one mo_band_wave_kernel launch from a committed rocprofv3 PMC summary
    (tools/summarize_prof.py) of the same bench config: HBM-side traffic FETCH_SIZE x 2 (the gfx950
    correction, MI355X_MICROARCH.md), and the L2 request rate (TCP_TCC_READ_REQ per launch / this
    run's launch time) against the measured gather ceiling. Only a summary whose source_hash
    matches the current kernel sources is used (the newest one); an older one is named as stale."""
    import glob
    cands = [path] if path else glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json"))
    want = kernel_source_hash()
    best, stale = None, None
    for f in cands:
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        meta = d.get("__meta__", {})
        if not path and meta.get("config", "c2") != config:
            continue
        e = next((v for k, v in d.items() if k.startswith("void mpss::mo_band_wave_kernel<false")), None)
        if not e or "fetch_bytes_corrected_mean" not in e:
            continue
        if meta.get("source_hash") != want:
            stale = stale or os.path.relpath(f, ROOT)
            continue
        if best is None or meta.get("written", "") > best[0]:
            best = (meta.get("written", ""), f, e)
    if best is None:
        if stale:
            return {"traffic": None, "source": "none current: PMC summary %s was profiled on other kernel sources "
                                              "(source_hash mismatch)" % stale}
        return None
    _, f, e = best
    out = {"traffic": e["fetch_bytes_corrected_mean"],
           "source": os.path.relpath(f, ROOT) + " (FETCH_SIZE x 2 per launch, includes Infinity-Cache hits)"}
    if "SQ_INSTS_VALU" in e and launch_ms > 0:
        # VALU issue: wave64 instructions per launch (against the measured mix ceiling: headline_bound)
        v = e["SQ_INSTS_VALU"]["mean"]
        out["valu"] = {"insts_per_launch": v}
        if "SQ_ACTIVE_INST_VALU" in e and e.get("SQ_BUSY_CU_CYCLES", {}).get("mean"):
            # quad-cycles with a VALU instruction in flight, summed over waves (per SIMD), over the CUs'
            # busy cycles: 4 SIMDs x quad-cycles / (4 x cycles) -> the fraction of SIMD cycles
            out["valu"]["busy"] = e["SQ_ACTIVE_INST_VALU"]["mean"] / e["SQ_BUSY_CU_CYCLES"]["mean"]
    if "TCP_TCC_READ_REQ_sum" in e and launch_ms > 0:
        req = e["TCP_TCC_READ_REQ_sum"]["mean"]
        out["l2"] = {"requests_per_launch": req, "achieved_req_per_s": req / (launch_ms * 1e-3),
                     "frac": req / (launch_ms * 1e-3) / L2_GATHER_CEILING_REQ_S, "hit_rate": e.get("l2_hit_rate")}
    return out


def cpu_baseline(sc, ctx, a):
    """The CPU restatement (oracle/, test infrastructure) timed on a bounded sample of the same
    workload: whole tiles of the same frame, same points, same sampler, until the time budget is
    spent. Reported as a baseline only; it never feeds `value`."""
    try:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_render
    except Exception as e:  # noqa: BLE001
        return {"value": None, "unit": "Msamples/s", "cores": None, "kind": "port", "sample": "unavailable: %s" % e}
    return oracle_render.time_cpu_baseline(sc, ctx, sc.spp, a.seed, a.cpu_baseline_seconds)


def check_devices(n):
    """Fail fast when the node has fewer GPUs than --gpus asks for (device_count() does not
    initialise the GPU on this image, so the self-spawn path stays exec-safe)."""
    import torch
    have = torch.cuda.device_count()
    if have < n:
        raise SystemExit("bench.py: --gpus %d but only %d HIP device(s) visible" % (n, have))


if __name__ == "__main__":
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        check_devices(args.gpus)
        launch(args, sys.argv[1:])
    else:
        main(args)
