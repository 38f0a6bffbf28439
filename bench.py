"""bench.py -- headline benchmark of the MI355X multipole skin path (BASELINE.json metric).

A step = the pixel loop of one skin.pbrt frame per GPU (config C2: 1024x1024, 64 spp,
MultipoleSubsurfaceIntegrator + LayeredSkin; SamplerRenderer::Render's task loop,
samplerrenderer.cpp:177-236): every camera sample is traced, shaded (direct lighting + the
Mo() octree gather) and splatted into the film. Frames are cut into 128x128 tiles dealt to
ranks round-robin; rank 0 collects every rank's film tiles with one RCCL gather per step.
Weak scaling: at N GPUs a step renders N frames (different sampler seeds). --config c3 / c5
run BASELINE.json's 8-GPU configs instead (one frame per step split over the GPUs: strong
scaling); they are reference points, the driver's bench line is C2.

Preprocess (tessellation, irradiance kernel, octree build) runs once before timing and is
reported separately, as SURVEY.md §8d prescribes.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c5]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
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


# BASELINE.json configs this bench runs: (label, resolution, spp, default scaling, mesh subdivision
# levels). C5's "synthetic 4M-triangle head mesh + 2M irradiance SurfacePoints": head.pbrt
# subdivided 1:4 four times (4.06 M triangles, the same surface) lit and shaded as skin.pbrt,
# with the 2.2 M points of the original mesh's tessellation handed over as a pointsfile would be.
CONFIGS = {
    "c2": ("C2: skin.pbrt 1024x1024 64 spp", 1024, 64, "weak", 0),
    "c3": ("C3: skin.pbrt 2048x2048 256 spp", 2048, 256, "strong", 0),
    "c5": ("C5: synthetic 4M-triangle head + 2.2M SurfacePoints, 4096x4096 512 spp", 4096, 512, "strong", 4),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c2",
                    help="BASELINE.json config: c2 (default; the metric's), c3 or c5 (8-GPU configs, strong scaling)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default=None,
                    help="weak: one frame per GPU per step; strong: one frame per step split over the GPUs "
                         "(default: the config's)")
    ap.add_argument("--scene", default=os.path.join(ROOT, "scenes", "skin.pbrt"))
    ap.add_argument("--res", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--tile", type=int, default=128)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--out", default=None, help="write rank 0's first frame as .pfm/.exr")
    ap.add_argument("--pmc-json", default=None,
                    help="rocprofv3 PMC summary (tools/summarize_prof.py) of this bench command; default: the "
                         "newest profiles/*_pmc.json with a FETCH_SIZE entry for mo_band_kernel")
    return ap.parse_args()


def main():
    a = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != a.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE %d" % (a.gpus, world))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import mpss
    from mpss import pbrtscene, tiles as tl

    label, res, spp, scaling, subdiv = CONFIGS[a.config]
    res = a.res or res
    spp = a.spp or spp
    scaling = a.scaling or scaling
    sc = pbrtscene.load(a.scene, xres=res, yres=res, spp=spp)
    pts = None
    if subdiv:
        pts = pbrtscene.mesh_points(sc)
        sc.meshes = [pbrtscene.subdivide_mesh(me, subdiv) for me in sc.meshes]
    t0 = time.perf_counter()
    ctx = pbrtscene.build_context(sc, device=local)
    t_materials = time.perf_counter() - t0
    if pts is not None:
        ctx.set_surface_points(pts)
    t0 = time.perf_counter()
    ctx.preprocess(seed=1)
    torch.cuda.synchronize()
    t_pre = time.perf_counter() - t0
    n_points = ctx.octree_info()["n_points"] if ctx.surface_points().size else 0

    frames = world if scaling == "weak" else 1  # weak: one frame's worth of work per GPU
    T = a.tile
    tiles = tl.tile_grid(sc.xres, sc.yres, T)
    items_all = [(f, t) for f in range(frames) for t in range(len(tiles))]
    items_by_rank = [[items_all[i] for i in tl.rank_items(len(items_all), r, world)] for r in range(world)]
    mine = items_by_rank[rank]
    slots = tl.slots_per_rank(len(items_all), world)
    seeds = [a.seed + f for f in range(frames)]
    out = torch.zeros((slots, T * T * 4), dtype=torch.float32, device="cuda")
    gath = [torch.zeros_like(out) for _ in range(world)] if (world > 1 and rank == 0) else None
    stream = torch.cuda.current_stream().cuda_stream

    def step():
        tl.render_items(ctx, mine, tiles, sc.spp, seeds, out, T, stream)
        if world > 1:
            dist.gather(out, gath if rank == 0 else None, dst=0)

    # traversal-count pass (untimed): octree records the Mo gather reads for this workload
    ctx.set_instrumentation(kernel_timing=False, count_traversal=True)
    ctx.reset_render_stats()
    tl.render_items(ctx, mine, tiles, sc.spp, seeds, out, T, stream)
    cnt = ctx.render_stats()
    ctx.set_instrumentation(kernel_timing=False, count_traversal=False)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ctx.set_instrumentation(kernel_timing=True, count_traversal=False)
    ctx.reset_render_stats()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    st = ctx.render_stats()
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())

    samples_per_step = frames * sc.xres * sc.yres * sc.spp
    value = samples_per_step * a.steps / dt / 1e6
    # dominant kernel + Mo gather roofline (per-launch averages over the timed region)
    kern = {"primary": (st["ms_camera"], st["n_camera"]), "shade_direct": (st["ms_direct"], st["n_direct"]),
            "mo_band": (st["ms_shade"], st["n_shade"]),
            "film": (st["ms_film"], st["n_film"])}
    dom = max(kern, key=lambda k: kern[k][0])
    nbands = [sum(1 for c in grp if c >= 0) for grp in cnt["group_bands"]]
    gvis = [cnt["group_nodes"][g] + cnt["group_points"][g] for g in range(8)]
    mo_bytes_step = sum(gvis[g] * 4 * nbands[g] for g in range(8)) + REC_HDR_BYTES * max(gvis)  # this rank
    shade_launch_ms = st["ms_shade"] / max(1, st["n_shade"])
    launches_per_step = max(1, st["n_shade"] // max(1, a.steps))
    mo_gbs = mo_bytes_step / launches_per_step / (shade_launch_ms * 1e-3) / 1e9 if shade_launch_ms > 0 else 0.0
    roofline = {"kernel": "mo_band_kernel (Mo gather, spectrally sharded)", "bound": "hbm", "achieved": round(mo_gbs, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(mo_gbs / HBM_PEAK_GBS, 4), "traffic": None,
                "bytes_per_launch": mo_bytes_step / launches_per_step, "avg_launch_ms": round(shade_launch_ms, 4),
                "dominant_kernel": dom,
                "kernel_ms_per_step": {k: round(v[0] / a.steps, 3) for k, v in kern.items()}}
    # the committed PMC summaries are of the C2 command; other configs report traffic only with --pmc-json
    pt = pmc_traffic(a.pmc_json, shade_launch_ms) if (a.config == "c2" or a.pmc_json) else None
    if pt:
        roofline["traffic"] = pt["traffic"]
        roofline["traffic_source"] = pt["source"] + " (FETCH_SIZE x 2 per launch, includes Infinity-Cache hits)"
        if "l2" in pt:
            roofline["l2_request_roofline"] = pt["l2"]

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(sc, ctx, a)

    if rank == 0:
        line = {"metric": "Msamples/s (%s pixel loop) + Mo()-gather HBM GB/s" % ("skin.pbrt C2" if a.config == "c2"
                                                                                   else a.config.upper()),
                "value": round(value, 3),
                "unit": "Msamples/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                "ms_per_step": round(dt / a.steps * 1e3, 3), "higher_is_better": True, "scaling": scaling,
                "vs_baseline": None, "dtype": "f32",
                "data": "synthetic (reconstructed skin.pbrt, head.pbrt mesh%s)" % (", subdivided" if subdiv else ""),
                "config": {"workload": "%s (%dx%d, %d spp%s), %dx%d tiles, RCCL film gather"
                           % (label, sc.xres, sc.yres, sc.spp, " per GPU" if scaling == "weak" else "", T, T),
                           "frames_per_step": frames, "triangles": int(sum(len(me["indices"]) for me in sc.meshes)),
                           "irradiance_points": n_points, "preprocess_s": round(t_pre, 3),
                           "material_build_s": round(t_materials, 3),
                           "mo_gbs": round(mo_gbs, 1), "mo_sss_samples": cnt["sss_samples"],
                           "mo_record_visits_per_sss_sample": round((cnt["mo_nodes"] + cnt["mo_points"]) /
                                                                    max(1, cnt["sss_samples"]), 2),
                           "mo_group_visits": [a + b for a, b in zip(cnt["group_nodes"], cnt["group_points"])],
                           "mo_lane_efficiency": round((cnt["mo_nodes"] + cnt["mo_points"]) /
                                                       max(1, 64 * (cnt["mo_wave_node_iters"] +
                                                                    cnt["mo_wave_point_iters"])), 4),
                           "mo_lookup_near_fraction": [round(x / max(1, cnt["mo_lookups"]), 4)
                                                       for x in cnt["mo_lookups_near"]]},
                "roofline": roofline, "cpu_baseline": cpu}
        print(json.dumps(line), flush=True)
    if a.out and rank == 0:
        from mpss import film
        img = np.zeros((frames, sc.yres, sc.xres, 4), np.float32)
        g = [x.cpu().numpy() for x in gath] if gath is not None else [out.cpu().numpy()]
        tl.assemble(img, g, items_by_rank, tiles, T)
        rgb = film.finalize(img[0])
        (film.write_exr if a.out.endswith(".exr") else film.write_pfm)(a.out, rgb)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


L2_PEAK_REQ_PER_S = 34.5e12 / 128  # MI355X L2 ~34.5 TB/s aggregate (MI355X_MICROARCH.md), 128-B lines


def pmc_traffic(path, launch_ms):
    """HBM-side traffic of one mo_band_kernel launch from a committed rocprofv3 PMC summary of
    the same bench command: FETCH_SIZE x 2 (the gfx950 correction, MI355X_MICROARCH.md), and
    the L2 request rate (TCC_HIT + TCC_MISS per launch / launch time)."""
    import glob
    cands = [path] if path else sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")),
                                       reverse=True)  # newest round tag first (r01j > r01i > ... > r01)
    for f in cands:
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        e = d.get("void mpss::mo_band_kernel<false>")
        if not e or "fetch_bytes_corrected_mean" not in e:
            continue
        out = {"traffic": e["fetch_bytes_corrected_mean"], "source": os.path.relpath(f, ROOT)}
        if "TCC_HIT_sum" in e and launch_ms > 0:
            req = e["TCC_HIT_sum"]["mean"] + e["TCC_MISS_sum"]["mean"]
            out["l2"] = {"requests_per_launch": req, "achieved_req_per_s": req / (launch_ms * 1e-3),
                         "peak_req_per_s": L2_PEAK_REQ_PER_S,
                         "frac": req / (launch_ms * 1e-3) / L2_PEAK_REQ_PER_S, "hit_rate": e.get("l2_hit_rate")}
        return out
    return None


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


if __name__ == "__main__":
    main()
