"""Config C4 (BASELINE.json): the Monte-Carlo layered profile of scenes/mcprofile.pbrt on one GPU,
with the CPU oracle (oracle/mc.c, all host threads up to 16) timed on a bounded photon sample.

    python tools/bench_mc.py [--photons 100000000] [--cpu-seconds 10]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pbrt-v2-skin_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default=os.path.join(ROOT, "scenes", "mcprofile.pbrt"))
    ap.add_argument("--photons", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--out", default=None, help="write the profile table (reference output layout)")
    a = ap.parse_args()
    import torch
    import mpss
    from mpss import pbrtscene
    sc = pbrtscene.load(a.scene)
    kind, ps = sc.renderer
    lay = ps.find("layers")
    layers = [tuple(lay[4 * i:4 * i + 4]) for i in range(len(lay) // 4)]
    mfpr = float(ps.one("mfprange", 16.0))
    nseg = int(ps.one("segments", 1024))
    n = a.photons or int(ps.one("photons", "100"))
    assert torch.cuda.is_available()
    ctx = mpss.Context()
    ctx.mc_profile(layers, mfpr, nseg, 100000, seed=1)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g = ctx.mc_profile(layers, mfpr, nseg, n, seed=89)
    dt = time.perf_counter() - t0
    line = {"metric": "photons/s (C4 mcprofile, Monte-Carlo layered profile)", "value": round(n / dt, 1),
            "unit": "photons/s", "photons": n, "seconds": round(dt, 3), "events_per_s": round(g["events"] / dt, 1),
            "total_r": g["total_r"], "total_t": g["total_t"], "layers": layers, "mfp_range": mfpr,
            "segments": nseg}
    line["roofline"] = mc_roofline(dt)
    if a.cpu_seconds > 0:
        import oracle_mc
        m = 20000
        t0 = time.perf_counter()
        while True:
            oracle_mc.mc_profile(layers, mfpr, nseg, m, seed=89)
            el = time.perf_counter() - t0
            if el > a.cpu_seconds or m >= n:
                break
            t0 = time.perf_counter()
            m *= 4
        line["cpu_baseline"] = {"value": round(m / el, 1), "unit": "photons/s", "cores": min(16, os.cpu_count()),
                                "kind": "port", "sample": "%d photons of the same layers, oracle/mc.c" % m}
    print(json.dumps(line), flush=True)
    if a.out:
        ext = None
        with open(a.out, "w") as f:
            import numpy as np
            mfp = np.mean([1.0 / (l[0] + l[1]) for l in layers])
            ext = mfpr * mfp
            dist = [(i + 0.5) * ext / nseg for i in range(nseg)]
            f.write("Name\tTotal" + "".join("\t%g" % d for d in dist) + "\n")
            f.write("Monte-Carlo Reflectance\t%g\t" % g["total_r"] + "\t".join("%g" % v for v in g["reflectance"]) + "\n")
            f.write("Monte-Carlo Transmittance\t%g\t" % g["total_t"] + "\t".join("%g" % v for v in g["transmittance"]) + "\n")


# VALU issue peak of MI355X: 256 CUs x 4 SIMDs x 2.4 GHz / 4 cycles per wave64 instruction (FP64
# FMA runs at the FP32 rate: 78.6 TFLOP/s FP64 vector = 256 x 4 x 16 lanes x 2 x 2.4 GHz)
VALU_PEAK_INST_S = 256 * 4 * 2.4e9 / 4


def mc_roofline(seconds):
    """The walk is FP64 arithmetic with LDS tallies: its bound is VALU issue. Instructions come from
    the committed PMC summary of this command (profiles/*_c4_pmc.json, tools/gpu.sh pmc_mc), the time
    from this run; none current -> achieved null."""
    import glob
    best = None
    for f in glob.glob(os.path.join(ROOT, "profiles", "*_c4_pmc.json")):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        e = next((v for k, v in d.items() if "mc_profile_kernel" in k), None)
        if not e or "SQ_INSTS_VALU" not in e:
            continue
        w = d.get("__meta__", {}).get("written", "")
        if best is None or w > best[0]:
            best = (w, f, e)
    r = {"kernel": "mc_profile_kernel (FP64 layered random walk)", "bound": "valu", "achieved": None,
         "peak": VALU_PEAK_INST_S / 1e9, "unit": "G wave64 VALU instructions/s", "frac": None, "traffic": None,
         "peak_source": "256 CUs x 4 SIMDs x 2.4 GHz / 4 cycles (MI355X_MICROARCH.md clocks and widths)",
         "note": "issue-slot fraction: an FP64 transcendental (log / sqrt / sin / cos of the walk) counts once "
                 "but holds its SIMD for several cycles"}
    if best:
        _, f, e = best
        inst = e["SQ_INSTS_VALU"]["mean"] * e["SQ_INSTS_VALU"]["dispatches"]
        # the PMC run counts the 1e5-photon warm-up walk too (0.1 % of the 1e8-photon walk's instructions)
        r["achieved"] = round(inst / seconds / 1e9, 2) if inst else None
        r["frac"] = round(inst / seconds / VALU_PEAK_INST_S, 4) if inst else None
        r["source"] = os.path.relpath(f, ROOT) + " (SQ_INSTS_VALU summed over the command's dispatches)"
        if "fetch_bytes_corrected_mean" in e:
            r["traffic"] = e["fetch_bytes_corrected_mean"] * e["FETCH_SIZE"]["dispatches"]
    return r


if __name__ == "__main__":
    main()
