"""Summarize a rocprofv3 output tree (gpurun_out/prof_TAG[_CFG], tools/gpu.sh kt / pmc steps) into
profiles/TAG[_CFG]_*: kernel_stats.csv copied as is, plus TAG[_CFG]_pmc.json with per-kernel means of
every PMC counter (and FETCH_SIZE x 2 in bytes, the gfx950 correction from MI355X_MICROARCH.md).
The summary records the bench config it profiled and the hash of the Mo-gather sources, so
bench.py attaches its counters only to a line of the same config and kernel code.

    python tools/summarize_prof.py r03c [c3]
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(tag, cfg="c2"):
    if cfg != "c2":
        tag = "%s_%s" % (tag, cfg)
    src = os.path.join(ROOT, "gpurun_out", "prof_" + tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    ks = os.path.join(src, "kt", "run_kernel_stats.csv")
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(dst, "%s_kernel_stats.csv" % tag))
    out = {}
    for f in sorted(glob.glob(os.path.join(src, "pmc_*", "run_counter_collection.csv"))):
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, d in agg.items():
            e = out.setdefault(k, {})
            if not isinstance(e, dict):
                continue
            for c, v in d.items():
                e[c] = {"dispatches": len(v), "mean": sum(v) / len(v)}
                if c == "FETCH_SIZE":
                    e["fetch_bytes_corrected_mean"] = 2 * 1024 * sum(v) / len(v)
            if "TCC_HIT_sum" in e and "TCC_MISS_sum" in e:
                h, m = e["TCC_HIT_sum"]["mean"], e["TCC_MISS_sum"]["mean"]
                e["l2_hit_rate"] = h / (h + m) if h + m else None
    sys.path.insert(0, ROOT)
    import subprocess
    from bench import kernel_source_hash  # the Mo-gather sources the counters describe
    head = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True,
                          text=True).stdout.strip()
    import time
    out["__meta__"] = {"source_hash": kernel_source_hash(), "git_head_at_summary": head, "config": cfg,
                       "written": time.strftime("%Y-%m-%dT%H:%M:%S")}
    with open(os.path.join(dst, "%s_pmc.json" % tag), "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print("wrote profiles/%s_*" % tag)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "c2")
