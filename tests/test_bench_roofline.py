"""bench.py's headline roofline from the committed measurements (CPU: no GPU call).

The VALU-issue peak comes from the committed microbenchmark of the gather's instruction mix
(bench.VALU_CEILING_JSON), the achieved rate from the committed PMC summary whose source hash
matches the gather's current sources; the PMC's own VALU-busy fraction (SQ_ACTIVE_INST_VALU /
SQ_BUSY_CU_CYCLES) must agree with its frac within 10 %, and the headline is whichever of VALU issue and
the L2 request rate runs at the larger fraction of its ceiling. The launch time is that of the bench
run the PMC summary was taken beside (profiles/r05z_bench_c2.jsonl)."""
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    import sys
    sys.path.insert(0, ROOT)
    import bench as b
    return b


def test_valu_ceiling_is_a_committed_measurement(bench):
    c = bench.valu_ceiling()
    assert c is not None, bench.VALU_CEILING_JSON
    rate, ghz, src = c
    # 1024 SIMDs issuing the mix every ~4 cycles at ~2.3 GHz: between the plain-f32 and packed rates
    assert 4e11 < rate < 1.1e12 and 1.5 < ghz < 2.6
    assert bench.VALU_CEILING_JSON in src


def test_headline_is_valu_issue_and_agrees_with_pmc_busy(bench, monkeypatch):
    # the final round-5 PMC summary and the bench line measured beside it (bench.py only uses a summary
    # whose source hash matches the gather's current sources; here the summary is named, and its own
    # hash stands in for the sources', so that the check does not depend on later source edits)
    tag = "r05z"
    pmc = os.path.join(ROOT, "profiles", tag + "_pmc.json")
    monkeypatch.setattr(bench, "kernel_source_hash", lambda: json.load(open(pmc))["__meta__"]["source_hash"])
    line = json.loads(open(os.path.join(ROOT, "profiles", tag + "_bench_c2.jsonl")).readline())
    launch_ms = line["roofline"]["avg_launch_ms"]
    pt = bench.pmc_traffic(pmc, launch_ms, "c2")
    assert pt is not None and "valu" in pt
    assert pt["traffic"] > 0 and 0 < pt["l2"]["frac"] < 1
    roof = {"bound": "l2_requests", "achieved": pt["l2"]["achieved_req_per_s"] / 1e9,
            "peak": bench.L2_GATHER_CEILING_REQ_S / 1e9, "frac": pt["l2"]["frac"], "peak_source": "l2"}
    bench.headline_bound(roof, pt, launch_ms)
    # both ceilings reported; the headline is the one run at the larger fraction
    valu = roof if roof["bound"] == "valu_issue" else roof["valu_issue"]
    l2 = roof["l2_requests"] if roof["bound"] == "valu_issue" else roof
    assert 0 < valu["frac"] <= 1.0 and 0 < l2["frac"] <= 1.0
    assert roof["frac"] == max(valu["frac"], l2["frac"])
    busy = valu["busy_pmc"] if "busy_pmc" in valu else roof["valu_busy_pmc"]
    assert abs(valu["frac"] / busy - 1) <= 0.10, (valu["frac"], busy)
