"""The image parity criterion of the GPU tests, and the report of the error they actually reach.

check_image(got, ref, name): north_star's criterion as stated -- film weights bit-exact (the
sample-to-pixel mapping) and XYZ within TOL = 1e-4 RELATIVE L-inf: max |gpu - cpu| / |cpu| over
every channel value with cpu != 0, no absolute floor, and no value zero on one side only. (Round 2
used a floor at 1e-3 of the window's peak; the measured unfloored error is <= 8e-7 on every
image test, profiles/r03b_parity.jsonl, so the floor is gone.) Each call appends its figures
(relative L-inf, where it occurs relative to the peak, the 99.9th percentile, and the round-2
floored figure) to the JSONL file named by $MPSS_PARITY_REPORT (tools/gpu.sh sets it).
"""
import json
import os

import numpy as np

TOL = 1e-4


def image_errors(got, ref):
    g, r = got[..., :3].astype(np.float64), ref[..., :3].astype(np.float64)
    peak = float(np.abs(r).max())
    err = np.abs(g - r)
    nz = r != 0
    rel = err[nz] / np.abs(r[nz])
    floored = err / (TOL * np.maximum(np.abs(r), 1e-3 * peak)) if peak > 0 else err
    # the relative error over the values above a fraction of the peak (where the worst one sits)
    above = {}
    for fr in (1e-3, 1e-5, 1e-7, 1e-9):
        sel = np.abs(r[nz]) >= fr * peak
        above["%g" % fr] = float(rel[sel].max()) if sel.any() else 0.0
    return {"peak": peak, "rel_linf": float(rel.max()) if rel.size else 0.0, "rel_linf_above": above,
            "rel_linf_at_value": float(np.abs(r[nz])[rel.argmax()] / peak) if rel.size and peak > 0 else None,
            "rel_p999": float(np.quantile(rel, 0.999)) if rel.size else 0.0,
            "zero_mismatch": int(((r == 0) != (g == 0)).sum()),
            "floored_worst": float(floored.max()) * TOL, "values": int(r.size)}


def record(name, stats):
    path = os.environ.get("MPSS_PARITY_REPORT")
    if path:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "a") as f:
            f.write(json.dumps(dict(test=name, **stats)) + "\n")


def check_image(got, ref, name=None):
    assert np.array_equal(got[..., 3], ref[..., 3]), "film weights differ (sample-to-pixel mapping)"
    st = image_errors(got, ref)
    record(name or os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0], st)
    assert st["peak"] > 0
    assert st["zero_mismatch"] == 0, "%d values are zero on one side only" % st["zero_mismatch"]
    assert st["rel_linf"] <= TOL, "relative L-inf %g > %g" % (st["rel_linf"], TOL)
    return st
