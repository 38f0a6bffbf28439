"""The image parity criterion of the GPU tests, and the report of the error they actually reach.

check_image(got, ref, name): film weights bit-exact (the sample-to-pixel mapping), XYZ within
TOL = 1e-4 relative per pixel with a floor at 1e-3 of the window's peak (pixels far below the
peak carry few samples, where a float reassociation of the Mo() sum is a larger fraction of the
pixel). It also computes the UNFLOORED relative L-inf, max |gpu - cpu| / |cpu| over every
channel value with cpu != 0 (and counts values that are 0 on one side only), and appends it,
with the floored figure, to the JSONL file named by $MPSS_PARITY_REPORT (tools/gpu.sh sets it).
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
    return {"peak": peak, "rel_linf": float(rel.max()) if rel.size else 0.0,
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
    assert st["floored_worst"] <= TOL, "max |gpu-cpu| / bound = %g" % (st["floored_worst"] / TOL)
    return st
