"""On-disk point clouds (row f4): the "pointsfile" of MultipoleSubsurfaceIntegrator.

The reference writes raw SurfacePoint records, 44 bytes each in native order
(TessellateSurfacePointsRenderer, surfacepoints.cpp:335-347: fwrite of points[]), and reads them
back with ReadBinaryFile<SurfacePoint> (floatfile.h:46-64: size / sizeof(T) records; a trailing
partial record is ignored). Checked here: the saved file is exactly the context's records, a
second context that loads it (the scene's "pointsfile" parameter) holds the same records, and its
Preprocess + render produce bit-identical irradiance and film to the context that tessellated.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _scene():
    from mpss import pbrtscene
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin.pbrt"), xres=32, yres=32, spp=2)
    sc.integrator["minsampledistance"] = 0.01
    for m in sc.materials:
        m["desired_length"] = 64
    return sc


def _render(torch, ctx, sc):
    out = torch.zeros((sc.xres * sc.yres * 4,), dtype=torch.float32, device="cuda")
    ctx.render_tile(sc.spp, 5, 0, sc.xres, 0, sc.yres, out.data_ptr())
    torch.cuda.synchronize()
    return out.cpu().numpy()


def test_pointsfile_round_trip(mpss, tmp_path):
    import torch
    assert torch.cuda.is_available()
    from mpss import pbrtscene
    sc = _scene()
    a = pbrtscene.build_context(sc)
    a.preprocess(seed=3)
    pts = a.surface_points()
    path = str(tmp_path / "head.points")
    a.save_pointsfile(path)
    raw = open(path, "rb").read()
    assert len(raw) == 44 * len(pts) and mpss.SURFACE_POINT.itemsize == 44
    assert raw == pts.tobytes()
    assert np.array_equal(np.fromfile(path, mpss.SURFACE_POINT), pts)

    sc.integrator["pointsfile"] = path  # the integrator reads instead of tessellating
    b = pbrtscene.build_context(sc)
    assert b.surface_points().tobytes() == raw
    b.preprocess(seed=3)
    assert np.array_equal(b.irradiance(), a.irradiance())
    assert np.array_equal(_render(torch, b, sc), _render(torch, a, sc))
    a.close()
    b.close()


def test_pointsfile_partial_record_and_foreign_writer(mpss, tmp_path):
    """A file written by other code (numpy here) with a trailing partial record: ReadBinaryFile
    keeps size / 44 whole records."""
    import torch
    assert torch.cuda.is_available()
    from mpss import pbrtscene
    sc = _scene()
    recs = pbrtscene.mesh_points(sc)
    path = str(tmp_path / "foreign.points")
    with open(path, "wb") as f:
        f.write(recs.tobytes() + b"\x01" * 17)
    ctx = pbrtscene.build_context(sc)
    ctx.load_pointsfile(path)
    assert ctx.surface_points().tobytes() == recs.tobytes()
    with pytest.raises(mpss.MpssError):
        ctx.load_pointsfile(str(tmp_path / "missing.points"))
    ctx.close()
