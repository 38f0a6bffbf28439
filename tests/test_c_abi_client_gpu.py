"""The Level-B drop-in exercised by a compiled C++ program, not Python.

tests/c_abi/client.cpp includes include/mpss.h, links libmpss.so with g++ (tests/c_abi/Makefile,
built by __graft_entry__.build()), builds skin.pbrt through the C entry points, runs Preprocess, calls
mpss_mo_batch from 8 pthreads on 8 hipStream_ts at once (pbrt's concurrent Li, integrator.h:51-72,
parallel.cpp:800-878) in the sharded and the reference-order gathers, renders one C2 window with
mpss_render_tile and checks the error convention. Here: its exit status, the window bit for bit
against the Python binding's render of the same window, and its reference-order Mo() against the
oracle's recursion (diffusionutil.h:175-210) bit for bit.
"""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLIENT = os.path.join(ROOT, "tests", "c_abi", "client")


def _client():
    src = os.path.join(ROOT, "tests", "c_abi", "client.cpp")
    lib = os.path.join(ROOT, "pbrt-v2-skin_amd", "mpss", "libmpss.so")
    if not os.path.exists(CLIENT) or os.path.getmtime(CLIENT) < max(os.path.getmtime(src), os.path.getmtime(lib)):
        subprocess.run(["make", "-s", "-C", os.path.dirname(CLIENT)], check=True, timeout=300)
    return CLIENT


def _write_scene(sc, d, mpss):
    """skin.pbrt as the loader parsed it, in the client's input files (the ABI's own struct layouts)."""
    from mpss import pbrtscene
    cfg = mpss.default_config(**pbrtscene.integrator_config(sc))
    m = sc.materials[0]
    kw = {k: v for k, v in m.items() if k not in ("Kr", "Kt", "albedo", "albedo_tex", "bump_tex")}
    for k in ("Kr", "Kt", "albedo"):
        if k in m:
            kw[k] = mpss.host_from_rgb(m[k])
    skin = mpss.default_skin(**kw)
    assert len(sc.meshes) == 1 and len(sc.lights) == 1 and not sc.meshes[0]["reverse"]
    me, li = sc.meshes[0], sc.lights[0]
    files = {"config.bin": bytes(cfg), "skin.bin": bytes(skin)}
    for k in ("P", "N", "S", "uv"):
        files[k + ".f32"] = b"" if me.get(k) is None else np.ascontiguousarray(me[k], np.float32).tobytes()
    files["indices.i32"] = np.ascontiguousarray(me["indices"], np.int32).tobytes()
    files["o2w.f32"] = np.ascontiguousarray(me["o2w"], np.float32).tobytes()
    files["w2o.f32"] = np.ascontiguousarray(me["w2o"], np.float32).tobytes()
    r2c, c2w = sc.raster_to_camera()
    files["raster_to_camera.f32"] = np.ascontiguousarray(r2c, np.float32).tobytes()
    files["camera_to_world.f32"] = np.ascontiguousarray(c2w, np.float32).tobytes()
    files["res.i32"] = np.int32([sc.xres, sc.yres]).tobytes()
    files["light.f32"] = np.concatenate([np.float32(li["center"]), np.float32([li["radius"]]),
                                         mpss.host_from_rgb(li["L"]), np.float32([li["nsamples"]])]).tobytes()
    for name, data in files.items():
        with open(os.path.join(d, name), "wb") as f:
            f.write(data)


def test_compiled_client_threads_streams_and_window(mpss, oracle, tmp_path):
    import torch
    from mpss import pbrtscene
    import oracle_lib
    assert torch.cuda.is_available()
    client = _client()
    sc = pbrtscene.load(os.path.join(ROOT, "scenes", "skin.pbrt"))
    scene_dir, out_dir = tmp_path / "scene", tmp_path / "out"
    scene_dir.mkdir()
    out_dir.mkdir()
    _write_scene(sc, str(scene_dir), mpss)
    # the Python binding's context of the same scene: the window to render, and the reference image
    ctx = pbrtscene.build_context(sc)
    ctx.preprocess(seed=1)
    W, H, w = sc.xres, sc.yres, 32
    rects = [(x, x + w, y, y + w) for y in range(0, H - w + 1, w) for x in range(0, W - w + 1, w)]
    sss, _ = ctx.tile_costs(rects)
    x0, x1, y0, y1 = min((abs((r[0] + r[1]) / 2 - W / 2) + abs((r[2] + r[3]) / 2 - H / 2), r)
                         for r, n in zip(rects, sss) if n == w * w)[1]
    nq = 200_000
    run = subprocess.run([client, str(scene_dir), str(out_dir), str(x0), str(x1), str(y0), str(y1), str(sc.spp), "7",
                          str(nq)], capture_output=True, text=True, timeout=600)
    print(run.stdout, run.stderr)
    assert run.returncode == 0, run.stdout + run.stderr
    assert "8 threads on 8 streams == the serial call" in run.stdout

    # the window, bit for bit as the Python path renders it
    tile = np.fromfile(out_dir / "tile.f32", np.float32).reshape(y1 - y0, x1 - x0, 4)
    out = torch.zeros(((y1 - y0) * (x1 - x0) * 4,), dtype=torch.float32, device="cuda")
    ctx.render_tile(sc.spp, 7, x0, x1, y0, y1, out.data_ptr())
    torch.cuda.synchronize()
    ref = out.cpu().numpy().reshape(y1 - y0, x1 - x0, 4)
    assert np.array_equal(tile, ref)
    assert (ref[..., 1] > 0).all()

    # the client's reference-order Mo() against the oracle's recursion on the same octree
    pts = np.fromfile(out_dir / "points.f32", np.float32).reshape(-1, 3)
    mo = np.fromfile(out_dir / "mo_exact.f32", np.float32).reshape(-1, 30)
    assert len(pts) == nq and len(mo) == nq
    sp = ctx.surface_points()
    assert np.array_equal(pts, sp["p"][:nq])
    tab, rcp, _, _ = ctx.material_tables(0)
    E = ctx.irradiance()
    t = oracle_lib.Octree(np.ascontiguousarray(sp["p"]), np.ascontiguousarray(sp["n"]), E,
                          np.ascontiguousarray(sp["area"]))
    k = 3000
    ref_mo = t.mo(np.ascontiguousarray(pts[:k]), tab, rcp, float(sc.integrator["maxerror"]))
    assert np.array_equal(mo[:k], ref_mo)
    assert (ref_mo > 0).mean() > 0.5
    ctx.close()
