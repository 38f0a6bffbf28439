"""The C-ABI library loads and exports every symbol include/mpss.h declares (CPU-only)."""
import os
import subprocess

import pytest


def test_library_exports_header_symbols(mpss):
    declared = mpss.exported_symbols()
    assert "mpss_mo_batch" in declared and "mpss_create" in declared
    out = subprocess.run(["nm", "-D", "--defined-only", mpss.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [s for s in declared if s not in exported]
    assert not missing, missing


def test_abi_version_and_errors(mpss):
    assert mpss.lib().mpss_abi_version() == 13
    # a null-argument call must fail with a message, not crash
    rc = mpss.lib().mpss_create(None, None)
    assert rc == -1
    assert b"null" in mpss.lib().mpss_last_error()


def test_defaults_match_reference_factories(mpss):
    c = mpss.default_config()
    # CreateMultipoleSubsurfaceIntegrator, multipolesubsurface.cpp (file) 393-400
    assert (c.max_depth, round(c.max_error, 6), round(c.min_sample_distance, 6), round(c.mix, 6)) == \
        (5, 0.05, 0.25, 0.5)
    # the sharded gather's choices (none changes a result bit; tests/test_mo_gpu.py)
    assert (c.mo_band_dealing, c.mo_work_stealing, c.mo_near_field) == (0, 1, 5088)
    assert c.mo_common_grid == 1  # the far field from the resampled group tables (within its checked bound)
    assert (c.octree_on_host, c.tessellate_on_host, c.profile_on_host) == (0, 0, 0)  # Preprocess on the GPU
    m = mpss.default_skin()
    # CreateLayeredSkinMaterial, layeredskin.cpp:234-257
    assert round(m.roughness, 6) == 0.4 and m.nmperunit == pytest.approx(100e6)
    assert m.desired_length == 512 and m.lerp_on_thin_slab == 1 and m.double_ref_sslf == 0
    assert list(m.albedo) == [1.0] * 30 and list(m.Kr) == [1.0] * 30 and list(m.Kt) == [1.0] * 30


def test_header_has_no_torch_types():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    txt = open(os.path.join(root, "include", "mpss.h")).read()
    code = txt.split("*/", 1)[1]  # declarations after the header comment
    assert "torch" not in code
    assert "hipStream_t" not in code and "std::" not in code
