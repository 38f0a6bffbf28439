"""rho_hd table on the GPU (row f1; reference src/core/multipole.cpp:488-549): one MT19937 stream
per entry twisted in LDS, terms Kahan-summed in sample order by one lane, so the table is the
oracle's bit for bit (both follow the double-then-round transcendental convention; only a
double-rounding tie of OCML vs glibc could move a term, and then by one ulp). The material build
uses it by default; the time per material build is reported."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rough,eta,fixed", [(0.3, 1.4, False), (0.35, 1.33, False), (0.0005, 1.4, False),
                                             (0.3, 1.4, True)])
def test_gpu_rho_table_vs_host_and_oracle(mpss, oracle, rough, eta, fixed):
    import torch
    assert torch.cuda.is_available()
    skin = mpss.default_skin(roughness=rough, layer_ior=(eta, 1.4), desired_length=16, double_ref_sslf=int(fixed))
    ctx = mpss.Context()
    t0 = time.perf_counter()
    mid = ctx.add_layeredskin(skin)
    dt = time.perf_counter() - t0
    _, _, rho, _ = ctx.material_tables(mid)
    ctx.close()
    host, _ = mpss.host_rho_table(rough, eta, double_ref_sslf=fixed)
    ulps = np.abs(rho.view(np.int32).astype(np.int64) - host.view(np.int32).astype(np.int64))
    assert ulps.max() <= 1 and (ulps == 0).mean() >= 0.999, (ulps.max(), (ulps != 0).sum())
    ref, _ = oracle.rho_table(rough, eta, fixed=fixed)  # FresnelDielectric, or FixedFresnelDielectric
    assert np.array_equal(host, ref)
    print("material build (profile 16 + rho 1025 x 256^2 on the GPU): %.3f s" % dt)
