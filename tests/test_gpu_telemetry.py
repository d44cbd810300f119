"""AMD SMI telemetry on a real MI355X (native/gpu/smi.cc through the C ABI): the sample the kubelet's
collectors export matches the KFD topology's PCI addresses, and a GEMM burst shows up as GFX
activity, a held clock and spent energy (tests/test_e2e_telemetry.py covers the collectors)."""
import time

import pytest

pytestmark = pytest.mark.gpu


def test_smi_sample_matches_topology_and_sees_load():
    import torch
    from kubeflow_rm_amd import native, ops
    s0 = native.call("smi_sample")
    assert s0["available"], s0["error"]
    assert s0["devices"], s0
    buses = set(s0["topology_buses"])
    mine = [d for d in s0["devices"] if d["bdf"] in buses]
    assert mine, (s0["devices"], buses)
    d0 = mine[0]
    assert 0 < d0["power_w"] < 2000 and 0 < d0["temp_hotspot_c"] < 120
    a = (torch.rand(8192, 8192, device="cuda") * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(8192, 8192, device="cuda") * 2 - 1).to(torch.bfloat16)
    c = torch.empty_like(a)
    t_end = time.time() + 1.5
    while time.time() < t_end:
        for _ in range(50):
            ops.gemm_nt(a, b, out=c)
        torch.cuda.synchronize()
        s1 = native.call("smi_sample")
    d1 = next(d for d in s1["devices"] if d["bdf"] == d0["bdf"])
    print("idle:", d0, "\nload:", d1)
    assert d1["gfx_activity"] > 50, d1
    assert 500 < d1["gfxclk_mhz"] <= 2500, d1
    if d0["energy_j"] >= 0:
        assert d1["energy_j"] > d0["energy_j"]
