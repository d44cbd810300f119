"""Node telemetry: the kubelet's AMD SMI collectors (native/gpu/smi.cc) on a synthetic
8x MI355X node, fed by a fixed gpu_metrics table (KFAMD_SMI_FAKE) instead of libamd_smi.

Checks: GFX / HBM-controller activity carry the pod that holds the device, per-link xGMI byte
counters, the held GFX clock, power, temperatures, energy, and the power/thermal throttle
residency computed from two samples' accumulators. The real-library path runs on the GPU box
(tests/test_gpu_telemetry.py)."""
import json
import time
import urllib.request

import pytest

NB = "kubeflow.org/v1"
BUSES = ["0000:%02x:00.0" % (0x05 + i * 0x10) for i in range(8)]  # GpuTopology::synthetic


def _table(acc, ppt, thm):
    return {"devices": [{"bdf": b, "gfx_activity": 90 + i, "umc_activity": 40 + i, "power_w": 1000 + i,
                         "temp_hotspot_c": 70 + i, "temp_mem_c": 60 + i, "gfxclk_mhz": 1700 + i,
                         "energy_j": 1e6 + i, "xgmi_read_bytes": [1024.0 * (i + 1)] * 7,
                         "xgmi_write_bytes": [2048.0 * (i + 1)] * 7, "accumulation_counter": acc,
                         "ppt_residency_acc": ppt, "thermal_residency_acc": thm} for i, b in enumerate(BUSES)]}


@pytest.fixture(scope="module")
def tele(tmp_path_factory):
    from tests.conftest import _ensure_native
    _ensure_native()
    from kubeflow_rm_amd.cluster import LocalCluster
    path = tmp_path_factory.mktemp("smi") / "gpu_metrics.json"
    path.write_text(json.dumps(_table(1000, 100, 0)))
    cl = LocalCluster(env={"ENABLE_CULLING": "false", "KFAMD_SMI_FAKE": str(path)})
    cl.start()
    yield cl, path
    cl.stop()


def _scrape(url):
    with urllib.request.urlopen(url + "/metrics", timeout=5) as r:
        return r.read().decode().splitlines()


def _series(lines, name):
    out = {}
    for line in lines:
        if line.startswith(name + "{"):
            labels = dict(kv.split("=", 1) for kv in line[len(name) + 1:line.index("}")].split(","))
            out[tuple(sorted((k, v.strip('"')) for k, v in labels.items()))] = float(line.split()[-1])
    return out


def test_telemetry_is_labelled_with_the_holding_pod(tele):
    cl, path = tele
    c = cl.client
    c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "tel"}})
    c.create({"apiVersion": NB, "kind": "Notebook", "metadata": {"name": "t2", "namespace": "tel"},
              "spec": {"template": {"spec": {"containers": [{"name": "t2", "image": "jupyter-scipy:latest",
                                                             "resources": {"limits": {"amd.com/gpu": "2"}}}]}}}})
    pod = c.wait_for("v1", "Pod", "t2-0", "tel", lambda o: "amd.com/gpu-ids" in o["metadata"].get("annotations", {}),
                     timeout=30)
    ids = set(pod["metadata"]["annotations"]["amd.com/gpu-ids"].split(","))
    lines = _scrape(cl.url)
    act = _series(lines, "kfamd_gpu_gfx_activity_percent")
    assert len(act) == 8
    held = {dict(k)["gpu"] for k in act if dict(k)["pod"] == "t2-0" and dict(k)["namespace"] == "tel"}
    assert held == ids
    for k, v in act.items():
        assert v == 90 + int(dict(k)["gpu"])
    hbm = _series(lines, "kfamd_gpu_hbm_activity_percent")
    assert {dict(k)["gpu"] for k in hbm if dict(k)["pod"] == "t2-0"} == ids
    clk = _series(lines, "kfamd_gpu_gfxclk_mhz")
    assert clk[(("gpu", "3"),)] == 1703
    assert _series(lines, "kfamd_gpu_power_watts")[(("gpu", "0"),)] == 1000
    temps = _series(lines, "kfamd_gpu_temperature_celsius")
    assert temps[(("gpu", "1"), ("sensor", "hbm"))] == 61 and temps[(("gpu", "1"), ("sensor", "hotspot"))] == 71
    rd = _series(lines, "kfamd_gpu_xgmi_read_bytes_total")
    wr = _series(lines, "kfamd_gpu_xgmi_write_bytes_total")
    assert len(rd) == 8 * 7 and rd[(("gpu", "2"), ("link", "6"))] == 3 * 1024
    assert wr[(("gpu", "0"), ("link", "0"))] == 2048
    assert any(line.startswith("# TYPE kfamd_gpu_xgmi_read_bytes_total counter") for line in lines)
    assert _series(lines, "kfamd_gpu_energy_joules_total")[(("gpu", "5"),)] == 1e6 + 5


def test_throttle_residency_from_two_samples(tele):
    cl, path = tele
    _scrape(cl.url)
    # 400 of the next 1000 accumulation ticks power-limited, 50 thermally limited
    path.write_text(json.dumps(_table(2000, 500, 50)))
    time.sleep(1.2)  # the kubelet samples AMD SMI at most once a second
    lines = _scrape(cl.url)
    thr = _series(lines, "kfamd_gpu_throttle_residency_ratio")
    assert thr[(("cause", "power"), ("gpu", "0"))] == pytest.approx(0.4)
    assert thr[(("cause", "thermal"), ("gpu", "7"))] == pytest.approx(0.05)
