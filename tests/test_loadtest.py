"""Load test (start_notebooks.py parity) + reconcile-latency histograms.

Reference: components/notebook-controller/loadtest/start_notebooks.py:50-96 (objects and names),
jupyter_test.yaml / jupyter_pvc.yaml (500m / 1Gi, 2Gi RWO claim). The reference records no timing;
the measure mode here is what BASELINE.md §3 asks for (reconcile latency p50/p99).
"""
import math

from kubeflow_rm_amd import loadtest as lt


def test_objects_match_reference_shapes():
    nb = lt.notebook_config(7, "kubeflow")
    assert nb["metadata"]["name"] == "jupyter-test-7"
    spec = nb["spec"]["template"]["spec"]
    assert spec["containers"][0]["name"] == "notebook-7"
    assert spec["containers"][0]["resources"]["requests"] == {"cpu": "500m", "memory": "1Gi"}
    assert spec["volumes"][0]["persistentVolumeClaim"]["claimName"] == "test-vol-7"
    assert spec["volumes"][1] == {"name": "dshm", "emptyDir": {"medium": "Memory"}}
    pvc = lt.pvc_config(7, "kubeflow")
    assert pvc["metadata"]["name"] == "test-vol-7"
    assert pvc["spec"]["resources"]["requests"]["storage"] == "2Gi"
    gpu = lt.notebook_config(1, "kubeflow", gpus=8)
    assert gpu["spec"]["template"]["spec"]["containers"][0]["resources"]["limits"] == {"amd.com/gpu": "8"}


def test_histogram_quantile_matches_promql():
    text = "\n".join([
        '# TYPE x histogram',
        'x_bucket{controller="a",le="0.1"} 0',
        'x_bucket{controller="a",le="0.2"} 50',
        'x_bucket{controller="a",le="0.4"} 100',
        'x_bucket{controller="a",le="+Inf"} 100',
        'x_sum{controller="a"} 20',
        'x_count{controller="a"} 100',
    ])
    h = lt.parse_histograms(text, "x")[(("controller", "a"),)]
    assert h["count"] == 100 and h["sum"] == 20
    assert math.isclose(lt.histogram_quantile(0.5, h["buckets"]), 0.2)
    assert math.isclose(lt.histogram_quantile(0.25, h["buckets"]), 0.15)
    assert math.isclose(lt.histogram_quantile(0.99, h["buckets"]), 0.2 + 0.2 * 49 / 50)


def test_measure_small_load():
    res = lt.measure(n=6, concurrency=3, timeout=60)
    assert res["ready"] == 6, res
    m = res["metrics"]
    rec = m["controller_runtime_reconcile_time_seconds"]["notebook-controller"]
    assert rec["count"] >= 6 and rec["p50_ms"] <= rec["p99_ms"]
    q = m["workqueue_queue_duration_seconds"]["notebook-controller"]
    assert q["count"] >= 6
    assert res["create_to_ready_p50_s"] < 30


def test_apiserver_bench_runs():
    """native/cmd/apiserver-bench.cc: in-process storage path (admission -> commit -> WAL -> watch fan-out)."""
    import json
    import subprocess
    from pathlib import Path
    exe = Path(lt.__file__).resolve().parent / "bin" / "apiserver-bench"
    out = subprocess.run([str(exe), "--pods", "50", "--updates", "200", "--watchers", "3"], capture_output=True,
                         text=True, timeout=60, check=True).stdout
    d = json.loads(out.strip().splitlines()[-1])
    assert d["create"]["n"] == 50 and d["update_status"]["n"] == 200
    assert d["watch_events_delivered"] == 3 * 250  # every create + update reaches every watcher
