"""BASELINE configs 4 and 5 as bench.py measures them (VERDICT r5 missing #5), on CPU with 8
synthetic MI355X: one Notebook holds all 8 GPUs and carries the in-pod RCCL smoke request, then a
TensorBoard and a PVCViewer attach to ITS ReadWriteOnce workspace PVC and land on its node through
the RWO affinity (tensorboard_controller.go:207-231, pvcviewer_controller.go:372-445). On a GPU box
the same function fills the config4_rccl_* keys from the pod's readiness report (tests/test_gpu_rccl.py)."""
from tests.conftest import _ensure_native


def test_config4_and_5_on_one_eight_gpu_notebook():
    _ensure_native()
    from kubeflow_rm_amd.bench_coldstart import measure_gpu_notebook_configs
    r = measure_gpu_notebook_configs(gpus_per_notebook=8, gpus=8, timeout=60)
    assert r["config4_readiness_args"] == "--rccl"
    assert r["config4_gpu_ids"] == "0,1,2,3,4,5,6,7" and r["config4_gpus"] == 8 and r["config4_ready_s"] < 30
    assert r["config5_pvc"] == "cfg-nb-workspace"
    assert r["config5_coscheduled"] is True, r
    assert r["config5_tensorboard_ready_s"] < 30 and r["config5_pvcviewer_ready_s"] < 30
