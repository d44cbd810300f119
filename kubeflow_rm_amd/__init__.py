"""kubeflow_rm_amd — an MI355X-native notebook control plane and in-pod compute stack.

Layers (re-designed MI355X-first):

* ``native/`` (C++17)  — kube-lite API server, controller runtime, the Notebook / Culling / ODH /
  Profile / Tensorboard / PVCViewer reconcilers, admission webhooks, KFAM, the local kubelet with
  xGMI-topology-aware GPU placement and HBM quota, and the in-pod readiness op.
* ``kernels/`` (HIP, gfx950) — hand-written CDNA4 kernels (MFMA bf16 GEMM, LayerNorm/RMSNorm).
* ``kubeflow_rm_amd.ops`` — torch-facing wrappers of those kernels (ctypes, in-tree .so).
* ``kubeflow_rm_amd.parallel`` — DP/TP wiring over RCCL (torch.distributed "nccl" on ROCm).
* ``kubeflow_rm_amd.models`` — CRD object models + the small transformer used by the DP/TP examples.
* ``kubeflow_rm_amd.webapps`` — Jupyter/TensorBoards/Volumes backends and the dashboard (Flask).
* ``kubeflow_rm_amd.client`` / ``cli`` — thin Kubernetes REST client and the ``kfctl`` CLI.
"""
__version__ = "0.1.0"
