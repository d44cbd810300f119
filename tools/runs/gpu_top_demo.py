#!/usr/bin/env python3
"""`kfctl top node|pod` on a real MI355X node: kube-lite with the discovered GPU(s), one torch-ready
notebook forked from the zygote, a GEMM load in it for a few seconds, and the top tables printed
while it runs (AMD SMI telemetry: activity, VRAM, power, clock, hotspot)."""
from __future__ import annotations

import os
import subprocess
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kubeflow_rm_amd.cluster import LocalCluster  # noqa: E402


def kfctl(url: str, *args: str) -> str:
    p = subprocess.run([sys.executable, "-m", "kubeflow_rm_amd.kfctl", *args, "--server", url],
                       capture_output=True, text=True, timeout=60)
    return p.stdout + p.stderr


def main() -> int:
    with LocalCluster(gpus=None, zygote=True) as cl:
        cl.wait_zygotes(timeout=300)
        c = cl.client
        c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "demo"}})
        c.create({"apiVersion": "kubeflow.org/v1", "kind": "Notebook", "metadata": {"name": "nb", "namespace": "demo"},
                  "spec": {"template": {"spec": {"containers": [{
                      "name": "nb", "image": "kfamd/jupyter-pytorch-rocm:latest",
                      "env": [{"name": "KFAMD_WARMUP", "value": "torch"}],
                      "resources": {"limits": {"amd.com/gpu": "1"}}}]}}}})
        c.wait_for("kubeflow.org/v1", "Notebook", "nb", "demo",
                   lambda o: (o.get("status") or {}).get("readyReplicas") == 1, timeout=120)
        print("== kfctl top node (notebook idle)")
        print(kfctl(cl.url, "top", "node"), flush=True)
        # a GEMM load on the same GPU from this process, so the telemetry has something to show
        import torch
        from kubeflow_rm_amd import ops
        a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
        b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
        stop = threading.Event()

        def load():
            while not stop.is_set():
                for _ in range(50):
                    ops.gemm_nt(a, b)
                torch.cuda.synchronize()
        t = threading.Thread(target=load)
        t.start()
        time.sleep(3)
        print("== kfctl top node (GEMM load on the GPU)")
        print(kfctl(cl.url, "top", "node"), flush=True)
        print("== kfctl top pod -A")
        print(kfctl(cl.url, "top", "pod", "-A"), flush=True)
        stop.set()
        t.join()
        c.delete("kubeflow.org/v1", "Notebook", "nb", "demo")
    return 0


if __name__ == "__main__":
    sys.exit(main())
