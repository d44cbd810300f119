"""K6 depth: MI355X partition modes, NUMA-local CPU sets and pod pinning.

A fake sysfs tree stands in for /sys (KFD topology nodes, PCI functions, NUMA nodes), laid out as
the amdgpu driver exposes it: every compute partition is its own KFD node (CPX: one XCD = 32 CUs
= 128 SIMDs each), its mem_banks hold the memory partition it sits in (NPS2: half the package),
and the PCI function carries current_compute_partition / current_memory_partition /
local_cpulist / numa_node.
"""
import json
import os
import time
import urllib.request

import pytest

from kubeflow_rm_amd.cluster import LocalCluster

GIB = 1 << 30


def fake_sysfs(root, packages=8, compute="SPX", memory="NPS1", numa_nodes=2, cpus_per_numa=4):
    parts = {"SPX": 1, "DPX": 2, "QPX": 4, "CPX": 8}[compute]
    nps = int(memory[3:])
    kfd = os.path.join(root, "class/kfd/kfd/topology/nodes")
    for n in range(numa_nodes):
        d = os.path.join(kfd, str(n))
        os.makedirs(d)
        open(os.path.join(d, "properties"), "w").write("cpu_cores_count 4\nsimd_count 0\n")
        nd = os.path.join(root, "devices/system/node", f"node{n}")
        os.makedirs(nd)
        open(os.path.join(nd, "cpulist"), "w").write(f"{n * cpus_per_numa}-{(n + 1) * cpus_per_numa - 1}\n")
    gpu_nodes = []
    node = numa_nodes
    for p in range(packages):
        numa = p * numa_nodes // packages
        bus = 0x05 + p * 0x10
        bdf = f"0000:{bus:02x}:00.0"
        pdir = os.path.join(root, "bus/pci/devices", bdf)
        os.makedirs(pdir)
        open(os.path.join(pdir, "current_compute_partition"), "w").write(compute + "\n")
        open(os.path.join(pdir, "current_memory_partition"), "w").write(memory + "\n")
        open(os.path.join(pdir, "numa_node"), "w").write(f"{numa}\n")
        open(os.path.join(pdir, "local_cpulist"), "w").write(f"{numa * cpus_per_numa}-{(numa + 1) * cpus_per_numa - 1}\n")
        for _ in range(parts):
            d = os.path.join(kfd, str(node))
            os.makedirs(os.path.join(d, "mem_banks/0"))
            os.makedirs(os.path.join(d, "io_links"))
            open(os.path.join(d, "properties"), "w").write(
                f"simd_count {1024 // parts}\nnum_xcc {8 // parts}\ngfx_target_version 90500\n"
                f"location_id {bus << 8}\ndomain 0\ndrm_render_minor {128 + node}\n")
            open(os.path.join(d, "mem_banks/0/properties"), "w").write(f"size_in_bytes {288 * GIB // nps}\n")
            gpu_nodes.append((node, p, numa))
            node += 1
    for node, p, numa in gpu_nodes:
        links = os.path.join(kfd, str(node), "io_links")
        i = 0
        os.makedirs(os.path.join(links, str(i)))
        open(os.path.join(links, str(i), "properties"), "w").write(f"type 2\nnode_to {numa}\n")
        for other, q, _ in gpu_nodes:
            if q == p:
                continue
            i += 1
            os.makedirs(os.path.join(links, str(i)))
            open(os.path.join(links, str(i), "properties"), "w").write(f"type 11\nnode_to {other}\nmax_bandwidth 153000\n")
    return root


def test_cpulist_parse_and_format(native):
    r = native.call("cpulist_roundtrip", s="0-3,8,10-11\n")
    assert r["cpus"] == [0, 1, 2, 3, 8, 10, 11] and r["formatted"] == "0-3,8,10-11"


def test_discover_spx_nps1(native, tmp_path):
    t = native.call("topology_discover", sysfs_root=fake_sysfs(str(tmp_path)))
    gpus = t["gpus"]
    assert len(gpus) == 8 and t["source"] == "kfd-sysfs"
    assert {g["computePartition"] for g in gpus} == {"SPX"} and {g["memoryPartition"] for g in gpus} == {"NPS1"}
    assert all(g["hbmBytes"] == 288 * GIB for g in gpus)
    assert [g["numa"] for g in gpus] == [0, 0, 0, 0, 1, 1, 1, 1]
    assert gpus[0]["cpulist"] == "0-3" and gpus[7]["cpulist"] == "4-7"
    assert [g["physical"] for g in gpus] == list(range(8)) and all(g["xgmiDegree"] == 7 for g in gpus)
    assert t["localCpusDevice0"] == [0, 1, 2, 3]
    assert t["describe"] == "8x gfx950 full-mesh xGMI, 2 NUMA node(s)"


def test_discover_cpx_nps2(native, tmp_path):
    t = native.call("topology_discover", sysfs_root=fake_sysfs(str(tmp_path), packages=2, compute="CPX", memory="NPS2"))
    gpus = t["gpus"]
    # CPX: every XCD is a device -> 2 packages x 8 partitions
    assert len(gpus) == 16
    assert [g["physical"] for g in gpus] == [0] * 8 + [1] * 8
    assert [g["partition"] for g in gpus] == list(range(8)) * 2
    assert all(g["simdCount"] == 128 for g in gpus)
    # NPS2: each device addresses its 144 GiB memory partition and is charged 288/8 = 36 GiB
    assert all(g["hbmVisibleBytes"] == 144 * GIB and g["hbmBytes"] == 36 * GIB for g in gpus)
    assert "2 packages in CPX/NPS2" in t["describe"]


def _wait(cond, timeout=30):
    deadline = time.time() + timeout
    while time.time() < deadline:
        v = cond()
        if v:
            return v
        time.sleep(0.05)
    raise TimeoutError


@pytest.mark.skipif(len(os.sched_getaffinity(0)) < 8, reason="needs 8 schedulable CPUs")
def test_pod_env_exposes_only_the_allocated_gpus(native):
    """Device-plugin Allocate semantics for process pods: ROCr sees only the allocated GPUs (it would
    otherwise bring up and tear down every GPU of the node per process), HIP numbers them 0..n-1,
    the ring is in those pod-local ordinals and KFAMD_GPU_IDS keeps the node ids."""
    env = {e["name"]: e["value"] for e in native.call("gpu_env_for", gpus=8, devices=[5, 4])}
    assert env["ROCR_VISIBLE_DEVICES"] == "5,4"
    assert env["HIP_VISIBLE_DEVICES"] == "0,1"
    assert env["KFAMD_GPU_IDS"] == "5,4"
    assert sorted(env["KFAMD_XGMI_RING"].split(",")) == ["0", "1"]
    assert env["WORLD_SIZE"] == env["LOCAL_WORLD_SIZE"] == "2"
    one = {e["name"]: e["value"] for e in native.call("gpu_env_for", gpus=8, devices=[3])}
    assert one["ROCR_VISIBLE_DEVICES"] == "3" and one["HIP_VISIBLE_DEVICES"] == "0" and "WORLD_SIZE" not in one


def test_gpu_pod_pinned_to_numa_local_cpus_and_partition_hbm_quota(tmp_path):
    """e2e: a kubelet on the fake CPX/NPS2 node advertises 16 devices x 36 GiB, a 1-GPU notebook
    lands on package 1's NUMA node and runs on exactly that node's CPUs, and quota charges 36 GiB."""
    from tests.conftest import _ensure_native
    _ensure_native()
    root = fake_sysfs(str(tmp_path / "sys"), packages=2, compute="CPX", memory="NPS2")
    cl = LocalCluster(gpus=None, args=["--sysfs-root", root], env={"USE_ISTIO": "true"})
    cl.start()
    try:
        c = cl.client
        node = c.list("v1", "Node")["items"][0]
        assert node["status"]["capacity"]["amd.com/gpu"] == "16"
        assert node["status"]["capacity"]["amd.com/gpu-memory"] == str(16 * 36)
        labels = node["metadata"]["labels"]
        assert labels["amd.com/gpu.compute-partitioning-mode"] == "cpx"
        assert labels["amd.com/gpu.memory-partitioning-mode"] == "nps2"
        assert labels["amd.com/gpu.hbm-gib-per-device"] == "36"
        c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "pin", "labels": {"istio-injection": "enabled"}}})
        c.create({"apiVersion": "v1", "kind": "ResourceQuota", "metadata": {"name": "q", "namespace": "pin"},
                  "spec": {"hard": {"amd.com/gpu-memory": "1000"}}})
        # fill package 0 (8 partitions, NUMA 0) so the notebook lands on package 1 (NUMA 1)
        c.create({"apiVersion": "kubeflow.org/v1", "kind": "Notebook",
                  "metadata": {"name": "big", "namespace": "pin", "annotations": {"kfamd.io/gpu-readiness-op": "false"}},
                  "spec": {"template": {"spec": {"containers": [{"name": "big", "image": "jupyter-scipy:latest",
                                                                 "resources": {"limits": {"amd.com/gpu": "8"}}}]}}}})
        _wait(lambda: (c.get("kubeflow.org/v1", "Notebook", "big", "pin").get("status") or {}).get("readyReplicas") == 1)
        c.create({"apiVersion": "kubeflow.org/v1", "kind": "Notebook",
                  "metadata": {"name": "nb", "namespace": "pin", "annotations": {"kfamd.io/gpu-readiness-op": "false"}},
                  "spec": {"template": {"spec": {"containers": [{"name": "nb", "image": "jupyter-scipy:latest",
                                                                 "resources": {"limits": {"amd.com/gpu": "1"}}}]}}}})
        _wait(lambda: (c.get("kubeflow.org/v1", "Notebook", "nb", "pin").get("status") or {}).get("readyReplicas") == 1)
        pod = c.get("v1", "Pod", "nb-0", "pin")
        assert int(pod["metadata"]["annotations"]["amd.com/gpu-ids"]) >= 8  # package 1
        info = _wait(lambda: _gpu_info(cl.gateway, "pin", "nb"))
        assert info["KFAMD_CPU_AFFINITY"] == "4-7"
        assert info["cpus_allowed"] == [4, 5, 6, 7]
        q = _wait(lambda: (c.get("v1", "ResourceQuota", "q", "pin").get("status") or {}).get("used", {}).get("amd.com/gpu-memory") == "324"
                  and True)
        assert q
    finally:
        cl.stop()


def _gpu_info(gateway, ns, name):
    try:
        with urllib.request.urlopen(f"{gateway}/notebook/{ns}/{name}/api/gpu", timeout=3) as r:
            return json.loads(r.read())
    except Exception:
        return None
