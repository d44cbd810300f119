"""The node's comgr seed (native/node/kubelet.cc seed_comgr_cache / link_comgr_seed).

A GPU container's code-object cache is per namespace (AMD_COMGR_CACHE_DIR=<root>/gpu-cache/comgr/<ns>):
tenants never share writable code objects. The kubelet builds RCCL's comgr entries once per host
with its own readiness op (GPU nodes only) and a namespace's NEW cache starts as reflink (copy-on-write)
copies of the completed seed's llvmcache-* entries, or read-only hard links where the filesystem has
no reflinks, so the first RCCL communicator in a namespace does
not pay the 3.8 s build (profiles/r6k_rccl_init). Here a completed seed is prepared by hand
(KFAMD_COMGR_SEED_DIR) on a synthetic-GPU node; the build itself needs a GPU.
"""
import os
import time

import pytest

from kubeflow_rm_amd.cluster import LocalCluster

_PROG = r"""
import os, sys, time
d = os.environ.get("AMD_COMGR_CACHE_DIR", "")
print("CACHE=" + d, flush=True)
print("FILES=" + ",".join(sorted(os.listdir(d))) if d else "FILES=", flush=True)
time.sleep(3600)
"""


def _pod(name, ns, gpus=1):
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": ns},
            "spec": {"containers": [{"name": "c", "image": "jupyter-pytorch-rocm:latest",
                                     "command": ["python3", "-c", _PROG],
                                     "resources": {"limits": {"amd.com/gpu": str(gpus)}}}]}}


def _wait_logs(c, name, ns, key, timeout=60):
    deadline = time.time() + timeout
    while time.time() < deadline:
        try:
            logs = c.pod_logs(name, ns) or ""
        except Exception:
            logs = ""
        vals = dict(ln.split("=", 1) for ln in logs.splitlines() if "=" in ln and ln.split("=", 1)[0] in ("CACHE", "FILES"))
        if key in vals:
            return vals
        time.sleep(0.2)
    pytest.fail(f"{ns}/{name}: no {key} in the logs")


def test_new_namespace_cache_starts_from_the_completed_seed(tmp_path):
    seed = tmp_path / "comgr-seed"
    seed.mkdir()
    (seed / "llvmcache-aaa").write_bytes(b"entry-a")
    (seed / "llvmcache-bbb").write_bytes(b"entry-b")
    (seed / "unrelated.tmp").write_text("not a cache entry")
    (seed / ".complete").write_text("1\n")
    with LocalCluster(gpus=2, env={"KFAMD_COMGR_SEED_DIR": str(seed)}) as cl:
        c = cl.client
        for ns in ("seed-a", "seed-b"):
            c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": ns}})
        c.create(_pod("p1", "seed-a"))
        got = _wait_logs(c, "p1", "seed-a", "FILES")
        cache = got["CACHE"]
        assert cache.endswith("/gpu-cache/comgr/seed-a"), cache
        assert got["FILES"].split(",") == ["llvmcache-aaa", "llvmcache-bbb"], got
        # reflink copies (own inode: a rewrite stays in this namespace) or, without reflinks,
        # read-only hard links to the seed's entries
        for n, body in (("llvmcache-aaa", b"entry-a"), ("llvmcache-bbb", b"entry-b")):
            ns_path = os.path.join(cache, n)
            st_seed, st_ns = os.stat(seed / n), os.stat(ns_path)
            assert open(ns_path, "rb").read() == body
            if (st_seed.st_ino, st_seed.st_dev) == (st_ns.st_ino, st_ns.st_dev):
                assert not st_ns.st_mode & 0o222
            else:
                with open(ns_path, "wb") as f:
                    f.write(b"rewritten-in-a")
                assert (seed / n).read_bytes() == body
        # another tenant's namespace gets its own directory (same read-only entries, no shared dir)
        c.create(_pod("p2", "seed-b"))
        got_b = _wait_logs(c, "p2", "seed-b", "FILES")
        assert got_b["CACHE"].endswith("/gpu-cache/comgr/seed-b") and got_b["CACHE"] != cache
        # an entry the tenant's pods add stays in that namespace's cache
        with open(os.path.join(cache, "llvmcache-ccc"), "wb") as f:
            f.write(b"tenant-a")
        assert not (seed / "llvmcache-ccc").exists()
        assert not os.path.exists(os.path.join(got_b["CACHE"], "llvmcache-ccc"))


def test_incomplete_seed_is_not_linked(tmp_path):
    seed = tmp_path / "comgr-seed"
    seed.mkdir()
    (seed / "llvmcache-aaa").write_bytes(b"half-built")  # no .complete marker
    with LocalCluster(gpus=1, env={"KFAMD_COMGR_SEED_DIR": str(seed)}) as cl:
        c = cl.client
        c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "seed-c"}})
        c.create(_pod("p", "seed-c"))
        got = _wait_logs(c, "p", "seed-c", "FILES")
        assert got["CACHE"].endswith("/gpu-cache/comgr/seed-c") and got["FILES"] == "", got
