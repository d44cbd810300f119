"""Pod addresses (native/node/kubelet.cc Kubelet::admit): each kubelet starts at a random point of
its /16, so two kubelets started one after the other on a host (test clusters, the bench's
cold-start variants) do not hand out the same address while a process of the first may still hold
it (profiles/r6y_final run 3); x.y.z.0 and .255 are never used. LocalCluster also picks a random
/16 per cluster; here both clusters get the same one, so only the kubelet's own offset separates
them."""
import ipaddress
import time

from kubeflow_rm_amd.cluster import LocalCluster


def _pod(name):
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default"},
            "spec": {"containers": [{"name": "c", "image": "busybox",
                                     "command": ["python3", "-c", "import time; time.sleep(3600)"]}]}}


def _pod_ips(cl, names, timeout=30):
    deadline = time.time() + timeout
    ips = {}
    while time.time() < deadline and len(ips) < len(names):
        for n in names:
            ip = (cl.client.get("v1", "Pod", n, "default").get("status") or {}).get("podIP")
            if ip:
                ips[n] = ip
        time.sleep(0.1)
    assert len(ips) == len(names), ips
    return ips


def test_pod_addresses_differ_between_kubelets_and_skip_network_octets():
    seen = []
    for _ in range(2):
        with LocalCluster(args=["--pod-cidr-prefix", "127.20"]) as cl:
            names = [f"p{i}" for i in range(3)]
            for n in names:
                cl.client.create(_pod(n))
            ips = _pod_ips(cl, names)
        assert len(set(ips.values())) == 3, ips  # unique within a kubelet
        for ip in ips.values():
            a = ipaddress.ip_address(ip)
            assert a in ipaddress.ip_network("127.20.0.0/16") and ip.split(".")[3] not in ("0", "255"), ip
        seen.append(set(ips.values()))
    # two kubelets in a row: the second does not start from the first one's addresses (a collision of
    # random starting points within three addresses has odds of about 1 in 10,000)
    assert not seen[0] & seen[1], seen
