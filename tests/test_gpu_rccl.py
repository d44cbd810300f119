"""The torch / RCCL process-group path executed on one GPU.

A one-GPU box cannot measure a scaling curve, but it can run every line of the multi-GPU code:
``parallel.dist.init`` through ``init_process_group("nccl", device_id=...)`` at WORLD_SIZE=1
(``KFAMD_FORCE_DIST=1``), device barriers, RCCL all-reduce / all-gather / broadcast /
reduce-scatter, the bucketed backward-overlapped DP all-reduce, the TP forward with its RCCL
all-reduces, the sweep that bench.py reports, the readiness op's ``--rccl-single`` stage and
``bench.py --force-dist`` under ``torch.distributed.run --nproc-per-node 1``. At world size 1 every
collective's result is its input, so each check is exact.

The reference's multi-GPU contract is the spawner's GPU counts 1/2/4/8
(/root/reference/components/crud-web-apps/jupyter/frontend/src/app/pages/form/form-new/form-gpus/form-gpus.component.ts:20-21)
with the /dev/shm volume (/root/reference/components/crud-web-apps/jupyter/backend/apps/common/form.py:264-276).
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def nccl_env():
    """One RCCL process group at world size 1 for the module (init once, destroy at the end)."""
    import torch.distributed as dist
    from kubeflow_rm_amd.parallel import dist as kd
    saved = {k: os.environ.get(k) for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
                                            "KFAMD_FORCE_DIST")}
    os.environ.update({"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(_port()), "KFAMD_FORCE_DIST": "1"})
    kd.shutdown()
    env = kd.init(backend="nccl", timeout_s=120)
    try:
        yield env
    finally:
        kd.shutdown()
        assert not dist.is_initialized()
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_init_creates_an_rccl_process_group_at_world_one(nccl_env):
    import torch.distributed as dist
    from kubeflow_rm_amd.parallel import dist as kd
    assert dist.is_initialized() and dist.get_backend() == "nccl"
    assert dist.get_world_size() == 1 and dist.get_rank() == 0
    assert nccl_env.backend == "nccl" and nccl_env.device.type == "cuda"
    kd.barrier()  # dist.barrier(device_ids=[...]) on the RCCL group
    dist.barrier(device_ids=[nccl_env.device.index])
    torch.cuda.synchronize()


def test_rccl_collectives_execute_and_are_exact(nccl_env):
    import torch.distributed as dist
    dev = nccl_env.device
    for dtype in (torch.float32, torch.bfloat16):
        x = torch.randn(1 << 20, device=dev).to(dtype)
        ref = x.clone()
        dist.all_reduce(x)
        assert torch.equal(x, ref)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        assert torch.equal(x, ref)
        out = torch.empty_like(x)
        dist.all_gather_into_tensor(out, x)
        assert torch.equal(out, ref)
        rs = torch.empty_like(x)
        dist.reduce_scatter_tensor(rs, x)
        assert torch.equal(rs, ref)
        dist.broadcast(x, src=0)
        assert torch.equal(x, ref)
    # async work objects, as the DP bucketer uses them
    y = torch.arange(4096, device=dev, dtype=torch.float32)
    w = dist.all_reduce(y, async_op=True)
    w.wait()
    torch.cuda.synchronize()
    assert torch.equal(y.cpu(), torch.arange(4096, dtype=torch.float32))


def test_allreduce_sweep_calls_rccl_at_world_one(nccl_env):
    from kubeflow_rm_amd.parallel.collectives import allreduce_sweep
    sw = allreduce_sweep(max_bytes=64 << 20, min_bytes=8, step=8, iters_small=5, iters_large=3,
                         dtype=torch.bfloat16, device=nccl_env.device)
    assert [r["bytes"] for r in sw] == [8 << (3 * i) for i in range(len(sw))] and sw[-1]["bytes"] == 16 << 20
    # every size launched RCCL work: a measurable time and a finite algbw (busbw is 0 at n = 1)
    assert all(r["us"] > 0 and r["algbw_GBps"] > 0 and r["busbw_GBps"] == 0 for r in sw), sw


def _tiny_gpt(dev, tp_group=None):
    from kubeflow_rm_amd.models import GPT, GPTConfig
    cfg = GPTConfig(vocab_size=512, d_model=256, n_layers=2, n_heads=4, d_ff=1024, max_seq=128)
    torch.manual_seed(0)
    return GPT(cfg, tp_group=tp_group, device=dev)


def test_dp_bucketed_allreduce_over_rccl_matches_plain_step(nccl_env):
    """One DP train step (bucketed, backward-overlapped RCCL all-reduces) against the same step
    without DP: at world size 1 the reduced gradients are the local ones, bit for bit."""
    from kubeflow_rm_amd import parallel
    dev = nccl_env.device
    idx = torch.randint(0, 512, (2, 128), generator=torch.Generator().manual_seed(1)).to(dev)
    tgt = torch.randint(0, 512, (2, 128), generator=torch.Generator().manual_seed(2)).to(dev)
    ref = _tiny_gpt(dev)
    ref(idx, tgt)[1].backward()
    model = _tiny_gpt(dev)
    dp = parallel.DataParallel(model, bucket_mb=0.25)  # several buckets: several async all-reduces
    assert dp.bucketer.active and len(dp.bucketer.buckets) > 2
    for _ in range(2):  # twice: bucket state resets between steps
        model.zero_grad(set_to_none=True)
        dp(idx, tgt)[1].backward()
        torch.cuda.synchronize()
        nb = len(dp.bucketer.buckets)
        assert dp.bucketer.last_launch_order == list(range(nb))
    assert dp.bucketer.comm_bytes > 0
    for (n, p), (_, q) in zip(model.named_parameters(), ref.named_parameters()):
        assert p.grad is not None and torch.equal(p.grad, q.grad), n


def test_tp_forward_backward_over_rccl_group(nccl_env):
    """The TP model on the RCCL group (KFAMD_FORCE_DIST: its all-reduces run at size 1) against the
    plain model: the row-parallel layers take the un-fused bias/residual path, so bf16 rounding
    differs slightly; the loss and the gradients agree to bf16 tolerance."""
    import torch.distributed as dist
    dev = nccl_env.device
    idx = torch.randint(0, 512, (2, 128), generator=torch.Generator().manual_seed(3)).to(dev)
    tgt = torch.randint(0, 512, (2, 128), generator=torch.Generator().manual_seed(4)).to(dev)
    ref = _tiny_gpt(dev)
    logits_r, loss_r = ref(idx, tgt)
    loss_r.backward()
    tp = _tiny_gpt(dev, tp_group=dist.group.WORLD)
    logits, loss = tp(idx, tgt)
    loss.backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - loss_r.item()) < 2e-2, (loss.item(), loss_r.item())
    assert (logits.float() - logits_r.float()).abs().max().item() < 0.1
    g, gr = tp.blocks[0].fc1.weight.grad.float(), ref.blocks[0].fc1.weight.grad.float()
    assert (g - gr).norm().item() <= 0.05 * gr.norm().item() + 1e-6


def test_readiness_rccl_single_stage():
    """The readiness op's RCCL stage on a one-GPU pod (``--rccl-single``): librccl loaded, a
    communicator created, the all-reduce sweep checked for the exact sum."""
    exe = ROOT / "kubeflow_rm_amd" / "bin" / "kfamd-readiness"
    p = subprocess.run([str(exe), "--rccl-single", "--skip-ln", "--m", "1024", "--n", "1024", "--k", "1024",
                        "--ar-max-bytes", str(16 << 20)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    rep = json.loads(p.stdout.strip().splitlines()[-1])
    ar = rep["allreduce"]
    assert rep["ok"] is True and ar["correct"] is True and ar["devices"] == 1, rep
    assert ar["comm_init_ms"] > 0 and rep["stages_ms"]["allreduce"] > 0 and rep["rccl_load_ms"] > 0
    assert [s["bytes"] for s in ar["sweep"]][-1] == 8 << 21 and all(s["us"] > 0 for s in ar["sweep"])


def test_bench_force_dist_runs_the_multi_gpu_path_under_torchrun(tmp_path):
    """``torchrun --nproc-per-node 1 bench.py --force-dist``: the nccl init, the gloo CPU group, the
    agree barrier, the RCCL sweep, the peer all-reduces, the xGMI probe and the cold-start parking
    all run, and the one JSON line carries their keys."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT",
                                                             "KFAMD_FORCE_DIST")}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "bench.py"),
           "--gpus", "1", "--steps", "5", "--warmup", "2", "--prewarm-s", "0.2", "--gemm-m", "2048", "--gemm-n",
           "2048", "--gemm-k", "2048", "--force-dist", "--coldstart-runs", "1", "--coldstart-torch-runs", "0", "--ab-blocks", "2",
           "--budget-s", "240"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    (tmp_path / "bench.log").write_text(p.stdout + "\n" + p.stderr)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["dist_path"] == "rccl" and d["n_gpus"] == 1 and d["correct"] is True
    st = d["extras_status"]
    for name in ("rccl_allreduce", "peer_allreduce", "xgmi_probe", "gemm_ab_vs_hipblaslt", "cold_start_stub"):
        assert st[name]["status"] == "ok", (name, st)
    for dt in ("fp32", "bf16"):
        sw = d[f"rccl_allreduce_{dt}"]
        assert sw[0]["bytes"] == 8 and sw[-1]["bytes"] == 1 << 30 and all(r["us"] > 0 for r in sw)
    assert all(r["correct"] for r in d["allreduce_oneshot_bf16"] + d["allreduce_twoshot_bf16"])
    assert d["ab_ours_tflops_median"] > 0 and d["ab_hipblaslt_tflops_median"] > 0
    assert d["cold_start_runs"] == 1


def test_config4_in_pod_rccl_and_config5_attach_on_the_gpu_notebook():
    """BASELINE configs 4 and 5 as bench.py runs them (config4_* / config5_* keys), on this box's
    GPUs: the notebook holding every GPU runs the RCCL stage inside its pod (``--rccl-single`` on one
    GPU) before Ready, and a TensorBoard + PVCViewer attach to its RWO workspace PVC on its node."""
    from kubeflow_rm_amd.bench_coldstart import measure_gpu_notebook_configs
    n = torch.cuda.device_count()
    r = measure_gpu_notebook_configs(gpus_per_notebook=n, timeout=90)
    assert r["config4_readiness_ok"] is True, r
    assert r["config4_rccl_devices"] == n and r["config4_rccl_correct"] is True, r
    assert r["config4_rccl_comm_init_ms"] > 0 and len(r["config4_rccl_sweep"]) >= 5
    assert r["config4_rccl_bytes"] == 16 << 20 and r["config4_rccl_algbw_GBps"] > 0
    assert r["config5_coscheduled"] is True, r
