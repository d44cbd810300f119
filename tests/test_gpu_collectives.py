"""K3 one-shot all-reduce kernel (kernels/allreduce_oneshot.hip) vs a plain fp32 PyTorch reference.

On the single-GPU test box the ranks are simulated on one device in ONE launch (gridDim.y = ranks):
the barrier protocol, vector/tail paths, epoch reuse and the timeout drain all run on the hardware.
"""
import ctypes
import time

import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(xs):
    acc = torch.zeros_like(xs[0], dtype=torch.float32)
    for x in xs:  # rank order, fp32 — what the kernel computes
        acc += x.float()
    return acc


@pytest.mark.parametrize("nranks", [2, 4, 8])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("numel", [8, 1001, 4096, 65536, 300_000])
def test_oneshot_matches_fp32_reference(nranks, dtype, numel):
    from kubeflow_rm_amd.ops import OneShotAllReduce
    ar = OneShotAllReduce(nranks, 1 << 19, dtype)
    g = torch.Generator(device="cuda").manual_seed(nranks * 1000 + numel)
    xs = [torch.randn(numel, device="cuda", generator=g).to(dtype) for _ in range(nranks)]
    outs = ar(xs)
    torch.cuda.synchronize()
    assert not ar.timed_out()
    ref = _ref(xs).to(dtype)
    for o in outs:
        torch.testing.assert_close(o, ref, rtol=0, atol=0)  # same order, same rounding: exact
    for o in outs[1:]:
        assert torch.equal(o, outs[0])


def test_oneshot_epochs_reuse_flags():
    from kubeflow_rm_amd.ops import OneShotAllReduce
    ar = OneShotAllReduce(4, 1 << 16, torch.float32)
    for it in range(1, 6):
        xs = [torch.full((5000,), float(r + it), device="cuda") for r in range(4)]
        outs = ar(xs)
        torch.cuda.synchronize()
        want = sum(r + it for r in range(4))
        assert all(torch.all(o == want).item() for o in outs), it
    assert ar.epoch == 5 and not ar.timed_out()


def test_oneshot_missing_peer_times_out_instead_of_hanging():
    from kubeflow_rm_amd.ops import _lib
    L = _lib.lib()
    n, nb = 4096, 1
    ins = [torch.ones(n, device="cuda") for _ in range(2)]
    outs = [torch.zeros(n, device="cuda") for _ in range(2)]
    flags = [torch.zeros(L.kfamd_allreduce_oneshot_flag_bytes(2, nb) // 4, dtype=torch.int32, device="cuda")
             for _ in range(2)]
    tmo = torch.zeros(1, dtype=torch.int32, device="cuda")
    arr = ctypes.c_void_p * 8
    L.kfamd_allreduce_oneshot_set_timeout_ms(200)
    try:
        t0 = time.perf_counter()
        rc = L.kfamd_allreduce_oneshot(arr(*[t.data_ptr() for t in ins]), arr(*[t.data_ptr() for t in outs]),
                                       arr(*[t.data_ptr() for t in flags]), 2, 0, 1, n, 0, 1, nb, tmo.data_ptr(),
                                       torch.cuda.current_stream().cuda_stream)
        assert rc == 0
        torch.cuda.synchronize()  # rank 1 never launched: the entry barrier gives up, the kernel drains
        dt = time.perf_counter() - t0
    finally:
        L.kfamd_allreduce_oneshot_set_timeout_ms(5000)
    assert tmo.item() == 1
    assert 0.15 < dt < 3.0, dt  # wall-clock deadline, not a spin count
    # a timed-out call never looks like a result: rank 0's output is NaN-poisoned, not a stale sum
    assert torch.isnan(outs[0]).all().item()


def test_oneshot_rejects_bad_arguments():
    from kubeflow_rm_amd.ops import _lib
    L = _lib.lib()
    arr = ctypes.c_void_p * 8
    z = arr(*([0] * 8))
    assert L.kfamd_allreduce_oneshot(z, z, z, 9, 0, 1, 16, 0, 1, 1, None, None) == -1  # > 8 ranks
    t = torch.zeros(64, device="cuda")
    p = arr(*([t.data_ptr()] * 8))
    tmo = torch.zeros(1, dtype=torch.int32, device="cuda")
    assert L.kfamd_allreduce_oneshot(p, p, p, 2, 0, 2, 16, 0, 0, 1, tmo.data_ptr(), None) == -1  # epoch 0
    assert L.kfamd_allreduce_oneshot(arr(*([t.data_ptr() + 4] * 8)), p, p, 2, 0, 2, 16, 0, 1, 1,
                                     tmo.data_ptr(), None) == -2  # misaligned input


def _ipc_worker(rank):
    import torch.distributed as dist
    from kubeflow_rm_amd.parallel.oneshot import IpcOneShotAllReduce
    torch.cuda.set_device(0)  # the test box has one GPU: both ranks share it (IPC within a device)
    dist.init_process_group("gloo")
    world = dist.get_world_size()
    ar = IpcOneShotAllReduce(max_bytes=1 << 20)
    worst = 0.0
    for dtype in (torch.float32, torch.bfloat16):
        for it, n in enumerate((8, 1001, 65536, 200_000)):
            def data(r):
                g = torch.Generator(device="cuda").manual_seed(1000 * r + it)
                return torch.randn(n, device="cuda", generator=g).to(dtype)
            t = data(rank)
            ar(t)
            torch.cuda.synchronize()
            ref = torch.zeros(n, device="cuda")
            for r in range(world):
                ref += data(r).float()
            worst = max(worst, (t.float() - ref.to(dtype).float()).abs().max().item())
    out = {"timed_out": ar.timed_out(), "worst": worst, "epochs": ar.epoch}
    ar.close()
    dist.destroy_process_group()
    return out


def _ipc_late_worker(rank, sleep_s, timeout_ms):
    import torch.distributed as dist
    from kubeflow_rm_amd.parallel.oneshot import IpcOneShotAllReduce, OneShotTimeout
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    ar = IpcOneShotAllReduce(max_bytes=1 << 16, timeout_ms=timeout_ms, check_every=1)
    res = {"ok": None, "raised": False}
    t = torch.full((1024,), float(rank + 1), device="cuda")
    if rank == 1:
        time.sleep(sleep_s)  # host-side skew: GC pause, logging, checkpointing on one TP rank
    try:
        ar(t)
        torch.cuda.synchronize()
        res["ok"] = bool(torch.all(t == 3.0).item())
    except OneShotTimeout:
        res["raised"] = True
        res["nan"] = bool(torch.isnan(t).all().item())
        try:
            ar(t)
        except OneShotTimeout:
            res["refuses_after"] = True
    dist.barrier()
    ar.close()
    dist.destroy_process_group()
    return res


def test_ipc_oneshot_tolerates_half_second_host_skew():
    """a 0.5 s late rank must not corrupt the sum (the deadline is wall clock, 5 s)."""
    from kubeflow_rm_amd.parallel.launch import spawn
    for r in spawn(_ipc_late_worker, 2, 0.5, 5000, timeout=180):
        assert r["raised"] is False and r["ok"] is True, r


def test_ipc_oneshot_timeout_is_fatal_not_silent():
    """A peer later than the deadline: NaN output + OneShotTimeout, and the communicator refuses
    further calls instead of running with out-of-step flags."""
    from kubeflow_rm_amd.parallel.launch import spawn
    res = spawn(_ipc_late_worker, 2, 1.5, 200, timeout=180)
    r0 = res[0]
    assert r0["raised"] is True and r0["nan"] is True and r0.get("refuses_after") is True, r0


@pytest.mark.parametrize("world", [2, 4])
def test_ipc_oneshot_ranks_as_processes(world):
    """torch.distributed ranks (separate processes) over HIP IPC-mapped buffers; on the 1-GPU box
    all processes share the device, exercising registration, handle exchange and the barrier."""
    from kubeflow_rm_amd.parallel.launch import spawn
    res = spawn(_ipc_worker, world, timeout=180)
    assert len(res) == world
    for r in res:
        assert r["timed_out"] is False, r
        assert r["worst"] == 0.0, r
        assert r["epochs"] == 8


def _tp_oneshot_worker(rank):
    import torch.distributed as dist
    from kubeflow_rm_amd.models import GPT, GPTConfig
    from kubeflow_rm_amd.parallel import tp as tpl
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    cfg = GPTConfig(vocab_size=512, d_model=256, n_layers=2, n_heads=4, d_ff=1024, max_seq=64)
    torch.manual_seed(0)
    idx = torch.randint(0, 512, (1, 32)).cuda()
    model = GPT(cfg, tp_group=dist.group.WORLD, device="cuda").eval()
    with torch.no_grad():
        ref = model(idx).float().cpu()  # TP all-reduces through gloo
        fast = tpl.enable_oneshot(dist.group.WORLD)
        out = model(idx).float().cpu()  # the same all-reduces on the one-shot IPC kernel
    torch.cuda.synchronize()
    res = {"max_diff": (out - ref).abs().max().item(), "calls": fast.epoch, "timed_out": fast.timed_out()}
    fast.close()
    tpl._FAST.clear()
    dist.destroy_process_group()
    return res


def test_tp_forward_on_oneshot_matches_reference_all_reduce():
    from kubeflow_rm_amd.parallel.launch import spawn
    for r in spawn(_tp_oneshot_worker, 2, timeout=180):
        assert r["timed_out"] is False and r["calls"] >= 4, r  # 2 row-parallel reduces per block
        assert r["max_diff"] == 0.0, r


# ---- r3: two-shot all-reduce, partial-timeout poisoning ------------------------------------------

@pytest.mark.parametrize("nranks", [2, 4, 8])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("numel", [8, 1001, 65536, 300_007, 2_000_000])
def test_twoshot_matches_fp32_reference(nranks, dtype, numel):
    """Reduce-scatter + all-gather in one launch: each slice is summed in rank order by its owner,
    so the result is bit-identical to the fp32 rank-order reference on every rank."""
    from kubeflow_rm_amd.ops import OneShotAllReduce
    ar = OneShotAllReduce(nranks, 1 << 21, dtype)
    g = torch.Generator(device="cuda").manual_seed(7 * nranks + numel)
    xs = [torch.randn(numel, device="cuda", generator=g).to(dtype) for _ in range(nranks)]
    outs = ar(xs, algo="twoshot")
    torch.cuda.synchronize()
    assert not ar.timed_out()
    ref = _ref(xs).to(dtype)
    for o in outs:
        torch.testing.assert_close(o, ref, rtol=0, atol=0)
    # alternate kinds on the shared flags: epochs keep them in step
    outs = ar(xs, algo="oneshot")
    torch.cuda.synchronize()
    assert all(torch.equal(o, ref) for o in outs) and not ar.timed_out()


@pytest.mark.parametrize("kind", ["oneshot", "twoshot"])
def test_partial_timeout_poisons_exactly_the_late_blocks_share(kind):
    """only SOME blocks miss the deadline (the late rank's blocks arrive one at a time).
    Rank 1 never launches; its entry-barrier flags are pre-set for half of rank 0's blocks. Those
    blocks pass and write correct sums, the others time out and must NaN exactly their own share:
    no element may keep the sentinel from before the call, none may be a wrong number."""
    from kubeflow_rm_amd.ops import _lib
    L = _lib.lib()
    n, nb, epoch = 40_000, 8, 1
    ins = [torch.randn(n, device="cuda") for _ in range(2)]
    outs = [torch.full((n,), 7.0, device="cuda") for _ in range(2)]
    fl = L.kfamd_allreduce_oneshot_flag_bytes(2, nb) // 4
    flags = [torch.zeros(fl, dtype=torch.int32, device="cuda") for _ in range(2)]
    for b in range(0, nb, 2):  # flags[me=0][phase 0][peer 1][block b] = epoch
        flags[0][(0 * 2 + 1) * nb + b] = epoch
    tmo = torch.zeros(1, dtype=torch.int32, device="cuda")
    arr = ctypes.c_void_p * 8
    fn = L.kfamd_allreduce_oneshot if kind == "oneshot" else L.kfamd_allreduce_twoshot
    L.kfamd_allreduce_oneshot_set_timeout_ms(150)
    try:
        rc = fn(arr(*[t.data_ptr() for t in ins]), arr(*[t.data_ptr() for t in outs]),
                arr(*[t.data_ptr() for t in flags]), 2, 0, 1, n, 0, epoch, nb, tmo.data_ptr(),
                torch.cuda.current_stream().cuda_stream)
        assert rc == 0
        torch.cuda.synchronize()
    finally:
        L.kfamd_allreduce_oneshot_set_timeout_ms(5000)
    assert tmo.item() == 1
    o = outs[0]
    nan = torch.isnan(o)
    assert not (o == 7.0).any().item(), "a timed-out block left part of its share unwritten"
    ref = ins[0] + ins[1]
    ok = ~nan
    if kind == "oneshot":  # passed blocks computed their share; two-shot blocks stop at the mid barrier
        assert ok.any().item() and nan.any().item()
    assert torch.equal(o[ok], ref[ok]), "a non-NaN element differs from the true sum"


def _ipc_twoshot_worker(rank):
    import torch.distributed as dist
    from kubeflow_rm_amd.parallel.oneshot import IpcOneShotAllReduce
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    world = dist.get_world_size()
    ar = IpcOneShotAllReduce(max_bytes=8 << 20)
    worst = 0.0
    for dtype in (torch.float32, torch.bfloat16):
        for it, n in enumerate((1001, 300_000, 1_000_003)):
            def data(r):
                g = torch.Generator(device="cuda").manual_seed(77 * r + it)
                return torch.randn(n, device="cuda", generator=g).to(dtype)
            t = data(rank)
            ar(t, algo="twoshot")
            torch.cuda.synchronize()
            ref = torch.zeros(n, device="cuda")
            for r in range(world):
                ref += data(r).float()
            worst = max(worst, (t.float() - ref.to(dtype).float()).abs().max().item())
    out = {"timed_out": ar.timed_out(), "worst": worst}
    ar.close()
    dist.destroy_process_group()
    return out


@pytest.mark.parametrize("world", [2, 4])
def test_ipc_twoshot_ranks_as_processes(world):
    from kubeflow_rm_amd.parallel.launch import spawn
    for r in spawn(_ipc_twoshot_worker, world, timeout=180):
        assert r["timed_out"] is False and r["worst"] == 0.0, r


def _probe_worker(rank):
    import torch.distributed as dist
    from kubeflow_rm_amd.parallel.collectives import fast_allreduce_sweep, xgmi_probe
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    xg = xgmi_probe(nbytes=32 << 20, iters=2)
    ts = fast_allreduce_sweep([256 << 10, 4 << 20], "twoshot", iters=3)
    os_ = fast_allreduce_sweep([16, 64 << 10], "oneshot", iters=3)
    dist.destroy_process_group()
    return {"xgmi": xg, "twoshot": ts, "oneshot": os_}


def test_bench_multi_gpu_probes_run_as_processes():
    """bench.py N > 1 extras (xGMI pair / all-pairs copy probe, one-/two-shot busbw sweeps) on
    processes sharing the one GPU of the test box: exercises IPC registration, the pair schedule
    and the result checks end to end (the numbers are same-device copies, not xGMI)."""
    from kubeflow_rm_amd.parallel.launch import spawn
    res = spawn(_probe_worker, 2, timeout=240)
    for r in res:
        xg = r["xgmi"]
        assert xg["pair_GBps"][0][1] > 0 and xg["pair_GBps"][1][0] > 0 and xg["pair_GBps"][0][0] == 0
        assert all(v > 0 for v in xg["all_pairs_egress_GBps_per_gpu"])
        assert all(row["correct"] for row in r["twoshot"] + r["oneshot"]), r


def test_readiness_op_twoshot_stage_simulated():
    """The in-pod readiness op's K3 stage with 4 simulated ranks and --full-sweep: one-shot sweep
    plus the two-shot 256 KiB..64 MiB sweep, every size checked exactly, busbw reported."""
    import json
    import subprocess
    from pathlib import Path
    exe = Path(__file__).resolve().parent.parent / "kubeflow_rm_amd" / "bin" / "kfamd-readiness"
    p = subprocess.run([str(exe), "--oneshot-sim", "4", "--full-sweep", "--skip-ln", "--m", "1024", "--n", "1024",
                        "--k", "1024"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    rep = json.loads(p.stdout.strip().splitlines()[-1])
    os_ = rep["allreduce_oneshot"]
    assert os_["correct"] is True and os_["ranks"] == 4
    ts = os_["twoshot_sweep"]
    assert [r["bytes"] for r in ts] == [256 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20]
    assert all(r["busbw_GBps"] > 0 for r in ts)
