"""DP / TP wiring on the CPU (gloo, world_size 2): the same code paths the multi-GPU notebook runs
over RCCL, checked for exact equivalence with the single-process model."""
import torch

from kubeflow_rm_amd.parallel.launch import spawn


def _tiny_cfg():
    from kubeflow_rm_amd.models import GPTConfig
    return GPTConfig(vocab_size=64, d_model=32, n_layers=2, n_heads=4, d_ff=64, max_seq=16, dtype=torch.float32)


def _tp_worker(rank):
    import torch.distributed as dist
    from kubeflow_rm_amd import parallel
    from kubeflow_rm_amd.models import GPT
    parallel.init(backend="gloo")
    torch.manual_seed(0)
    idx = torch.randint(0, 64, (2, 8))
    tgt = torch.randint(0, 64, (2, 8))
    model = GPT(_tiny_cfg(), tp_group=dist.group.WORLD)
    logits, loss = model(idx, tgt)
    loss.backward()
    out = {"logits": logits.detach(), "loss": loss.item(), "ln_grad": model.blocks[0].ln1.weight.grad.clone(),
           "tok_grad": model.tok.grad.clone()}
    parallel.shutdown()
    return out


def test_tensor_parallel_matches_single_process():
    from kubeflow_rm_amd.models import GPT
    torch.manual_seed(0)
    idx = torch.randint(0, 64, (2, 8))
    tgt = torch.randint(0, 64, (2, 8))
    ref = GPT(_tiny_cfg())
    logits, loss = ref(idx, tgt)
    loss.backward()
    outs = spawn(_tp_worker, 2)
    for o in outs:
        assert torch.allclose(torch.from_numpy(o["logits"]), logits.detach(), atol=1e-5, rtol=1e-4)
        assert abs(o["loss"] - loss.item()) < 1e-5
        assert torch.allclose(torch.from_numpy(o["ln_grad"]), ref.blocks[0].ln1.weight.grad, atol=1e-5, rtol=1e-4)
        assert torch.allclose(torch.from_numpy(o["tok_grad"]), ref.tok.grad, atol=1e-5, rtol=1e-4)


def _dp_worker(rank):
    import torch.distributed as dist
    from kubeflow_rm_amd import parallel
    parallel.init(backend="gloo")
    torch.manual_seed(123)  # same init everywhere; rank-0 broadcast must keep it
    net = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 8))
    dp = parallel.DataParallel(net, bucket_mb=0.001)  # tiny buckets: several async all-reduces
    x = torch.randn(4, 16, generator=torch.Generator().manual_seed(rank))
    dp(x).square().mean().backward()
    grads = [p.grad.clone() for p in net.parameters()]
    # reference: per-rank grads, averaged explicitly
    net2 = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 8))
    net2.load_state_dict(net.state_dict())
    net2(x).square().mean().backward()
    ref = []
    for p in net2.parameters():
        g = p.grad.clone()
        dist.all_reduce(g)
        ref.append(g / dist.get_world_size())
    nb = len(dp.bucketer.buckets)
    parallel.shutdown()
    return grads, ref, nb


def test_bucketed_data_parallel_grads():
    for grads, ref, nbuckets in spawn(_dp_worker, 2):
        assert nbuckets > 1
        for g, r in zip(grads, ref):
            assert torch.allclose(torch.from_numpy(g), torch.from_numpy(r), atol=1e-6)


def _coll_worker(rank):
    from kubeflow_rm_amd import parallel
    parallel.init(backend="gloo")
    r = parallel.allreduce_sweep(max_bytes=1 << 16, iters_small=3, iters_large=2)
    parallel.shutdown()
    return r


def test_allreduce_sweep_gloo():
    res = spawn(_coll_worker, 2)
    assert len(res[0]) >= 4 and all(x["busbw_GBps"] >= 0 for x in res[0])
