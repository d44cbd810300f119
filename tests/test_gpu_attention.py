"""Flash attention kernels (kernels/attention_bf16.hip) against fp32 PyTorch.

Every check compares the bf16 kernel with ``F.scaled_dot_product_attention`` evaluated in fp32 on
the same bf16-rounded inputs: the output, the forward's log-sum-exp, and dq / dk / dv for a random
upstream gradient. Shapes cover T in {40, 65, 128, 1000, 2048, 4096} (40 / 65 / 1000: partial query and key tiles),
odd batch / head counts, head dims 64 and 128, causal and not. The online-softmax rescale is forced
by a spiked key (cdna_hip_programming.md §5.4 rule 26), and the fused-QKV entry point is checked
against the view entry point (same numbers, gradients in the QKV layout).
"""
from __future__ import annotations

import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _inputs(B, H, T, D, seed=0, scale_in=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    q, k, v = (torch.randn(B, H, T, D, generator=g) * scale_in for _ in range(3))
    return [x.to(DEV, torch.bfloat16) for x in (q, k, v)]


def _ref(q, k, v, causal, do=None):
    qf, kf, vf = (x.detach().float().requires_grad_(True) for x in (q, k, v))
    o = F.scaled_dot_product_attention(qf, kf, vf, is_causal=causal)
    if do is None:
        return o, None
    o.backward(do.float())
    return o, (qf.grad, kf.grad, vf.grad)


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


SHAPES = [
    (1, 1, 128, 64, True),
    (2, 3, 1000, 128, True),
    (3, 5, 1000, 64, True),
    (1, 2, 2048, 128, True),
    (2, 2, 2048, 64, True),
    (1, 1, 4096, 128, True),
    (2, 3, 1000, 128, False),
    (1, 2, 256, 64, False),
    (1, 2, 40, 128, True),   # shorter than one key tile and than one 128-row block
    (2, 1, 65, 64, False),   # one row / key past a tile
    # grids of >= 256 workgroups of 256 query rows: the one-workgroup-per-CU forward (attn_fwd_pp)
    (8, 32, 512, 128, True),  # paired query blocks
    (2, 64, 700, 128, True),  # an odd number of 256-row blocks (unpaired), partial tiles
    (4, 64, 1000, 128, False),
]


@pytest.mark.parametrize("B,H,T,D,causal", SHAPES)
def test_flash_forward_matches_fp32(B, H, T, D, causal):
    from kubeflow_rm_amd import ops
    q, k, v = _inputs(B, H, T, D, seed=T + D)
    o = ops.flash_attention(q, k, v, causal=causal)
    ref, _ = _ref(q, k, v, causal)
    assert o.shape == ref.shape and o.dtype == torch.bfloat16
    err = (o.float() - ref).abs().max().item()
    assert err < 2e-2, err
    assert _rel(o, ref) < 8e-3


@pytest.mark.parametrize("B,H,T,D,causal", SHAPES)
def test_flash_backward_matches_fp32(B, H, T, D, causal):
    from kubeflow_rm_amd import ops
    q, k, v = _inputs(B, H, T, D, seed=7 * T + D)
    g = torch.Generator(device="cpu").manual_seed(99)
    do = torch.randn(B, H, T, D, generator=g).to(DEV, torch.bfloat16)
    qs, ks, vs = (x.clone().requires_grad_(True) for x in (q, k, v))
    o = ops.flash_attention(qs, ks, vs, causal=causal)
    o.backward(do)
    _, (dq, dk, dv) = _ref(q, k, v, causal, do)
    for name, got, want in (("dq", qs.grad, dq), ("dk", ks.grad, dk), ("dv", vs.grad, dv)):
        assert got is not None and got.dtype == torch.bfloat16
        assert torch.isfinite(got.float()).all(), name
        assert _rel(got, want) < 2e-2, (name, _rel(got, want))


@pytest.mark.parametrize("H", [2, 256])  # 256 heads: the attn_fwd_pp grid
def test_forward_lse_and_rescale_branch_forced(H):
    """Keys whose scores jump at a later tile force the online-softmax rescale of O and l (rule 26):
    one query row's max is set by a key far into the sequence, another row's max moves at every tile."""
    from kubeflow_rm_amd import ops
    from kubeflow_rm_amd.ops import attention as A
    B, T, D = 1, 1000, 128
    q, k, v = _inputs(B, H, T, D, seed=3)
    q[:, :, 900] = 0.5
    k[:, :, 700] = 4.0          # query 900 meets a far larger score at key 700 (tile 10)
    ramp = torch.linspace(0.0, 3.0, T, device=DEV).view(1, 1, T, 1)
    k[:, 1:] = (k[:, 1:].float() * 0.1 + ramp).to(torch.bfloat16)  # head 1: max grows every tile
    o = ops.flash_attention(q, k, v, causal=True)
    ref, _ = _ref(q, k, v, True)
    assert (o.float() - ref).abs().max().item() < 3e-2
    # the saved log-sum-exp equals logsumexp(scale * q k^T) over the causal keys
    o2 = A._bhtd(torch.empty(B, T, H, D, device=DEV, dtype=torch.bfloat16))
    lse = A._fwd(q, k, v, o2, True, 1.0 / math.sqrt(D))
    s = (q.float() @ k.float().transpose(-1, -2)) / math.sqrt(D)
    s = s.masked_fill(torch.triu(torch.ones(T, T, dtype=torch.bool, device=DEV), 1), float("-inf"))
    assert (lse - torch.logsumexp(s, -1)).abs().max().item() < 1e-3


@pytest.mark.parametrize("T,hd", [(256, 64), (1000, 128)])
def test_attention_qkv_matches_view_entry_point(T, hd):
    """The model's entry point (fused QKV in, [B, T, h*hd] out, dqkv in the QKV layout) computes
    the same numbers as the [B, H, T, D] entry point."""
    from kubeflow_rm_amd import ops
    B, h = 2, 3
    g = torch.Generator(device="cpu").manual_seed(5)
    qkv = torch.randn(B, T, 3 * h * hd, generator=g).to(DEV, torch.bfloat16).requires_grad_(True)
    y = ops.attention_qkv(qkv, h, hd)
    dy = torch.randn(B, T, h * hd, generator=g).to(DEV, torch.bfloat16)
    y.backward(dy)
    x = qkv.detach().view(B, T, 3, h, hd).permute(2, 0, 3, 1, 4)
    q, k, v = (t.clone().requires_grad_(True) for t in x)
    o = ops.flash_attention(q, k, v)
    o.backward(dy.view(B, T, h, hd).permute(0, 2, 1, 3))
    assert torch.equal(y.view(B, T, h, hd).permute(0, 2, 1, 3), o)
    want = torch.stack([q.grad, k.grad, v.grad], 0).permute(1, 3, 0, 2, 4).reshape(B, T, 3 * h * hd)
    assert torch.equal(qkv.grad, want)


def test_gpt_attention_runs_on_the_flash_kernel():
    """The model's attention goes through ops.attention_qkv (no SDPA call) and matches the torch
    reference mode (SDPA + torch ops) on the same weights."""
    from unittest import mock
    from kubeflow_rm_amd import ops
    from kubeflow_rm_amd.models import GPT, GPTConfig
    cfg = GPTConfig(vocab_size=512, d_model=256, n_layers=2, n_heads=4, d_ff=1024, max_seq=256)
    torch.manual_seed(0)
    model = GPT(cfg, device=DEV)
    idx = torch.randint(0, 512, (2, 256), device=DEV)
    tgt = torch.randint(0, 512, (2, 256), device=DEV)
    with mock.patch.object(F, "scaled_dot_product_attention", side_effect=AssertionError("SDPA called")):
        _, loss = model(idx, tgt)
        loss.backward()
    g_native = model.blocks[0].qkv.weight.grad.clone()
    model.zero_grad(set_to_none=True)
    with ops.torch_reference():
        _, loss_ref = model(idx, tgt)
        loss_ref.backward()
    assert abs(loss.item() - loss_ref.item()) < 2e-2
    assert _rel(g_native, model.blocks[0].qkv.weight.grad) < 5e-2
