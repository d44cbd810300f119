"""GPT-style decoder LM built on the framework's gfx950 ops — the in-notebook workload.

Used by the multi-GPU notebook smoke (BASELINE config 4: DP/TP over RCCL inside a pod), the
examples and ``smoke()``. Every projection runs on the hand-written MFMA GEMM with its fused
epilogue (bias + GELU for the MLP up-projection; residual for the down-projection), LayerNorm
on the wave-per-row kernel, the LM-head loss on the bf16 cross-entropy kernel, causal attention on
the hand-written flash kernels (``ops.attention_qkv``: reads the fused QKV output in place, writes
the output projection's input layout; head dims 64 / 128). Other head dims and the torch reference
mode use ``scaled_dot_product_attention``.
With a tensor-parallel group the attention heads and the MLP are split Megatron-style
(QKV / fc1 column-parallel, out-proj / fc2 row-parallel: one all-reduce per sub-block).

On CPU tensors the same module runs torch's reference ops (used by the gloo tests).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn.functional as F

from kubeflow_rm_amd import ops
from kubeflow_rm_amd.parallel import tp as tpl


@dataclass
class GPTConfig:
    vocab_size: int = 32000
    d_model: int = 1024
    n_layers: int = 12
    n_heads: int = 16
    d_ff: int = 4096
    max_seq: int = 2048
    dropout: float = 0.0
    dtype: torch.dtype = torch.bfloat16

    @property
    def head_dim(self) -> int:
        return self.d_model // self.n_heads


CONFIGS = {
    "gpt-tiny": GPTConfig(vocab_size=512, d_model=256, n_layers=2, n_heads=4, d_ff=1024, max_seq=256),
    "gpt-small": GPTConfig(vocab_size=32000, d_model=768, n_layers=12, n_heads=12, d_ff=3072, max_seq=2048),
    "gpt-1b": GPTConfig(vocab_size=32000, d_model=2048, n_layers=24, n_heads=16, d_ff=8192, max_seq=4096),
}


def _layer_norm(x, w, b, eps=1e-5):
    if x.is_cuda:
        from kubeflow_rm_amd import ops
        if ops.native_enabled():
            return ops.layer_norm(x, w, b, eps)
        return F.layer_norm(x, (x.shape[-1],), w, b, eps)
    return F.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), eps).to(x.dtype)


def _cross_entropy(logits, targets):
    if logits.is_cuda:
        from kubeflow_rm_amd import ops
        if ops.native_enabled():
            return ops.cross_entropy(logits, targets)  # bf16 logits, no fp32 copy
    return F.cross_entropy(logits.float().view(-1, logits.shape[-1]), targets.reshape(-1))


class LayerNorm(torch.nn.Module):
    def __init__(self, d, dtype, device=None):
        super().__init__()
        self.weight = torch.nn.Parameter(torch.ones(d, dtype=dtype, device=device))
        self.bias = torch.nn.Parameter(torch.zeros(d, dtype=dtype, device=device))

    def forward(self, x):
        return _layer_norm(x, self.weight, self.bias)

    def with_residual(self, x):
        """(LayerNorm(x), r) with r = x for the block's residual add: on the HIP path the two gradient
        contributions to x are summed inside the LayerNorm backward kernel (no separate add)."""
        if x.is_cuda:
            from kubeflow_rm_amd import ops
            if ops.native_enabled():
                return ops.layer_norm_residual(x, self.weight, self.bias)
        return self(x), x


def _qkv_shard(cfg: GPTConfig, tp: int, rank: int, seed: int, device) -> torch.Tensor:
    full = tpl.full_weight((3 * cfg.d_model, cfg.d_model), seed)
    hl, hd = cfg.n_heads // tp, cfg.head_dim
    rows = []
    for part in range(3):  # q, k, v
        base = part * cfg.d_model + rank * hl * hd
        rows.append(full[base:base + hl * hd])
    return torch.cat(rows, 0).to(dtype=cfg.dtype, device=device)


class Block(torch.nn.Module):
    def __init__(self, cfg: GPTConfig, layer: int, tp_group=None, device=None):
        super().__init__()
        tp = tpl._world(tp_group)
        if cfg.n_heads % tp:
            raise ValueError(f"n_heads={cfg.n_heads} not divisible by tp={tp}")
        self.cfg, self.tp_group = cfg, tp_group
        self.local_heads = cfg.n_heads // tp
        seed = 1000 * (layer + 1)
        self.ln1 = LayerNorm(cfg.d_model, cfg.dtype, device)
        # fused QKV, column-parallel: each rank owns local_heads of q, k and v
        self.qkv = tpl.ColumnParallelLinear(cfg.d_model, 3 * cfg.d_model, group=tp_group, dtype=cfg.dtype, device=device,
                                            seed=seed + 1)
        if tp > 1:
            # the canonical full QKV weight is [q_all; k_all; v_all]; this rank's column shard must
            # hold q, k and v rows of *its* heads so the sharded model equals the unsharded one
            with torch.no_grad():
                self.qkv.weight.copy_(_qkv_shard(cfg, tp, tpl._rank(tp_group), seed + 1, device))
        self.proj = tpl.RowParallelLinear(cfg.d_model, cfg.d_model, group=tp_group, dtype=cfg.dtype, device=device, seed=seed + 2)
        self.ln2 = LayerNorm(cfg.d_model, cfg.dtype, device)
        self.fc1 = tpl.ColumnParallelLinear(cfg.d_model, cfg.d_ff, act="gelu_tanh", group=tp_group, dtype=cfg.dtype,
                                            device=device, seed=seed + 3)
        self.fc2 = tpl.RowParallelLinear(cfg.d_ff, cfg.d_model, group=tp_group, dtype=cfg.dtype, device=device, seed=seed + 4)

    def attention(self, x, residual=None):
        B, T, _ = x.shape
        h, hd = self.local_heads, self.cfg.head_dim
        # the fused single-rank path whenever the TP layers would issue no collective; a forced-distributed
        # run at world size 1 (KFAMD_FORCE_DIST) takes the TP layers and their RCCL all-reduces
        if x.is_cuda and ops.native_enabled() and ops.attention_supported(x, hd) and not tpl._collective(self.tp_group):
            # one autograd node on the HIP path (ops.attn_block): its backward runs the QKV and
            # output-projection weight gradients as one GEMM launch
            return ops.attn_block(x, self.qkv.weight, self.qkv.bias, self.proj.weight, self.proj.bias, h, hd,
                                  residual=residual)
        qkv = self.qkv(x)  # [B, T, 3 * h * hd] — the column shard is [q_h | k_h | v_h] per rank
        if ops.native_enabled() and ops.attention_supported(qkv, hd):
            y = ops.attention_qkv(qkv.contiguous(), h, hd, causal=True)  # [B, T, h * hd]
            return self.proj(y, residual=residual)
        q, k, v = ops.split_heads(qkv, h, hd)  # backward: one pass into the QKV gradient layout
        y = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        return self.proj(y.transpose(1, 2).reshape(B, T, h * hd), residual=residual)

    def mlp(self, h, residual):
        # without TP, fc1 + fc2 are one autograd node on the HIP path (ops.mlp): fc2's dgrad applies
        # fc1's gelu backward in its GEMM epilogue
        if h.is_cuda and ops.native_enabled() and not tpl._collective(self.tp_group):
            return ops.mlp(h, self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias, act=self.fc1.act,
                           residual=residual)
        return self.fc2(self.fc1(h), residual=residual)

    def forward(self, x):
        # both residual adds ride in the output projections' GEMM epilogues (without TP); the
        # residual gradient joins the LayerNorm backward's dx store (LayerNorm.with_residual)
        h, r = self.ln1.with_residual(x)
        x = self.attention(h, residual=r)
        h, r = self.ln2.with_residual(x)
        return self.mlp(h, r)


class GPT(torch.nn.Module):
    def __init__(self, cfg: GPTConfig, tp_group=None, device=None):
        super().__init__()
        self.cfg = cfg
        g = torch.Generator(device="cpu").manual_seed(7)
        emb = torch.randn(cfg.vocab_size, cfg.d_model, generator=g) * 0.02
        pos = torch.randn(cfg.max_seq, cfg.d_model, generator=g) * 0.01
        self.tok = torch.nn.Parameter(emb.to(dtype=cfg.dtype, device=device))
        self.pos = torch.nn.Parameter(pos.to(dtype=cfg.dtype, device=device))
        self.blocks = torch.nn.ModuleList([Block(cfg, i, tp_group, device) for i in range(cfg.n_layers)])
        self.ln_f = LayerNorm(cfg.d_model, cfg.dtype, device)

    def forward(self, idx, targets=None):
        B, T = idx.shape
        x = F.embedding(idx, self.tok) + self.pos[:T]
        for blk in self.blocks:
            x = blk(x)
        x = self.ln_f(x)
        logits = tpl._linear(x, self.tok)  # tied output head [B, T, vocab]
        if targets is None:
            return logits
        return logits, _cross_entropy(logits, targets)

    def flops_per_token(self, seq: int) -> float:
        """Training FLOPs/token (fwd+bwd = 3x fwd): dense matmuls + attention scores."""
        c = self.cfg
        dense = 2 * (4 * c.d_model * c.d_model + 2 * c.d_model * c.d_ff) * c.n_layers + 2 * c.d_model * c.vocab_size
        attn = 2 * 2 * seq * c.d_model * c.n_layers
        return 3.0 * (dense + attn)


def build(name_or_cfg, tp_group=None, device=None) -> GPT:
    cfg = CONFIGS[name_or_cfg] if isinstance(name_or_cfg, str) else name_or_cfg
    return GPT(cfg, tp_group=tp_group, device=device)


def num_params(model: torch.nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())


def init_scale(d: int) -> float:
    return 1.0 / math.sqrt(d)
