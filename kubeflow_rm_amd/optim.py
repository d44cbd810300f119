"""AdamW on the multi-tensor HIP kernel (kernels/adamw_bf16.hip).

``AdamW(params, lr, betas, eps, weight_decay)`` has torch.optim.AdamW's update (decoupled weight
decay, bias-corrected moments) and its defaults. Every bf16 CUDA parameter with a gradient is updated
by ONE kernel launch per step, from a device-resident table of (param, grad, exp_avg, exp_avg_sq)
pointers that is rebuilt only when a pointer changes (a gradient re-allocated by
``zero_grad(set_to_none=True)`` usually lands at the same address). Moments are kept in the
parameter dtype, as torch's fused AdamW keeps them. Anything else (fp32 parameters, CPU tensors,
amsgrad / maximize) goes through ``torch.optim.AdamW``'s own functional update.
"""
from __future__ import annotations

import math

import torch


class AdamW(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 1e-2):
        if lr < 0 or eps < 0 or not 0 <= betas[0] < 1 or not 0 <= betas[1] < 1 or weight_decay < 0:
            raise ValueError("invalid AdamW hyper-parameter")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay))
        # (device, (group index, step-count rank)) -> (pointers, table, ntensors, nchunks, pinned host copy)
        self._tables: dict = {}

    def _native_ok(self, p: torch.Tensor) -> bool:
        from kubeflow_rm_amd import ops
        return (p.is_cuda and p.dtype == torch.bfloat16 and p.grad is not None and p.grad.dtype == torch.bfloat16
                and p.is_contiguous() and p.grad.is_contiguous() and not p.grad.is_sparse and ops.native_enabled())

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            lr, (b1, b2), eps, wd = group["lr"], group["betas"], group["eps"], group["weight_decay"]
            native, other = [], []
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                elif torch.is_tensor(st["step"]):  # a state loaded from torch.optim.AdamW keeps a tensor
                    st["step"] = int(st["step"].item())
                st["step"] += 1
                (native if self._native_ok(p) else other).append(p)
            # one launch per (device, step count); normally one. The pointer table of each is cached
            # under its rank among this step's step counts on that device, which stays the same
            # from step to step (keying it by the step count would rebuild it every step)
            by_step: dict = {}
            for p in native:
                by_step.setdefault((p.device, self.state[p]["step"]), []).append(p)
            rank: dict = {}
            for (dev, t), ps in sorted(by_step.items(), key=lambda kv: (str(kv[0][0]), kv[0][1])):
                k = rank[dev] = rank.get(dev, -1) + 1
                self._launch((gi, k), dev, ps, t, lr, b1, b2, eps, wd)
            if other:
                torch.optim._functional.adamw(
                    [p for p in other], [p.grad for p in other], [self.state[p]["exp_avg"] for p in other],
                    [self.state[p]["exp_avg_sq"] for p in other], [],
                    [torch.tensor(float(self.state[p]["step"] - 1)) for p in other],  # (it counts the step itself)
                    foreach=False, amsgrad=False, beta1=b1, beta2=b2, lr=lr, weight_decay=wd, eps=eps,
                    maximize=False, capturable=False, differentiable=False, fused=None, grad_scale=None,
                    found_inf=None, has_complex=False)
        return loss

    def _launch(self, gi, dev, ps, t, lr, b1, b2, eps, wd):
        from kubeflow_rm_amd.ops import _lib
        L = _lib.lib()
        chunk = L.kfamd_adamw_chunk()
        ptrs = []
        for p in ps:
            st = self.state[p]
            ptrs.append((p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(),
                         p.numel()))
        key = tuple(ptrs)
        cached = self._tables.get((dev, gi))
        if cached is None or cached[0] != key:
            rows, owner, c0 = [], [], 0
            for i, (pp, gp, mp, vp, n) in enumerate(ptrs):
                rows.append([pp, gp, mp, vp, n, c0])
                nc = -(-n // chunk)
                owner.append(torch.full((nc,), i, dtype=torch.int32))
                c0 += nc
            assert L.kfamd_adamw_tensor_bytes() == 48
            host = (torch.tensor(rows, dtype=torch.int64).pin_memory(), torch.cat(owner).pin_memory())
            table, own = host[0].to(dev, non_blocking=True), host[1].to(dev, non_blocking=True)
            cached = (key, (table, own), len(rows), c0, host)
            self._tables[(dev, gi)] = cached
        _, (table, own), _, nchunks, _ = cached
        step_size = lr / (1.0 - b1 ** t)
        inv_sqrt_bc2 = 1.0 / math.sqrt(1.0 - b2 ** t)
        rc = L.kfamd_adamw_bf16(table.data_ptr(), own.data_ptr(), nchunks, float(lr), float(b1), float(b2), float(eps),
                                float(wd), float(step_size), float(inv_sqrt_bc2),
                                torch.cuda.current_stream(dev).cuda_stream)
        _lib.check(rc, "adamw")
