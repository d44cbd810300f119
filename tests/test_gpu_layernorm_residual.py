"""LayerNorm backward with the residual gradient folded into its dx store:
``ops.layer_norm_residual`` against fp32 autograd of ``F.layer_norm`` plus the residual path, on the
wave kernels (hidden 768 / 2048 / 4096 / 8192) and the block kernel (hidden 1000)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,H", [(256, 768), (513, 2048), (128, 4096), (64, 8192), (96, 1000)])
def test_layer_norm_residual_grads_match_fp32(rows, H):
    from kubeflow_rm_amd import ops
    g = torch.Generator(device="cpu").manual_seed(H)
    x0 = torch.randn(rows, H, generator=g).to("cuda", torch.bfloat16)
    w0 = (1 + 0.1 * torch.randn(H, generator=g)).to("cuda", torch.bfloat16)
    b0 = (0.1 * torch.randn(H, generator=g)).to("cuda", torch.bfloat16)
    gy = torch.randn(rows, H, generator=g).to("cuda", torch.bfloat16)
    gr = torch.randn(rows, H, generator=g).to("cuda", torch.bfloat16)
    x, w, b = (t.clone().requires_grad_(True) for t in (x0, w0, b0))
    y, r = ops.layer_norm_residual(x, w, b)
    torch.autograd.backward([y, r], [gy, gr])
    xf, wf, bf = (t.float().clone().requires_grad_(True) for t in (x0, w0, b0))
    yf = F.layer_norm(xf, (H,), wf, bf, 1e-5)
    torch.autograd.backward([yf, xf], [gy.float(), gr.float()])
    assert torch.allclose(y.float(), yf, atol=3e-2, rtol=2e-2)
    assert torch.equal(r, x0)

    def rel(a, b):
        return ((a.float() - b).norm() / b.norm()).item()
    assert rel(x.grad, xf.grad) < 1e-2
    assert rel(w.grad, wf.grad) < 1e-2 and rel(b.grad, bf.grad) < 1e-2


def test_gpt_block_has_no_separate_residual_add_in_backward():
    """The block's backward: one LayerNorm backward node per norm takes both gradient contributions
    (no AddBackward joining the residual stream's two paths)."""
    from kubeflow_rm_amd.models import GPT, GPTConfig
    cfg = GPTConfig(vocab_size=512, d_model=256, n_layers=1, n_heads=4, d_ff=1024, max_seq=128)
    m = GPT(cfg, device="cuda")
    idx = torch.randint(0, 512, (2, 128), device="cuda")
    x = F.embedding(idx, m.tok) + m.pos[:128]
    out = m.blocks[0](x)
    seen, stack, names = set(), [out.grad_fn], []
    while stack:
        fn = stack.pop()
        if fn is None or fn in seen:
            continue
        seen.add(fn)
        names.append(type(fn).__name__)
        stack.extend(f for f, _ in fn.next_functions)
    assert names.count("_LayerNormResidualBackward") == 2, names
    # the embedding sum is the only add left on the way into the block
    assert names.count("AddBackward0") == 1, names
