"""Numerics of the hand-written gfx950 kernels against plain PyTorch fp32 references."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rand(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return ((torch.rand(*shape, generator=g, device="cuda") * 2 - 1) * scale).to(torch.bfloat16)


def _ref_gemm(a, b, bias=None, act="none", residual=None, alpha=1.0):
    c = alpha * (a.float() @ b.float().transpose(-1, -2))
    if bias is not None:
        c = c + bias.float()
    if act == "relu":
        c = torch.relu(c)
    elif act in ("gelu", "gelu_tanh"):
        c = torch.nn.functional.gelu(c, approximate="tanh")
    elif act == "silu":
        c = torch.nn.functional.silu(c)
    if residual is not None:
        c = c + residual.float()
    return c


def _assert_close(out, ref, K):
    err = (out.float() - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-6
    # bf16 output rounding (2^-8 relative) + fp32 accumulation order
    assert err <= 1e-2 * scale + 1e-2, f"max err {err} vs scale {scale} (K={K})"


def test_native_library_loaded():
    from kubeflow_rm_amd import ops
    assert "gfx950" in ops.build_info()


@pytest.mark.parametrize("variant", ["fast", "pipe", "pipe_sched", "w4", "w4s", "auto"])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (256, 256, 128), (512, 768, 192), (512, 768, 1024),
                                   (1024, 1024, 4096), (4096, 4096, 4096)])
def test_gemm_fast_path(M, N, K, variant):
    from kubeflow_rm_amd.ops import gemm_nt
    a, b = _rand(M, K, seed=1), _rand(N, K, seed=2)
    out = gemm_nt(a, b, variant=variant)
    torch.cuda.synchronize()
    _assert_close(out, _ref_gemm(a, b), K)


@pytest.mark.parametrize("M,N,K", [(4096, 4096, 16448), (4096, 8192, 12288)])
def test_gemm_superblock_raster_past_the_mall(M, N, K):
    """Operands past 256 MiB take the 16 x 16-tile superblock raster (gemm_w4.h KFW4_SUPER): every
    output tile written once, from the right A rows and B columns."""
    from kubeflow_rm_amd.ops import gemm_nt
    assert (M + N) * K * 2 > 256 << 20 and M % 4096 == 0 and N % 4096 == 0
    a, b = _rand(M, K, seed=11), _rand(N, K, seed=12)
    out = gemm_nt(a, b, variant="w4")
    torch.cuda.synchronize()
    rows = torch.arange(7, M, 61, device="cuda")  # rows in every 256-row tile row; all N columns
    _assert_close(out.index_select(0, rows), _ref_gemm(a.index_select(0, rows), b), K)
    cols = torch.arange(5, N, 53, device="cuda")
    _assert_close(out.index_select(1, cols), _ref_gemm(a, b.index_select(0, cols)), K)


def test_gemm_identity_asymmetric():
    """A = I with an asymmetric B catches a transposed C write (cdna_hip_programming.md §3)."""
    from kubeflow_rm_amd.ops import gemm_nt
    n = 256
    eye = torch.eye(n, device="cuda", dtype=torch.bfloat16)
    b = (torch.arange(n * n, device="cuda", dtype=torch.float32).reshape(n, n) % 97 - 48).to(torch.bfloat16)
    for v in ("fast", "pipe", "pipe_sched", "w4", "w4s"):
        out = gemm_nt(eye, b, variant=v)  # = I @ b^T = b^T
        assert torch.equal(out.float(), b.float().t())
        out2 = gemm_nt(b, eye, variant=v)  # = b
        assert torch.equal(out2.float(), b.float())


@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (17, 33, 65), (100, 300, 77), (257, 255, 130), (1000, 512, 64)])
def test_gemm_generic_path(M, N, K):
    from kubeflow_rm_amd.ops import gemm_nt
    a, b = _rand(M, K, seed=3), _rand(N, K, seed=4)
    out = gemm_nt(a, b)
    torch.cuda.synchronize()
    _assert_close(out, _ref_gemm(a, b), K)


@pytest.mark.parametrize("M,N,K", [(3000, 2900, 1000), (4000, 4000, 4000), (1030, 4100, 1000), (2000, 2000, 2000)])
def test_gemm_unaligned_shapes_on_padded_tiles(M, N, K):
    """Off-tile shapes above the padding threshold run zero-padded on the tiled kernels; the fused
    epilogue (bias, activation) and the residual are padded with them and the corner copied out."""
    from kubeflow_rm_amd.ops import gemm_nt
    a, b, bias = _rand(M, K, seed=21), _rand(N, K, seed=22), _rand(N, seed=23)
    out = gemm_nt(a, b, bias=bias, act="silu", alpha=0.5)
    _assert_close(out, _ref_gemm(a, b, bias, "silu", alpha=0.5), K)
    r = _rand(M, N, seed=24)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    assert gemm_nt(a, b, residual=r, out=out) is out
    _assert_close(out, _ref_gemm(a, b, residual=r), K)
    a3, b3 = _rand(2, 1500, 1000, seed=25), _rand(2, 1700, 1000, seed=26)  # batched, above the threshold
    _assert_close(gemm_nt(a3, b3), _ref_gemm(a3, b3), 1000)
    # only N off the grid (an lm_head with an odd vocabulary): A is used in place
    a2, b2 = _rand(2048, 768, seed=27), _rand(5003, 768, seed=28)
    _assert_close(gemm_nt(a2, b2), _ref_gemm(a2, b2), 768)
    # only K off the grid: the tiled kernel writes straight into the output
    a4, b4 = _rand(2048, 1000, seed=29), _rand(2048, 1000, seed=30)
    _assert_close(gemm_nt(a4, b4, bias=bias[:0].new_zeros(2048)), _ref_gemm(a4, b4), 1000)


@pytest.mark.parametrize("variant", ["fast", "pipe", "generic", "w4", "w4s"])
@pytest.mark.parametrize("act", ["none", "relu", "gelu_tanh", "silu"])
def test_gemm_epilogue(variant, act):
    from kubeflow_rm_amd.ops import gemm_nt
    M, N, K = 512, 512, 256
    a, b, bias = _rand(M, K, seed=5), _rand(N, K, seed=6), _rand(N, seed=7)
    out = gemm_nt(a, b, bias=bias, act=act, alpha=0.5, variant=variant)
    _assert_close(out, _ref_gemm(a, b, bias, act, alpha=0.5), K)


@pytest.mark.parametrize("variant", ["fast", "pipe", "generic", "w4", "w4s"])
def test_gemm_residual_and_batch(variant):
    from kubeflow_rm_amd.ops import gemm_nt
    B, M, N, K = 3, 256, 512, 128
    a, b, r = _rand(B, M, K, seed=8), _rand(B, N, K, seed=9), _rand(B, M, N, seed=10)
    out = gemm_nt(a, b, residual=r, variant=variant)
    _assert_close(out, _ref_gemm(a, b, residual=r), K)


def test_linear_autograd():
    from kubeflow_rm_amd.ops import linear
    x = _rand(4, 64, 256, seed=11).requires_grad_(True)
    w = _rand(512, 256, seed=12, scale=0.1).requires_grad_(True)
    bias = _rand(512, seed=13).requires_grad_(True)
    y = linear(x, w, bias, act="gelu_tanh")
    g = _rand(*y.shape, seed=14)
    y.backward(g)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, bias))
    yr = torch.nn.functional.gelu(xr @ wr.t() + br, approximate="tanh")
    yr.backward(g.float())
    for got, ref in ((y, yr), (x.grad, xr.grad), (w.grad, wr.grad), (bias.grad, br.grad)):
        err = (got.float() - ref).abs().max().item()
        assert err <= 2e-2 * (ref.abs().max().item() + 1e-3) + 2e-2, err


@pytest.mark.parametrize("rows,H", [(64, 512), (128, 4096), (33, 8192), (10, 1000), (7, 3), (65, 1536), (40, 2560),
                                    (37, 3072), (19, 5120), (23, 6144), (50, 768), (9, 256), (31, 1280)])
def test_layernorm_fwd_bwd(rows, H):
    from kubeflow_rm_amd.ops import layer_norm
    x = (_rand(rows, H, seed=15, scale=3.0).float() + 1.5).to(torch.bfloat16).requires_grad_(True)
    w = _rand(H, seed=16).requires_grad_(True)
    b = _rand(H, seed=17).requires_grad_(True)
    y = layer_norm(x, w, b, 1e-5)
    gy = _rand(rows, H, seed=18)
    y.backward(gy)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yr = torch.nn.functional.layer_norm(xr, (H,), wr, br, 1e-5)
    yr.backward(gy.float())
    assert (y.float() - yr).abs().max().item() < 5e-2
    assert (x.grad.float() - xr.grad).abs().max().item() < 5e-2 * (xr.grad.abs().max().item() + 1)
    assert (w.grad.float() - wr.grad).abs().max().item() < 2e-2 * (wr.grad.abs().max().item() + 1)
    assert (b.grad.float() - br.grad).abs().max().item() < 2e-2 * (br.grad.abs().max().item() + 1)


@pytest.mark.parametrize("rows,H", [(8192, 2048), (3001, 2048), (5000, 1024), (777, 768), (2049, 1536), (300, 1280)])
def test_layernorm_backward_fused_with_residual(rows, H):
    """The one-pass backward (layernorm_bf16.hip ln_bwd_fused: dx, the residual gradient folded into
    its store, and the dgamma / dbeta partials from the same reads) at model widths and row counts
    that give every wave several rows and the last block a short chunk; vs fp32 autograd."""
    from kubeflow_rm_amd.ops import layernorm as LN
    x = (_rand(rows, H, seed=61, scale=2.0).float() + 0.5).to(torch.bfloat16).requires_grad_(True)
    w = _rand(H, seed=62).requires_grad_(True)
    b = _rand(H, seed=63).requires_grad_(True)
    y, r = LN.layer_norm_residual(x, w, b, 1e-5)
    gy, gr = _rand(rows, H, seed=64), _rand(rows, H, seed=65)
    torch.autograd.backward((y, r), (gy, gr))
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yr = torch.nn.functional.layer_norm(xr, (H,), wr, br, 1e-5)
    torch.autograd.backward((yr, xr * 1.0), (gy.float(), gr.float()))
    assert (x.grad.float() - xr.grad).abs().max().item() < 5e-2 * (xr.grad.abs().max().item() + 1)
    # dgamma / dbeta sum `rows` products: bf16 output rounding on values of size ~sqrt(rows)
    assert (w.grad.float() - wr.grad).abs().max().item() < 1e-2 * (wr.grad.abs().max().item() + 1)
    assert (b.grad.float() - br.grad).abs().max().item() < 1e-2 * (br.grad.abs().max().item() + 1)


@pytest.mark.parametrize("rows,H,rms", [(6001, 4096, False), (8192, 4096, False), (12289, 1024, False),
                                        (6001, 4096, True), (8192, 8192, False), (37, 8192, False),
                                        (4099, 8192, True), (20000, 8192, False), (32768, 512, False)])
def test_norm_forward_launch_paths(rows, H, rms):
    """The forward's launch policy (layernorm_bf16.hip norm_fwd): 1-2 generations of resident waves
    take the streaming kernel (resident waves, next row prefetched, gamma/beta in LDS) — 6001 / 8192
    rows at hidden 4096, 12289 at 1024, odd counts leave waves with one row fewer; hidden 8192 up to
    two generations the rolling-reload stream (37, 4099, 8192 rows), beyond it the gamma/beta-prefetch
    kernel (20000); 32768 x 512 the one-shot kernel. Output and saved statistics vs fp32."""
    from kubeflow_rm_amd import ops
    x = (_rand(rows, H, seed=41, scale=2.0).float() + 0.5).to(torch.bfloat16)
    w, b = _rand(H, seed=42), _rand(H, seed=43)
    xf = x.float()
    if rms:
        y = ops.rms_norm(x, w, 1e-6)
        ref = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-6) * w.float()
        assert (y.float() - ref).abs().max().item() < 3e-2
        return
    y, mean, rstd = ops.layer_norm_fwd(x, w, b, save_stats=True)
    ref = torch.nn.functional.layer_norm(xf, (H,), w.float(), b.float(), 1e-5)
    assert (y.float() - ref).abs().max().item() < 5e-2
    assert torch.allclose(mean.float().view(-1), xf.mean(-1), atol=1e-4, rtol=1e-4)
    assert torch.allclose(rstd.float().view(-1), torch.rsqrt(xf.var(-1, unbiased=False) + 1e-5), atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("rows,H", [(64, 4096), (5, 777), (41, 3072), (9, 6144), (26, 768)])
def test_rmsnorm(rows, H):
    from kubeflow_rm_amd.ops import rms_norm
    x, w = _rand(rows, H, seed=19), _rand(H, seed=20)
    y = rms_norm(x, w, 1e-6)
    xf = x.float()
    ref = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-6) * w.float()
    assert (y.float() - ref).abs().max().item() < 3e-2
    # backward (dx, dw) against fp32 autograd
    xg, wg = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    gy = _rand(rows, H, seed=31)
    rms_norm(xg, wg, 1e-6).backward(gy)
    xr, wr = x.float().requires_grad_(True), w.float().requires_grad_(True)
    (xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6) * wr).backward(gy.float())
    assert (xg.grad.float() - xr.grad).abs().max().item() <= 2e-2 * xr.grad.abs().max().item() + 1e-2
    assert (wg.grad.float() - wr.grad).abs().max().item() <= 2e-2 * wr.grad.abs().max().item() + 1e-2


def test_gemm_w4_output_rows_off_16b():
    """An output with ldc % 8 != 0 (rows off the 16-B grid) takes the w4 epilogue's element-wise
    path on the explicit variants and auto alike (same result, nothing written past the row)."""
    from kubeflow_rm_amd.ops import gemm_nt
    M = N = K = 512
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    big = torch.zeros(M, N + 4, device="cuda", dtype=torch.bfloat16)
    out = big[:, :N]
    ref = (a.float() @ b.float().t())
    for v in ("w4", "w4s", "auto"):
        out.zero_()
        gemm_nt(a, b, out=out, variant=v)
        torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-1)
    assert torch.all(big[:, N:] == 0)  # nothing written past the row


def test_gemm_rejects_bad_out_tensor():
    """a user-supplied ``out`` of the wrong dtype / shape / device must be refused, not
    filled with bf16 bit patterns."""
    from kubeflow_rm_amd import ops
    a, b = _rand(256, 64), _rand(256, 64, seed=1)
    with pytest.raises(TypeError):
        ops.gemm_nt(a, b, out=torch.empty(256, 256, device="cuda", dtype=torch.float32))
    with pytest.raises(ValueError):
        ops.gemm_nt(a, b, out=torch.empty(256 * 256, device="cuda", dtype=torch.bfloat16))
    with pytest.raises(ValueError):
        ops.gemm_nt(a, b, out=torch.empty(256, 512, device="cuda", dtype=torch.bfloat16)[:, ::2])
    out = torch.empty(256, 256, device="cuda", dtype=torch.bfloat16)
    assert ops.gemm_nt(a, b, out=out) is out


# ---- r3: in-kernel edge tiles, transposed operand layouts, pre-activation output, act-grad ----------

@pytest.mark.parametrize("M,N,K", [(1500, 1500, 1500), (4000, 4000, 4000), (3000, 3000, 3000), (8000, 8000, 8000),
                                   (257, 264, 72), (129, 136, 8), (130, 1000, 520), (640, 384, 1000),
                                   (128, 128, 64), (300, 200, 4104)])
def test_gemm_edge_tiles_in_kernel(M, N, K):
    """Off-grid M / N (shifted last tile, masked stores) and K (zero-filled first K tile) on the w4
    kernels, both tile sizes, with the fused epilogue."""
    from kubeflow_rm_amd.ops import gemm_nt
    a, b, bias = _rand(M, K, seed=41), _rand(N, K, seed=42), _rand(N, seed=43)
    from kubeflow_rm_amd.ops.gemm import _w4_nt_shape
    for v in ("w4", "w4s", "auto"):
        if v != "auto" and (not _w4_nt_shape(M, N, K) or (v == "w4" and (M < 256 or N < 256))):
            continue  # outside the tiled contract: auto pads up to it
        out = gemm_nt(a, b, bias=bias, act="gelu_tanh", alpha=0.5, variant=v)
        _assert_close(out, _ref_gemm(a, b, bias, "gelu_tanh", alpha=0.5), K)
    r = _rand(M, N, seed=44)
    _assert_close(gemm_nt(a, b, residual=r), _ref_gemm(a, b, residual=r), K)


def test_gemm_edge_store_mask_leaves_neighbours():
    """The shifted edge tile recomputes rows/columns its neighbour owns: with an in-place residual
    (out aliases R) a double store would add the residual twice."""
    from kubeflow_rm_amd.ops import gemm_nt
    M, N, K = 300, 392, 200
    a, b = _rand(M, K, seed=45), _rand(N, K, seed=46)
    c = _rand(M, N, seed=47)
    ref = _ref_gemm(a, b, residual=c)
    gemm_nt(a, b, residual=c, out=c)
    _assert_close(c, ref, K)


def _ref_mm(a, b, ta, tb, alpha=1.0, residual=None):
    af = a.float().transpose(-1, -2) if ta else a.float()
    bf = b.float().transpose(-1, -2) if tb else b.float()
    c = alpha * (af @ bf)
    return c + residual.float() if residual is not None else c


@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (True, True), (False, True)])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 1024), (4096, 4096, 4096), (1500, 1000, 776),
                                   (136, 128, 100), (2048, 1024, 8192)])
def test_mm_operand_layouts(M, N, K, ta, tb):
    """k-major operands through ds_read_b64_tr_b16 (no transposed copies) vs fp32."""
    from kubeflow_rm_amd.ops import mm
    a = _rand(*((K, M) if ta else (M, K)), seed=51)
    b = _rand(*((N, K) if tb else (K, N)), seed=52)
    out = mm(a, b, trans_a=ta, trans_b=tb)
    _assert_close(out, _ref_mm(a, b, ta, tb), K)
    # accumulate in place (gradient accumulation): out += alpha * op(a) op(b)
    ref = _ref_mm(a, b, ta, tb, alpha=0.25, residual=out)
    mm(a, b, trans_a=ta, trans_b=tb, out=out, residual=out, alpha=0.25)
    _assert_close(out, ref, K)


@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (True, True)])
def test_mm_identity_asymmetric(ta, tb):
    """A = I with an asymmetric B through each layout: catches a transposed fragment or C write."""
    from kubeflow_rm_amd.ops import mm
    n = 384
    eye = torch.eye(n, device="cuda", dtype=torch.bfloat16)
    b = (torch.arange(n * n, device="cuda", dtype=torch.float32).reshape(n, n) % 97 - 48).to(torch.bfloat16)
    out = mm(eye, b, trans_a=ta, trans_b=tb)
    assert torch.equal(out.float(), (b.float().t() if tb else b.float()))
    out2 = mm(b, eye, trans_a=ta, trans_b=tb)
    assert torch.equal(out2.float(), (b.float().t() if ta else b.float()))


def test_mm_batched_layouts():
    from kubeflow_rm_amd.ops import mm
    a, b = _rand(3, 512, 256, seed=53), _rand(3, 512, 384, seed=54)
    _assert_close(mm(a, b, trans_a=True), _ref_mm(a, b, True, False), 512)


@pytest.mark.parametrize("act", ["gelu_tanh", "silu"])
def test_gemm_preactivation_output(act):
    from kubeflow_rm_amd.ops import gemm_nt_preact
    M, N, K = 1000, 1536, 520
    x, w, bias = _rand(M, K, seed=55), _rand(N, K, seed=56), _rand(N, seed=57)
    y, z = gemm_nt_preact(x, w, bias, act)
    _assert_close(z, _ref_gemm(x, w, bias), K)
    _assert_close(y, _ref_gemm(x, w, bias, act), K)


@pytest.mark.parametrize("act", ["none", "relu", "gelu_tanh", "silu"])
@pytest.mark.parametrize("rows,cols", [(8192, 4096), (100, 136), (1, 8)])
def test_act_grad_fused(act, rows, cols):
    from kubeflow_rm_amd.ops import act_grad
    gy, z = _rand(rows, cols, seed=58), _rand(rows, cols, seed=59, scale=3.0)
    g, db = act_grad(gy, z, act, True)
    zf = z.float().requires_grad_(True)
    F = torch.nn.functional
    f = {"none": lambda t: t, "relu": torch.relu, "gelu_tanh": lambda t: F.gelu(t, approximate="tanh"),
         "silu": F.silu}[act](zf)
    (gr,) = torch.autograd.grad(f, zf, gy.float())
    assert (g.float() - gr).abs().max().item() <= 1e-2 * (gr.abs().max().item() + 1e-3) + 1e-2
    dbr = g.float().sum(0)
    assert (db - dbr).abs().max().item() <= 1e-3 * (dbr.abs().max().item() + 1.0)
    # the bias grad written as bf16 by the kernel (the linear backward's form): fp32 sums, one rounding
    _, db16 = act_grad(gy, z, act, True, db_dtype=torch.bfloat16)
    assert db16.dtype == torch.bfloat16
    assert (db16.float() - dbr).abs().max().item() <= 2 ** -8 * dbr.abs().max().item() + 1e-3 * (dbr.abs().max().item() + 1.0)


@pytest.mark.parametrize("act", ["none", "relu", "gelu_tanh", "silu"])
@pytest.mark.parametrize("shape", [(4, 256, 1024, 512), (1, 1000, 776, 1032)])
def test_linear_backward_layouts(act, shape):
    """Full linear fwd+bwd: pre-activation from the forward epilogue, fused act/bias grad, dgrad and
    wgrad on the transposed-layout kernels — all vs fp32 autograd."""
    from kubeflow_rm_amd.ops import linear
    B, T, K, N = shape
    x = _rand(B, T, K, seed=61).requires_grad_(True)
    w = _rand(N, K, seed=62, scale=0.05).requires_grad_(True)
    bias = _rand(N, seed=63).requires_grad_(True)
    y = linear(x, w, bias, act=act)
    g = _rand(*y.shape, seed=64)
    y.backward(g)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, bias))
    F = torch.nn.functional
    pre = xr @ wr.t() + br
    yr = {"none": lambda t: t, "relu": torch.relu, "gelu_tanh": lambda t: F.gelu(t, approximate="tanh"),
          "silu": F.silu}[act](pre)
    yr.backward(g.float())
    for got, ref in ((y, yr), (x.grad, xr.grad), (w.grad, wr.grad), (bias.grad, br.grad)):
        err = (got.float() - ref).abs().max().item()
        assert err <= 2e-2 * (ref.abs().max().item() + 1e-3) + 2e-2, err


@pytest.mark.parametrize("M,N,K", [(1000, 1000, 4104), (1024, 1024, 4096), (1000, 1504, 6152), (136, 128, 2120),
                                   (512, 768, 8192), (768, 3072, 16384)])
def test_splitk_plan_and_numerics(M, N, K):
    """Split-K (fp32 partials + reduce) for under-filled problems: the plan splits, the result
    matches fp32 and the last (partial) split is zero-filled, through every operand layout."""
    from kubeflow_rm_amd.ops import gemm_nt, mm
    from kubeflow_rm_amd.ops.gemm import splitk_plan
    splits, kper = splitk_plan(M, N, K)
    assert splits >= 2 and kper % 64 == 0 and (splits - 1) * kper < K <= splits * kper
    a, b = _rand(M, K, seed=71), _rand(N, K, seed=72)
    _assert_close(gemm_nt(a, b), _ref_gemm(a, b), K)
    for ta, tb in ((True, False), (True, True), (False, True)):
        aa = a.t().contiguous() if ta else a
        bb = b if tb else b.t().contiguous()
        out = mm(aa, bb, trans_a=ta, trans_b=tb)
        _assert_close(out, _ref_mm(aa, bb, ta, tb), K)
        ref = _ref_mm(aa, bb, ta, tb, alpha=0.5, residual=out)
        mm(aa, bb, trans_a=ta, trans_b=tb, out=out, residual=out, alpha=0.5)
        _assert_close(out, ref, K)


@pytest.mark.parametrize("act", ["none", "relu", "gelu_tanh", "silu"])
def test_splitk_epilogues(act):
    """bias / activation / residual / pre-activation output run in the split-K reduce."""
    from kubeflow_rm_amd.ops import gemm_nt, gemm_nt_preact
    from kubeflow_rm_amd.ops.gemm import splitk_plan
    M, N, K = 384, 512, 2056
    assert splitk_plan(M, N, K) is not None
    a, b, bias = _rand(M, K, seed=73), _rand(N, K, seed=74, scale=0.1), _rand(N, seed=75)
    _assert_close(gemm_nt(a, b, bias=bias, act=act, alpha=0.5), _ref_gemm(a, b, bias, act, alpha=0.5), K)
    if act == "none":
        r = _rand(M, N, seed=76)
        _assert_close(gemm_nt(a, b, bias=bias, residual=r), _ref_gemm(a, b, bias, residual=r), K)
    if act in ("gelu_tanh", "silu"):
        y, z = gemm_nt_preact(a, b, bias, act)
        _assert_close(z, _ref_gemm(a, b, bias), K)
        _assert_close(y, _ref_gemm(a, b, bias, act), K)


def test_splitk_batched_matches_unsplit():
    from kubeflow_rm_amd.ops import gemm, gemm_nt
    a, b = _rand(2, 256, 4096, seed=77), _rand(2, 256, 4096, seed=78)
    assert gemm.splitk_plan(256, 256, 4096, 2) is not None
    split = gemm_nt(a, b)
    gemm.SPLITK = False
    try:
        whole = gemm_nt(a, b)
    finally:
        gemm.SPLITK = True
    ref = _ref_gemm(a, b)
    _assert_close(split, ref, 4096)
    _assert_close(whole, ref, 4096)


@pytest.mark.parametrize("M,N,K", [(4096, 2048, 8192), (4000, 1800, 8200), (3072, 768, 32768)])
def test_fixk_plan_and_numerics(M, N, K):
    """Split-K with the in-kernel fixup (256 tile, the last split of each tile adds the others' fp32
    partials): the plan takes it, every layout it runs (NT, wgrad TN-T, dgrad) matches fp32 and the
    unsplit kernel, in-place accumulation (residual = out) works, and the arrival counters are back
    to zero after every call."""
    from kubeflow_rm_amd.ops import gemm, gemm_nt, mm
    splits, kper = gemm.fixk_plan(M, N, K)
    assert splits >= 2 and kper % 64 == 0 and (splits - 1) * kper < K <= splits * kper
    a, b = _rand(M, K, seed=91), _rand(N, K, seed=92)
    ref = _ref_gemm(a, b)
    _assert_close(gemm_nt(a, b), ref, K)
    for ta, tb in ((True, True), (False, True)):
        aa = a.t().contiguous() if ta else a
        bb = b if tb else b.t().contiguous()
        out = mm(aa, bb, trans_a=ta, trans_b=tb)
        _assert_close(out, _ref_mm(aa, bb, ta, tb), K)
        gemm.FIXK = False
        try:
            whole = mm(aa, bb, trans_a=ta, trans_b=tb)
        finally:
            gemm.FIXK = True
        err = (out.float() - whole.float()).abs().max().item()
        assert err <= 1e-2 * (whole.float().abs().max().item() + 1e-3), err
        ref2 = _ref_mm(aa, bb, ta, tb, alpha=0.5, residual=out)
        mm(aa, bb, trans_a=ta, trans_b=tb, out=out, residual=out, alpha=0.5)
        _assert_close(out, ref2, K)
    torch.cuda.synchronize()
    for w, cnt in gemm._fixk_ws.values():
        assert int(cnt.abs().sum().item()) == 0


@pytest.mark.parametrize("S", [2, 3, 5, 16])
def test_fixk_forced_splits_batched(S):
    """Any split count, batched operands, repeated launches over the same workspace."""
    from kubeflow_rm_amd.ops import gemm, mm
    a, b = _rand(2, 4096, 512, seed=93), _rand(2, 4096, 768, seed=94)
    gemm.FIXK_SPLITS = S
    try:
        assert gemm.fixk_plan(512, 768, 4096, 2)[0] == S
        for _ in range(3):
            out = mm(a, b, trans_a=True)
            _assert_close(out, _ref_mm(a, b, True, False), 4096)
    finally:
        gemm.FIXK_SPLITS = None


@pytest.fixture
def streamk_on():
    from kubeflow_rm_amd.ops import gemm
    old = gemm.STREAMK
    gemm.STREAMK = True
    yield
    gemm.STREAMK = old


@pytest.mark.parametrize("M,N,K", [(3072, 3072, 8192), (3000, 3000, 3000), (6144, 2048, 4096), (1000, 5000, 3000),
                                   (2304, 2304, 1024), (1024, 8192, 8200)])
def test_streamk_plan_and_numerics(M, N, K, streamk_on):
    """Stream-K (persistent grid, the last partial wave's K-tiles shared over all CUs): the plan
    picks it, the result matches fp32 (edge tiles, K tails, segments crossing tiles) and the plain
    kernel's output."""
    from kubeflow_rm_amd.ops import gemm, gemm_nt
    grid, splits = gemm.streamk_plan(M, N, K)
    assert grid == 256 and splits >= 2
    a, b = _rand(M, K, seed=81), _rand(N, K, seed=82)
    sk = gemm_nt(a, b)
    _assert_close(sk, _ref_gemm(a, b), K)
    gemm.STREAMK = False
    dp = gemm_nt(a, b)
    err = (sk.float() - dp.float()).abs().max().item()
    assert err <= 1e-2 * (dp.float().abs().max().item() + 1e-3), err


@pytest.mark.parametrize("act", ["none", "gelu_tanh", "silu", "relu"])
def test_streamk_epilogues(act, streamk_on):
    """bias / activation / residual on the stream-K owner's epilogue (adds the producers' fp32
    partials first); the pre-activation output (plain kernel) next to it."""
    from kubeflow_rm_amd.ops import gemm, gemm_nt, gemm_nt_preact
    M, N, K = 3072, 3072, 4096
    assert gemm.streamk_plan(M, N, K) is not None
    a, b, bias = _rand(M, K, seed=83), _rand(N, K, seed=84, scale=0.1), _rand(N, seed=85)
    _assert_close(gemm_nt(a, b, bias=bias, act=act, alpha=0.5), _ref_gemm(a, b, bias, act, alpha=0.5), K)
    if act == "none":
        r = _rand(M, N, seed=86)
        _assert_close(gemm_nt(a, b, bias=bias, residual=r), _ref_gemm(a, b, bias, residual=r), K)
    if act in ("gelu_tanh", "silu"):
        y, z = gemm_nt_preact(a, b, bias, act)
        _assert_close(z, _ref_gemm(a, b, bias), K)
        _assert_close(y, _ref_gemm(a, b, bias, act), K)


def test_streamk_deadline_path_and_epochs():
    """Owners whose producers' partials never arrive (test mode: producers publish a flag value no
    owner accepts) recompute those splits after the deadline, and the result is still exact; a
    grid of 4x the CUs (not co-resident) and repeated calls (new epochs over the same flag words)
    stay correct."""
    from kubeflow_rm_amd.ops import gemm
    M, N, K = 2304, 2304, 2048  # 81 tiles, 32 K-tiles each
    a, b = _rand(M, K, seed=87), _rand(N, K, seed=88)
    ref = _ref_gemm(a, b)
    c = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    for plan, force in (((256, 3), True), ((256, 3), False), ((1024, 8), False), ((256, 4), False), ((256, 3), False)):
        c.zero_()
        rc = gemm._streamk(a, b, c, M, N, K, K, K, N, plan, bias=None, r_ptr=None, ldr=0, aux=None, alpha=1.0,
                           act="none", _force_deadline=force)
        assert rc == 0
        _assert_close(c, ref, K)


@pytest.mark.parametrize("M,N,K", [(1500, 1500, 1504), (1000, 1001, 512), (300, 130, 2048), (2000, 1499, 1000)])
@pytest.mark.parametrize("v", ["w4", "w4s"])
def test_gemm_odd_output_width(M, N, K, v):
    """N (and so the shifted edge tile's n0) off the 8-column grid: the element-wise epilogue path,
    every epilogue (bias, activation, pre-activation output, in-place residual)."""
    from kubeflow_rm_amd.ops import gemm_nt, gemm_nt_preact
    if v == "w4" and (M < 256 or N < 256):
        pytest.skip("256 tile needs M, N >= 256")
    a, b, bias = _rand(M, K, seed=81), _rand(N, K, seed=82, scale=0.2), _rand(N, seed=83)
    for act in ("none", "relu", "silu"):
        _assert_close(gemm_nt(a, b, bias=bias, act=act, alpha=0.5, variant=v),
                      _ref_gemm(a, b, bias, act, alpha=0.5), K)
    c = _rand(M, N, seed=84)
    ref = _ref_gemm(a, b, bias, residual=c)
    gemm_nt(a, b, bias=bias, residual=c, out=c, variant=v)
    _assert_close(c, ref, K)
    y, z = gemm_nt_preact(a, b, bias, "gelu_tanh")
    _assert_close(z, _ref_gemm(a, b, bias), K)
    _assert_close(y, _ref_gemm(a, b, bias, "gelu_tanh"), K)


def test_gemm_odd_output_stride_leaves_padding():
    """C as a column slice of a wider buffer (ldc = 1503, rows off 16 B): the odd path writes exactly
    the [M, N] window."""
    from kubeflow_rm_amd.ops import gemm_nt
    M, N, K = 640, 1496, 256
    a, b = _rand(M, K, seed=85), _rand(N, K, seed=86)
    big = torch.full((M, 1503), 7.0, device="cuda", dtype=torch.bfloat16)
    out = big[:, 3:3 + N]
    gemm_nt(a, b, out=out, variant="w4")
    _assert_close(out, _ref_gemm(a, b), K)
    assert torch.all(big[:, :3] == 7.0) and torch.all(big[:, 3 + N:] == 7.0)


@pytest.mark.parametrize("M,N,K", [(1500, 1500, 1500), (1000, 1000, 1001), (257, 300, 77), (4000, 4000, 3998)])
def test_gemm_k_off_grid_packed(M, N, K):
    """K % 8 != 0: both operands packed (zero tail) by one kfamd_pad_k_bf16 launch, then the tiled
    kernel; also batched."""
    from kubeflow_rm_amd.ops import gemm_nt
    from kubeflow_rm_amd.ops.gemm import pad_k
    a, b, bias = _rand(M, K, seed=87), _rand(N, K, seed=88), _rand(N, seed=89)
    ap, bp = pad_k(a, b, (K + 7) // 8 * 8)
    assert torch.equal(ap[:, :K], a) and torch.all(ap[:, K:] == 0) and torch.equal(bp[:, :K], b)
    _assert_close(gemm_nt(a, b, bias=bias, act="gelu_tanh"), _ref_gemm(a, b, bias, "gelu_tanh"), K)
    a3, b3 = _rand(2, 256, K, seed=90), _rand(2, 384, K, seed=91)
    _assert_close(gemm_nt(a3, b3), _ref_gemm(a3, b3), K)


@pytest.mark.parametrize("bias", [True, False])
def test_linear_residual_in_epilogue(bias):
    """y = x W^T + b + r with r in the GEMM epilogue; dr = dy, the other grads as without r."""
    from kubeflow_rm_amd.ops import linear
    x = _rand(2, 300, 512, seed=92).requires_grad_(True)
    w = _rand(768, 512, seed=93, scale=0.05).requires_grad_(True)
    b = _rand(768, seed=94).requires_grad_(True) if bias else None
    r = _rand(2, 300, 768, seed=95).requires_grad_(True)
    y = linear(x, w, b, residual=r)
    g = _rand(*y.shape, seed=96)
    y.backward(g)
    xr, wr, rr = (t.detach().float().requires_grad_(True) for t in (x, w, r))
    br = b.detach().float().requires_grad_(True) if bias else None
    yr = xr @ wr.t() + (br if bias else 0) + rr
    yr.backward(g.float())
    pairs = [(y, yr), (x.grad, xr.grad), (w.grad, wr.grad), (r.grad, rr.grad)] + ([(b.grad, br.grad)] if bias else [])
    for got, ref in pairs:
        err = (got.float() - ref).abs().max().item()
        assert err <= 2e-2 * (ref.abs().max().item() + 1e-3) + 2e-2, err


@pytest.mark.parametrize("act", ["relu", "gelu_tanh", "silu"])
def test_linear_activation_with_residual_grads(act):
    """y = act(x W^T + b) + r. The activation's derivative must come from the
    pre-residual values: the residual (here offset by +2, so y > 0 almost everywhere) must not leak
    into relu's mask. Every gradient against F.linear + act + add in fp32."""
    from kubeflow_rm_amd.ops import linear
    F = torch.nn.functional
    x = _rand(2, 256, 512, seed=101).requires_grad_(True)
    w = _rand(768, 512, seed=102, scale=0.05).requires_grad_(True)
    b = _rand(768, seed=103).requires_grad_(True)
    r = (_rand(2, 256, 768, seed=104).float() + 2.0).to(torch.bfloat16).requires_grad_(True)
    y = linear(x, w, b, act=act, residual=r)
    g = _rand(*y.shape, seed=105)
    y.backward(g)
    xr, wr, br, rr = (t.detach().float().requires_grad_(True) for t in (x, w, b, r))
    zr = F.linear(xr, wr, br)
    ar = torch.relu(zr) if act == "relu" else (F.gelu(zr, approximate="tanh") if act == "gelu_tanh" else F.silu(zr))
    yr = ar + rr
    yr.backward(g.float())
    for got, ref in [(y, yr), (x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad), (r.grad, rr.grad)]:
        err = (got.float() - ref).abs().max().item()
        assert err <= 2e-2 * (ref.abs().max().item() + 1e-3) + 2e-2, (act, err)


@pytest.mark.parametrize("act", ["gelu_tanh", "silu"])
@pytest.mark.parametrize("mode", ["fused", "split"])
def test_preact_modes_agree(act, mode):
    """gelu / silu forward in the GEMM epilogue or as GEMM + one elementwise pass: same y and z."""
    from kubeflow_rm_amd.ops import gemm as G
    M, N, K = 1024, 2048, 512
    x, w, bias = _rand(M, K, seed=97), _rand(N, K, seed=98, scale=0.1), _rand(N, seed=99)
    G.PREACT_MODE = mode
    try:
        y, z = G.gemm_nt_preact(x, w, bias, act)
    finally:
        G.PREACT_MODE = "auto"
    _assert_close(z, _ref_gemm(x, w, bias), K)
    _assert_close(y, _ref_gemm(x, w, bias, act), K)


def test_matmul_shapes_without_copies():
    """matmul: 2-D, leading dims folded into M, and batched, all vs fp32."""
    from kubeflow_rm_amd.ops import matmul
    a, b = _rand(3, 200, 256, seed=100), _rand(256, 384, seed=101)
    _assert_close(matmul(a, b), a.float() @ b.float(), 256)
    a3, b3 = _rand(2, 256, 512, seed=102), _rand(2, 512, 384, seed=103)
    _assert_close(matmul(a3, b3), a3.float() @ b3.float(), 512)
    _assert_close(matmul(a3[0], b3[0]), a3[0].float() @ b3[0].float(), 512)


@pytest.mark.parametrize("rows,V", [(512, 32000), (37, 1000), (8, 50257)])
def test_cross_entropy_matches_fp32(rows, V):
    """bf16 softmax cross-entropy (fwd: loss via log-sum-exp; bwd: softmax - onehot scaled by the
    upstream gradient / counted rows) vs torch's fp32 cross-entropy, with ignored targets."""
    from kubeflow_rm_amd.ops import cross_entropy
    x = (torch.randn(rows, V, device="cuda") * 3).to(torch.bfloat16).requires_grad_(True)
    t = torch.randint(0, V, (rows,), device="cuda")
    t[::5] = -100
    loss = cross_entropy(x, t)
    (loss * 0.5).backward()
    xr = x.detach().float().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(xr, t, ignore_index=-100)
    (ref * 0.5).backward()
    assert abs(loss.item() - ref.item()) <= 1e-3 * abs(ref.item()) + 1e-3, (loss.item(), ref.item())
    err = (x.grad.float() - xr.grad).abs().max().item()
    assert err <= 1e-2 * xr.grad.abs().max().item() + 1e-6, err


@pytest.mark.parametrize("B,T,h,hd", [(2, 256, 4, 64), (1, 100, 3, 128)])
def test_split_heads_backward_packs_qkv_grad(B, T, h, hd):
    """ops.split_heads: the same q / k / v views as view + permute, and a backward (the HIP pack of
    SDPA's dq / dk / dv into the fused QKV gradient) bitwise equal to autograd's own."""
    from kubeflow_rm_amd import ops
    qkv = _rand(B, T, 3 * h * hd, seed=95).requires_grad_(True)
    ref = qkv.detach().clone().requires_grad_(True)
    q, k, v = ops.split_heads(qkv, h, hd)
    qr, kr, vr = ref.view(B, T, 3, h, hd).permute(2, 0, 3, 1, 4)
    for a, b in ((q, qr), (k, kr), (v, vr)):
        assert a.shape == b.shape and torch.equal(a, b)
    F = torch.nn.functional
    y = F.scaled_dot_product_attention(q, k, v, is_causal=True)
    yr = F.scaled_dot_product_attention(qr, kr, vr, is_causal=True)
    g = _rand(*y.shape, seed=96)
    y.backward(g)
    yr.backward(g)
    assert torch.equal(qkv.grad, ref.grad)
    # a gradient autograd does not produce (v unused) packs zeros
    qkv.grad = None
    q, k, v = ops.split_heads(qkv, h, hd)
    (q.float().sum() + 2 * k.float().sum()).backward()
    gq = qkv.grad.view(B, T, 3, h, hd)
    assert torch.equal(gq[:, :, 0], torch.ones_like(gq[:, :, 0]))
    assert torch.equal(gq[:, :, 1], torch.full_like(gq[:, :, 1], 2))
    assert not gq[:, :, 2].any()


def _dact_ref(z, act):
    zf = z.float().requires_grad_(True)
    F = torch.nn.functional
    if act == "relu":
        y = F.relu(zf)
    elif act == "silu":
        y = F.silu(zf)
    else:
        y = F.gelu(zf, approximate="tanh")
    (d,) = torch.autograd.grad(y.sum(), zf)
    return d


@pytest.mark.parametrize("act", ["gelu_tanh", "silu", "relu"])
@pytest.mark.parametrize("M,K,N", [(512, 256, 768), (256, 2048, 1024), (1024, 512, 256)])
def test_dgrad_act_matches_fp32(act, M, K, N):
    """The act-grad GEMM epilogue (gemm_w4.h DACT): g = (gy @ W) * act'(z) against fp32, and the
    bias-gradient column sums (fp32 sums of the unrounded products) against the sums of the
    kernel's own bf16 g."""
    from kubeflow_rm_amd import ops
    gy, w = _rand(M, K, seed=71), _rand(K, N, seed=72, scale=0.05)
    z = _rand(M, N, seed=73, scale=2.0)
    out = ops.dgrad_act(gy, w, z, act, True, torch.float32)
    assert out is not None, "the fused kernel refused a 256-multiple shape"
    g, db = out
    ref = (gy.float() @ w.float()) * _dact_ref(z, act)
    err = (g.float() - ref).abs().max().item()
    assert err <= 2e-2 * (ref.abs().max().item() + 1e-3), err
    # the kernel sums the fp32 products before their bf16 rounding: within the rounding of g
    col = g.float().sum(0)
    assert (db - col).abs().max().item() <= 1e-3 * g.float().abs().sum(0).max().item() + 1e-3
    # bf16 bias gradient, no bias gradient
    g2, db2 = ops.dgrad_act(gy, w, z, act, True, torch.bfloat16)
    assert db2.dtype == torch.bfloat16 and torch.equal(g2, g)
    g3, db3 = ops.dgrad_act(gy, w, z, act, False)
    assert db3 is None and torch.equal(g3, g)


def test_dgrad_act_refuses_odd_shapes():
    from kubeflow_rm_amd import ops
    gy, w, z = _rand(300, 256, seed=74), _rand(256, 512, seed=75), _rand(300, 512, seed=76)
    assert ops.dgrad_act(gy, w, z, "gelu_tanh", True) is None


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("act", ["gelu_tanh", "silu"])
def test_mlp_matches_fp32(fused, act):
    """ops.mlp (fc1 + act + fc2 + residual as one autograd node) forward and every gradient vs fp32
    autograd, with fc2's dgrad fused with the activation backward (default) and in two steps."""
    from kubeflow_rm_amd import ops
    from kubeflow_rm_amd.ops import gemm as G
    B, T, D, Fd = 2, 256, 512, 1024
    x = _rand(B, T, D, seed=81).requires_grad_(True)
    w1, b1 = _rand(Fd, D, seed=82, scale=0.05).requires_grad_(True), _rand(Fd, seed=83).requires_grad_(True)
    w2, b2 = _rand(D, Fd, seed=84, scale=0.05).requires_grad_(True), _rand(D, seed=85).requires_grad_(True)
    r = _rand(B, T, D, seed=86).requires_grad_(True)
    gy = _rand(B, T, D, seed=87)
    old = G.FUSED_DGRAD_ACT
    G.FUSED_DGRAD_ACT = fused
    try:
        y = ops.mlp(x, w1, b1, w2, b2, act=act, residual=r)
        y.backward(gy)
    finally:
        G.FUSED_DGRAD_ACT = old
    ts = [t.detach().float().requires_grad_(True) for t in (x, w1, b1, w2, b2, r)]
    F = torch.nn.functional
    h = F.linear(ts[0], ts[1], ts[2])
    h = F.gelu(h, approximate="tanh") if act == "gelu_tanh" else F.silu(h)
    yr = F.linear(h, ts[3], ts[4]) + ts[5]
    yr.backward(gy.float())
    assert (y.float() - yr).abs().max().item() < 3e-2 * (yr.abs().max().item() + 1)
    for got, ref in zip((x.grad, w1.grad, b1.grad, w2.grad, b2.grad, r.grad), (t.grad for t in ts)):
        err = (got.float() - ref).abs().max().item()
        assert err <= 3e-2 * (ref.abs().max().item() + 1e-3) + 1e-2, err


@pytest.mark.parametrize("K,M1,M2,N,N2,plan", [(512, 768, 256, 512, 512, None), (1000, 6144, 2048, 2048, 2048, None),
                                                (384, 296, 520, 264, 264, None), (4096, 768, 256, 256, 768, (3, 1408)),
                                                (4000, 3072, 768, 768, 3072, (2, 2048)),
                                                (2112, 520, 296, 264, 520, (5, 448))])
def test_wgrad_pair_matches_fp32(K, M1, M2, N, N2, plan):
    """Two weight gradients in one launch (gemm_w4.h GRP): each against its fp32 product, including
    edge tiles (M / N not multiples of 256), a K that is not a multiple of 64, a second problem of
    its own width, and K split with the in-kernel fixup (SPLIT == 2) across both problems' tiles."""
    from kubeflow_rm_amd import ops
    g1, x1 = _rand(K, M1, seed=91), _rand(K, N, seed=92)
    g2, x2 = _rand(K, M2, seed=93), _rand(K, N2, seed=94)
    out = ops.wgrad_pair(g1, x1, g2, x2, force=True, plan=plan)
    assert out is not None
    for got, (g, x) in zip(out, ((g1, x1), (g2, x2))):
        _assert_close(got, g.float().t() @ x.float(), K)


@pytest.mark.parametrize("B,T,D,h,hd", [(1, 512, 2048, 16, 128), (2, 128, 512, 4, 64)])
def test_attn_block_matches_fp32(B, T, D, h, hd):
    """ops.attn_block (QKV projection + flash attention + output projection + residual as one autograd
    node; at D = 2048 both weight gradients in one launch, at D = 512 the separate path) forward and
    every gradient against fp32 autograd with F.scaled_dot_product_attention."""
    from kubeflow_rm_amd import ops
    F = torch.nn.functional
    x = _rand(B, T, D, seed=101).requires_grad_(True)
    wq, bq = _rand(3 * h * hd, D, seed=102, scale=0.03).requires_grad_(True), _rand(3 * h * hd, seed=103).requires_grad_(True)
    wp, bp = _rand(D, h * hd, seed=104, scale=0.03).requires_grad_(True), _rand(D, seed=105).requires_grad_(True)
    r = _rand(B, T, D, seed=106).requires_grad_(True)
    gy = _rand(B, T, D, seed=107)
    y = ops.attn_block(x, wq, bq, wp, bp, h, hd, residual=r)
    y.backward(gy)
    ts = [t.detach().float().requires_grad_(True) for t in (x, wq, bq, wp, bp, r)]
    qkv = F.linear(ts[0], ts[1], ts[2]).view(B, T, 3, h, hd)
    q, k, v = (qkv[:, :, i].transpose(1, 2) for i in range(3))
    o = F.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2).reshape(B, T, h * hd)
    yr = F.linear(o, ts[3], ts[4]) + ts[5]
    yr.backward(gy.float())
    assert (y.float() - yr).abs().max().item() < 3e-2 * (yr.abs().max().item() + 1)
    for name, got, ref in zip(("x", "wqkv", "bqkv", "wproj", "bproj", "res"),
                              (x.grad, wq.grad, bq.grad, wp.grad, bp.grad, r.grad), (t.grad for t in ts)):
        err = (got.float() - ref).abs().max().item()
        assert err <= 3e-2 * (ref.abs().max().item() + 1e-3) + 1e-2, (name, err)
