"""K3 one-shot all-reduce kernel (kernels/allreduce_oneshot.hip) vs a plain fp32 PyTorch reference.

On the single-GPU test box the ranks are simulated on one device in ONE launch (gridDim.y = ranks):
the barrier protocol, vector/tail paths, epoch reuse and the timeout drain all run on the hardware.
"""
import ctypes

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
    rc = L.kfamd_allreduce_oneshot(arr(*[t.data_ptr() for t in ins]), arr(*[t.data_ptr() for t in outs]),
                                   arr(*[t.data_ptr() for t in flags]), 2, 0, 1, n, 0, 1, nb, tmo.data_ptr(),
                                   torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()  # rank 1 never launched: both barriers give up, the kernel drains
    assert tmo.item() == 1


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
