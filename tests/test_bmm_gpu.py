"""Batched products with per-batch right operands on the own persistent kernel (gemm4p batched
mode: one launch over every item's tiles). Reference: phi/kernels/impl/matmul_kernel_impl.h:88
(MatMulFunction's batched branch). Numerics against an fp32 torch bmm of the same bf16 inputs."""
import pytest
import torch

import paddle_hackathon_amd as paddle

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _on_gpu():
    paddle.set_device("gpu")
    yield
    paddle.set_device("cpu")


def _rel(a, b):
    a = a.to(b.device)
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
def test_bmm_layouts_match_fp32(ta, tb):
    from paddle_hackathon_amd.ops import fallback, gemm
    torch.manual_seed(0)
    B, M, N, K = 6, 264, 328, 192
    a = torch.randn(B, K, M, device="cuda").bfloat16() if ta else torch.randn(B, M, K, device="cuda").bfloat16()
    b = torch.randn(B, N, K, device="cuda").bfloat16() if tb else torch.randn(B, K, N, device="cuda").bfloat16()
    x = a.transpose(1, 2) if ta else a
    y = b.transpose(1, 2) if tb else b
    before = fallback.counts().get("matmul", 0) if hasattr(fallback, "counts") else None
    c = gemm.bmm_own(x, y)
    assert c is not None
    ref = torch.bmm(x.float(), y.float())
    assert c.shape == ref.shape
    assert _rel(c, ref) < 1e-2
    # paddle.bmm / matmul route there too
    out = paddle.matmul(paddle.to_tensor(a), paddle.to_tensor(b), transpose_x=ta, transpose_y=tb)
    assert _rel(out._t, ref) < 1e-2
    if before is not None:
        assert fallback.counts().get("matmul", 0) == before


def test_bmm_broadcast_and_4d():
    from paddle_hackathon_amd.ops import gemm
    torch.manual_seed(1)
    q = torch.randn(2, 3, 128, 64, device="cuda").bfloat16()
    k = torch.randn(2, 3, 256, 64, device="cuda").bfloat16()
    s = gemm.matmul(q, k, False, True)
    ref = torch.matmul(q.float(), k.float().transpose(-1, -2))
    assert s.shape == (2, 3, 128, 256) and _rel(s, ref) < 1e-2
    w = torch.randn(64, 128, device="cuda").bfloat16()   # 2-D right operand: flattened into M
    assert _rel(gemm.matmul(q, w), torch.matmul(q.float(), w.float())) < 1e-2
    wb = torch.randn(1, 3, 64, 128, device="cuda").bfloat16()   # broadcast batch dim (stride 0)
    assert _rel(gemm.matmul(q, wb), torch.matmul(q.float(), wb.float())) < 1e-2


def test_bmm_backward_matches_fp32():
    from paddle_hackathon_amd.ops import gemm
    torch.manual_seed(2)
    a = torch.randn(4, 136, 256, device="cuda").bfloat16().requires_grad_(True)
    b = torch.randn(4, 256, 200, device="cuda").bfloat16().requires_grad_(True)
    c = gemm.matmul(a, b)
    g = torch.randn_like(c)
    da, db = torch.autograd.grad(c, (a, b), g)
    af, bf = a.detach().float().requires_grad_(True), b.detach().float().requires_grad_(True)
    rda, rdb = torch.autograd.grad(torch.bmm(af, bf), (af, bf), g.float())
    assert _rel(da, rda) < 1e-2 and _rel(db, rdb) < 1e-2
