"""Bias gradients from the weight-gradient GEMM (gemm4p TN with G4P_COLSUM, ops/gemm.mm_tn_db): the
column sums of dY come from the B fragments the TN kernel's MFMAs already hold, each tile row of
the grid summing its own 1/tiles_m of the token range. dW must be bitwise the plain TN product
(the extra VALU work does not touch the accumulators) and db must match an fp32 column sum —
unsplit and split-K grids, ragged M / N tails, K ranges shorter than the tile-row count, fp16.
Then the linear / MLP backward paths that take it (reference: fused_gemm_epilogue_op.cu:298)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _r(*s, g, dt=torch.bfloat16):
    return (torch.rand(*s, device="cuda", generator=g) * 2 - 1).to(dt)


@pytest.mark.parametrize("K,M,N", [(4096, 2048, 2048), (8192, 768, 3072), (1024, 2048, 6144), (128, 2048, 512),
                                   (640, 1000, 776), (2048, 264, 136)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_mm_tn_db_matches_plain_tn_and_fp32_colsum(K, M, N, dt):
    from paddle_hackathon_amd.ops import gemm as G
    g = torch.Generator(device="cuda").manual_seed(K + M + N)
    x, dy = _r(K, M, g=g, dt=dt), _r(K, N, g=g, dt=dt)
    sp = G._splits(M, N, K, x.device)
    ref = G.gemm_p(x, dy, True, True, splits=sp, epi_extra=G.EPI_EARLY)
    dw, part = G.gemm_p(x, dy, True, True, splits=sp, colsum=True)
    assert torch.equal(dw, ref), "the column sums changed the product"
    assert part.shape == (2 * sp * -(-M // 256) + 8, N)
    db = G.colsum_rows_finish(part, torch.float32)
    f32 = dy.float().sum(0)
    assert ((db - f32).abs().max() / f32.abs().max().clamp_min(1)).item() < 1e-5
    dw2, db2 = G.mm_tn_db(x, dy)
    assert torch.equal(dw2, ref) and db2.dtype == dt
    assert ((db2.float() - f32).abs().max() / f32.abs().max().clamp_min(1)).item() < 1e-2


def test_forced_splits_and_refused_layouts():
    from paddle_hackathon_amd.ops import gemm as G
    g = torch.Generator(device="cuda").manual_seed(3)
    x, dy = _r(2048, 512, g=g), _r(2048, 512, g=g)
    for sp in (1, 2, 4, 8):
        dw, part = G.gemm_p(x, dy, True, True, splits=sp, colsum=True)
        assert torch.equal(dw, G.gemm_p(x, dy, True, True, splits=sp, epi_extra=G.EPI_EARLY))
        db = G.colsum_rows_finish(part, torch.float32)
        assert torch.allclose(db, dy.float().sum(0), rtol=1e-5, atol=1e-3)
    with pytest.raises(AssertionError):
        G.gemm_p(x.t().contiguous(), dy.t().contiguous(), colsum=True)   # NT: no column sums


def test_linear_and_mlp_backward_bias_grads():
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.ops import mlp
    paddle.set_device("gpu")
    try:
        g = torch.Generator(device="cuda").manual_seed(7)
        x = _r(4, 512, 1024, g=g)
        w, b = paddle.to_tensor(_r(1024, 768, g=g) * 0.05, stop_gradient=False), \
            paddle.to_tensor(_r(768, g=g), stop_gradient=False)
        y = paddle.nn.functional.linear(paddle.to_tensor(x), w, b)
        gy = _r(4, 512, 768, g=g)
        y.backward(paddle.to_tensor(gy))
        ref_db = gy.float().reshape(-1, 768).sum(0)
        ref_dw = x.float().reshape(-1, 1024).t() @ gy.float().reshape(-1, 768)
        assert ((b.grad._t.float() - ref_db).abs().max() / ref_db.abs().max()).item() < 1e-2
        assert ((w.grad._t.float() - ref_dw).norm() / ref_dw.norm()).item() < 1e-2
        # the fused MLP: db2 from the fc2 dW GEMM, db1 from the fc1 dW GEMM over dGELU
        H, F = 1024, 4096
        x2 = _r(2048, H, g=g).requires_grad_(True)
        w1, w2 = (_r(H, F, g=g) * 0.03).requires_grad_(True), (_r(F, H, g=g) * 0.03).requires_grad_(True)
        b1, b2 = (_r(F, g=g) * 0.1).requires_grad_(True), (_r(H, g=g) * 0.1).requires_grad_(True)
        for approx in (True, False):   # tanh GELU (GPT) and exact erf GELU (BERT, chain 0)
            for t in (x2, w1, b1, w2, b2):
                t.grad = None
            y2 = mlp.fused_mlp(x2, w1, b1, w2, b2, approximate=approx)
            gy2 = _r(2048, H, g=g)
            y2.backward(gy2)
            xs = [t.detach().float().requires_grad_(True) for t in (x2, w1, b1, w2, b2)]
            h = torch.nn.functional.gelu(xs[0] @ xs[1] + xs[2], approximate="tanh" if approx else "none")
            yr = h @ xs[3] + xs[4]
            yr.backward(gy2.float())
            assert ((y2.float() - yr).norm() / yr.norm()).item() < 1e-2
            for got, ref in zip((x2.grad, w1.grad, b1.grad, w2.grad, b2.grad), xs):
                ref = ref.grad
                assert ((got.float() - ref).norm() / ref.norm()).item() < 2e-2, approx
    finally:
        paddle.set_device("cpu")
