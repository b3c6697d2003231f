"""Dropout that survives hipGraph replay: the fused bias-dropout-residual-LN and flash-attention
dropout kernels xor a device seed word into their host seed (ops/hip.dropout_seed). The word must
act exactly like xor-ing the host seed (forward and the backward's regenerated mask), and a
captured BERT step must draw new masks on every replay instead of the masks baked in at capture."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_bdrln_device_seed_word_equals_xored_host_seed():
    from paddle_hackathon_amd.ops import hip as H
    g = torch.Generator(device="cuda").manual_seed(0)
    rows, C = 300, 768
    x = torch.randn(rows, C, device="cuda", generator=g).bfloat16()
    r = torch.randn(rows, C, device="cuda", generator=g).bfloat16()
    xb = torch.randn(C, device="cuda", generator=g).bfloat16()
    w, b = torch.rand(C, device="cuda", generator=g) + 0.5, torch.randn(C, device="cuda", generator=g) * 0.1
    seed, word, thresh, ks = 12345, 0x5a5a1234, int(0.1 * 65536), 1 / 0.9
    dev = torch.tensor([word], dtype=torch.int32, device="cuda")
    a = H.bdrln_fwd(x, xb, r, w, b, 1e-5, seed, thresh, ks, seed_dev=dev)
    ref = H.bdrln_fwd(x, xb, r, w, b, 1e-5, seed ^ word, thresh, ks)
    for u, v in zip(a, ref):
        assert torch.equal(u, v)
    other = H.bdrln_fwd(x, xb, r, w, b, 1e-5, seed, thresh, ks)
    assert not torch.equal(other[3], ref[3])   # the word changes the mask
    dh = torch.randn(rows, C, device="cuda", generator=g).bfloat16()
    da = H.dropout_bias_bwd(dh, seed, thresh, ks, torch.bfloat16, seed_dev=dev)
    dr = H.dropout_bias_bwd(dh, seed ^ word, thresh, ks, torch.bfloat16)
    assert torch.equal(da[0], dr[0]) and torch.equal(da[1], dr[1])


def test_flash_attention_dropout_device_seed_word(monkeypatch):
    from paddle_hackathon_amd.ops import hip as H
    g = torch.Generator(device="cuda").manual_seed(1)
    B, S, Hh, D = 2, 256, 4, 64
    q, k, v = (torch.randn(B, S, Hh, D, device="cuda", generator=g).bfloat16().requires_grad_(True) for _ in range(3))
    word = 0x13572468
    dev = torch.tensor([word], dtype=torch.int32, device="cuda")

    def run(seed_pair):
        monkeypatch.setattr(H, "dropout_seed", lambda device: seed_pair)
        o = H.FlashAttentionExt.apply(q, k, v, False, 0.125, None, 0.2)
        gs = torch.autograd.grad(o.float().square().sum(), (q, k, v))
        return [o] + list(gs)
    got = run((777, dev))
    ref = run((777 ^ word, None))
    for u, v_ in zip(got, ref):
        assert torch.equal(u, v_)


def test_graphed_bert_step_draws_new_masks_each_replay():
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.models import bert_config, BertForPretraining, BertPretrainingCriterion
    from paddle_hackathon_amd.device.cuda.graphs import wrap_cuda_graph
    paddle.set_device("gpu")
    try:
        paddle.seed(3)
        cfg = bert_config("bert-tiny")
        model = paddle.amp.decorate(BertForPretraining(cfg), level="O2", dtype="bfloat16")
        crit = BertPretrainingCriterion(cfg.vocab_size)
        opt = paddle.optimizer.AdamW(learning_rate=0.0, parameters=model.parameters(), multi_precision=True)
        B, S = 4, 128
        g = torch.Generator(device="cuda").manual_seed(0)
        ids = paddle.to_tensor(torch.randint(0, cfg.vocab_size, (B, S), device="cuda", generator=g))
        tt = paddle.to_tensor(torch.zeros(B, S, dtype=torch.long, device="cuda"))
        mpos = paddle.to_tensor(torch.arange(0, B * S, 7, device="cuda"))
        mlab = paddle.to_tensor(torch.randint(0, cfg.vocab_size, (mpos.shape[0],), device="cuda", generator=g))
        nlab = paddle.to_tensor(torch.randint(0, 2, (B,), device="cuda", generator=g))
        stream = torch.cuda.Stream()

        def step():
            with paddle.amp.auto_cast(level="O2", dtype="bfloat16"):
                mlm, nsp = model(ids, tt, masked_positions=mpos)
            loss = crit(mlm, nsp, mlab, nlab)
            loss.backward()
            opt.step()
            opt.clear_grad(set_to_zero=False)
            return loss
        with torch.cuda.stream(stream):
            gstep = wrap_cuda_graph(step)
            gstep._stream = stream
            losses = [float(gstep().item()) for _ in range(5)]   # eager, capture, then replays
        assert all(map(lambda v: v == v and abs(v) < 1e4, losses)), losses
        # lr 0: the weights never change, so replays differ only through their dropout masks
        assert len(set(round(v, 6) for v in losses[2:])) == 3, losses
    finally:
        paddle.set_device("cpu")


@pytest.mark.parametrize("C,dtype,wdt", [(768, torch.bfloat16, torch.float32), (2048, torch.bfloat16, torch.float32),
                                         (768, torch.float32, torch.float32), (1024, torch.float16, torch.float16)])
def test_ln_dropout_fused_backward_equals_two_passes(C, dtype, wdt):
    """the one-pass LN + dropout' backward (pha_layer_norm_dropout_bwd) is bitwise the LN backward
    followed by dropout_bias_bwd on the stored residual gradient, incl. the device seed word"""
    from paddle_hackathon_amd.ops import hip as H
    g = torch.Generator(device="cuda").manual_seed(1)
    rows = 1000
    x = torch.randn(rows, C, device="cuda", generator=g).to(dtype)
    r = torch.randn(rows, C, device="cuda", generator=g).to(dtype)
    w = (torch.rand(C, device="cuda", generator=g) + 0.5).to(wdt)
    b = (torch.randn(C, device="cuda", generator=g) * 0.1).to(wdt)
    gy = torch.randn(rows, C, device="cuda", generator=g).to(dtype)
    seed, thresh, ks = 777, int(0.1 * 65536), 1 / 0.9
    dev = torch.tensor([0x1234567], dtype=torch.int32, device="cuda")
    _, mean, rstd, hs = H.bdrln_fwd(x, None, r, w, b, 1e-5, seed, thresh, ks, dev)
    dh0, dw0, db0 = H.layer_norm_bwd(gy, hs, w, mean, rstd, True)
    dx0, _ = H.dropout_bias_bwd(dh0, seed, thresh, ks, None, dev)
    dh1, dx1, dw1, db1 = H.layer_norm_dropout_bwd(gy, hs, w, mean, rstd, True, seed, thresh, ks, dev)
    torch.cuda.synchronize()
    assert torch.equal(dh0, dh1) and torch.equal(dx0, dx1)
    assert torch.equal(dw0, dw1) and torch.equal(db0, db1)
    keep = (dx1 != 0).float().mean().item()
    assert 0.88 < keep < 0.92


def test_bdrln_autograd_fused_backward_matches_unfused(monkeypatch):
    """_BiasDropoutResidualLN backward with and without the one-pass kernel: same gradients"""
    import paddle_hackathon_amd.ops.fused as FU
    g = torch.Generator(device="cuda").manual_seed(2)
    rows, C = 512, 768
    x0 = torch.randn(rows, C, device="cuda", generator=g).bfloat16()
    r0 = torch.randn(rows, C, device="cuda", generator=g).bfloat16()
    w = torch.rand(C, device="cuda", generator=g) + 0.5
    b = torch.randn(C, device="cuda", generator=g) * 0.1
    gy = torch.randn(rows, C, device="cuda", generator=g).bfloat16()
    outs = []
    for fused in (True, False):
        monkeypatch.setattr(FU, "_LN_DROP_FUSED", fused)
        torch.manual_seed(5)   # same host dropout seed both times
        x, r = x0.clone().requires_grad_(True), r0.clone().requires_grad_(True)
        wl, bl = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
        y = FU.bias_dropout_residual_layer_norm(x, r, None, wl, bl, 0.1, True, 1e-5)
        y.backward(gy)
        outs.append((y.detach(), x.grad, r.grad, wl.grad, bl.grad))
    for a, c in zip(*outs):
        assert torch.equal(a, c)
