"""metric, hapi Model/callbacks/summary/flops, profiler, distribution, text, inference,
onnx, legacy reader/dataset — each checked against closed forms / brute force / numpy."""
import itertools
import json
import os

import numpy as np
import pytest
import torch

import paddle_hackathon_amd as paddle


# ----------------------------------------------------------------------------- metric
def test_accuracy_metric_topk():
    m = paddle.metric.Accuracy(topk=(1, 2))
    pred = paddle.to_tensor([[0.1, 0.7, 0.2], [0.5, 0.2, 0.3], [0.2, 0.3, 0.5]])
    label = paddle.to_tensor([[1], [2], [0]])
    c = m.compute(pred, label)
    m.update(c)
    top1, top2 = m.accumulate()
    assert top1 == pytest.approx(1 / 3) and top2 == pytest.approx(2 / 3)
    assert m.name() == ["acc_top1", "acc_top2"]
    acc = paddle.metric.accuracy(pred, label, k=1)
    assert float(acc) == pytest.approx(1 / 3)


def test_precision_recall_auc():
    preds = np.array([0.1, 0.9, 0.8, 0.3, 0.7])
    labels = np.array([0, 1, 0, 1, 1])
    p, r = paddle.metric.Precision(), paddle.metric.Recall()
    p.update(preds, labels)
    r.update(preds, labels)
    assert p.accumulate() == pytest.approx(2 / 3)
    assert r.accumulate() == pytest.approx(2 / 3)
    auc = paddle.metric.Auc()
    scores = np.stack([1 - preds, preds], 1)
    auc.update(scores, labels)
    # exact AUC by pair counting
    pos, neg = preds[labels == 1], preds[labels == 0]
    exact = np.mean([(a > b) + 0.5 * (a == b) for a in pos for b in neg])
    assert auc.accumulate() == pytest.approx(exact, abs=1e-3)


# ----------------------------------------------------------------------------- hapi
class _DS(paddle.io.Dataset):
    def __init__(self, n=64):
        rng = np.random.RandomState(0)
        self.x = rng.rand(n, 4).astype("float32")
        self.y = (self.x.sum(1) > 2).astype("int64")[:, None]

    def __getitem__(self, i):
        return self.x[i], self.y[i]

    def __len__(self):
        return len(self.x)


def test_model_fit_evaluate_predict_save_load(tmp_path):
    paddle.seed(0)
    net = paddle.nn.Sequential(paddle.nn.Linear(4, 16), paddle.nn.ReLU(), paddle.nn.Linear(16, 2))
    model = paddle.Model(net)
    model.prepare(paddle.optimizer.Adam(0.01, parameters=net.parameters()), paddle.nn.CrossEntropyLoss(),
                  paddle.metric.Accuracy())
    es = paddle.callbacks.EarlyStopping(monitor="loss", patience=100)
    model.fit(_DS(), _DS(32), batch_size=16, epochs=3, verbose=0, callbacks=[es])
    res = model.evaluate(_DS(32), batch_size=16, verbose=0)
    assert "loss" in res and "acc" in res and res["acc"] > 0.5
    pred = model.predict(_DS(8), batch_size=4, stack_outputs=True)
    assert pred[0].shape == (8, 2)
    model.save(str(tmp_path / "ckpt"))
    assert os.path.exists(tmp_path / "ckpt.pdparams") and os.path.exists(tmp_path / "ckpt.pdopt")
    net2 = paddle.nn.Sequential(paddle.nn.Linear(4, 16), paddle.nn.ReLU(), paddle.nn.Linear(16, 2))
    m2 = paddle.Model(net2)
    m2.prepare(paddle.optimizer.Adam(0.01, parameters=net2.parameters()))
    m2.load(str(tmp_path / "ckpt"))
    x = paddle.randn([3, 4])
    np.testing.assert_allclose(net(x).numpy(), net2(x).numpy(), rtol=1e-6)


def test_summary_and_flops(capsys):
    net = paddle.nn.Sequential(paddle.nn.Conv2D(3, 8, 3), paddle.nn.ReLU(), paddle.nn.Flatten(),
                               paddle.nn.Linear(8 * 6 * 6, 10))
    info = paddle.summary(net, (1, 3, 8, 8))
    assert info["total_params"] == 3 * 8 * 9 + 8 + 288 * 10 + 10
    f = paddle.flops(net, [1, 3, 8, 8])
    assert f == 8 * 36 * 27 + 8 * 36 + 10 * 288 + 10


def test_reduce_lr_on_plateau():
    net = paddle.nn.Linear(2, 2)
    m = paddle.Model(net)
    opt = paddle.optimizer.SGD(1.0, parameters=net.parameters())
    m.prepare(opt)
    cb = paddle.callbacks.ReduceLROnPlateau(patience=1, factor=0.5)
    cb.set_model(m)
    for v in (1.0, 1.0):
        cb.on_eval_end({"loss": [v]})
    assert opt.get_lr() == pytest.approx(0.5)
    cb.on_eval_end({"loss": [0.5]})  # improvement resets patience
    assert opt.get_lr() == pytest.approx(0.5)
    cb.on_eval_end({"loss": [0.5]})
    assert opt.get_lr() == pytest.approx(0.25)


# ----------------------------------------------------------------------------- profiler
def test_profiler_scheduler_and_export(tmp_path):
    import paddle_hackathon_amd.profiler as profiler
    sched = profiler.make_scheduler(closed=1, ready=1, record=2, repeat=1)
    states = [sched(i) for i in range(6)]
    S = profiler.ProfilerState
    assert states == [S.CLOSED, S.READY, S.RECORD, S.RECORD_AND_RETURN, S.CLOSED, S.CLOSED]
    net = paddle.nn.Linear(4, 4)
    p = profiler.Profiler(targets=[profiler.ProfilerTarget.CPU], scheduler=(1, 3),
                          on_trace_ready=profiler.export_chrome_tracing(str(tmp_path)))
    p.start()
    for _ in range(4):
        with profiler.RecordEvent("my_step"):
            net(paddle.randn([2, 4])).sum().backward()
        p.step(num_samples=2)
    p.stop()
    files = os.listdir(tmp_path)
    assert len(files) == 1
    ev = profiler.load_profiler_result(str(tmp_path / files[0])).events
    names = [e["name"] for e in ev]
    assert names.count("my_step") == 2 and "Linear" in names and "linear" in names
    assert "ProfileStep#1" in names and "ProfileStep#2" in names
    txt = p.summary()
    assert "my_step" in txt
    pb = str(tmp_path / "t.pb")
    p.export(pb, "pb")
    assert len(profiler.load_profiler_result(pb).events) == len(ev)
    assert "ips" in p.step_info()


# ----------------------------------------------------------------------------- distribution
def test_distributions_vs_torch():
    D = paddle.distribution
    td = torch.distributions
    n, m = D.Normal([0.0, 1.0], [1.0, 2.0]), D.Normal([0.5, 0.0], [1.5, 1.0])
    tn, tm = td.Normal(torch.tensor([0.0, 1.0]), torch.tensor([1.0, 2.0])), td.Normal(torch.tensor([0.5, 0.0]),
                                                                                   torch.tensor([1.5, 1.0]))
    v = paddle.to_tensor([0.3, -0.2])
    np.testing.assert_allclose(n.log_prob(v).numpy(), tn.log_prob(v._t).numpy(), rtol=1e-5)
    np.testing.assert_allclose(n.entropy().numpy(), tn.entropy().numpy(), rtol=1e-5)
    np.testing.assert_allclose(D.kl_divergence(n, m).numpy(), td.kl_divergence(tn, tm).numpy(), rtol=1e-5)
    assert n.sample([5]).shape == [5, 2]
    u = D.Uniform(0.0, 2.0)
    assert float(u.entropy()) == pytest.approx(np.log(2.0))
    b = D.Beta(2.0, 3.0)
    np.testing.assert_allclose(b.log_prob(paddle.to_tensor(0.4)).numpy(),
                               td.Beta(2.0, 3.0).log_prob(torch.tensor(0.4)).numpy(), rtol=1e-5)
    dd = D.Dirichlet(paddle.to_tensor([1.0, 2.0, 3.0]))
    x = paddle.to_tensor([0.2, 0.3, 0.5])
    np.testing.assert_allclose(dd.log_prob(x).numpy(), td.Dirichlet(torch.tensor([1.0, 2.0, 3.0])).log_prob(x._t).numpy(),
                               rtol=1e-5)
    mn = D.Multinomial(10, paddle.to_tensor([0.2, 0.3, 0.5]))
    s = mn.sample([7])
    assert s.shape == [7, 3] and (s.numpy().sum(-1) == 10).all()
    np.testing.assert_allclose(mn.log_prob(paddle.to_tensor([2.0, 3.0, 5.0])).numpy(),
                               td.Multinomial(10, torch.tensor([0.2, 0.3, 0.5])).log_prob(torch.tensor([2.0, 3.0, 5.0])).numpy(),
                               rtol=1e-5)


def test_categorical_reference_semantics():
    D = paddle.distribution
    logits = paddle.to_tensor([0.2, 0.3, 0.5])
    c = D.Categorical(logits)
    # probs(): logits normalised by their sum (reference categorical.py:118)
    np.testing.assert_allclose(c.probs(paddle.to_tensor([0, 2])).numpy(), [0.2, 0.5], rtol=1e-6)
    # entropy(): softmax of logits
    p = torch.softmax(logits._t, -1)
    np.testing.assert_allclose(c.entropy().numpy(), [-(p * p.log()).sum().item()], rtol=1e-5)


def test_transformed_and_independent():
    D = paddle.distribution
    td = D.TransformedDistribution(D.Normal(0.0, 1.0), [D.ExpTransform()])
    ln = torch.distributions.LogNormal(0.0, 1.0)
    assert float(td.log_prob(paddle.to_tensor(2.0))) == pytest.approx(float(ln.log_prob(torch.tensor(2.0))), rel=1e-5)
    ind = D.Independent(D.Normal(paddle.zeros([3, 4]), paddle.ones([3, 4])), 1)
    assert ind.batch_shape == (3,) and ind.event_shape == (4,)
    assert ind.log_prob(paddle.zeros([3, 4])).shape == [3]
    t = D.StickBreakingTransform()
    x = paddle.to_tensor([0.1, -0.3])
    y = t.forward(x)
    assert float(y.sum()) == pytest.approx(1.0, rel=1e-6)
    np.testing.assert_allclose(t.inverse(y).numpy(), x.numpy(), atol=1e-5)
    ch = D.ChainTransform([D.AffineTransform(paddle.to_tensor(1.0), paddle.to_tensor(2.0)), D.TanhTransform()])
    np.testing.assert_allclose(ch.inverse(ch.forward(x)).numpy(), x.numpy(), atol=1e-5)
    # log-det of affine∘tanh vs autograd
    xt = x._t.clone().requires_grad_(True)
    yt = torch.tanh(1 + 2 * xt)
    ldj = torch.log(torch.stack([torch.autograd.grad(yt[i], xt, retain_graph=True)[0][i] for i in range(2)]).abs())
    np.testing.assert_allclose(ch.forward_log_det_jacobian(x).numpy(), ldj.detach().numpy(), rtol=1e-5)


# ----------------------------------------------------------------------------- text
@pytest.mark.parametrize("bos", [False, True])
def test_viterbi_decode_bruteforce(bos):
    paddle.seed(3)
    B, T, N = 3, 4, 5
    emission = paddle.rand((B, T, N))
    trans = paddle.rand((N, N))
    length = paddle.to_tensor([3, 4, 1])
    scores, path = paddle.text.viterbi_decode(emission, trans, length, bos)
    e, t = emission.numpy(), trans.numpy()
    for b in range(B):
        L = int(length.numpy()[b])
        best = None
        for pth in itertools.product(range(N), repeat=L):
            sc = e[b, 0, pth[0]] + (t[N - 1, pth[0]] if bos else 0)
            for i in range(1, L):
                sc += t[pth[i - 1], pth[i]] + e[b, i, pth[i]]
            if bos:
                sc += t[N - 2, pth[-1]]
            if best is None or sc > best[0]:
                best = (sc, pth)
        assert scores.numpy()[b] == pytest.approx(best[0], rel=1e-5)
        assert list(path.numpy()[b][:L]) == list(best[1])


def test_text_datasets_structure():
    T = paddle.text
    x, y = T.UCIHousing(mode="train")[0]
    assert x.shape == (13,) and y.shape == (1,)
    doc, lab = T.Imdb(mode="train")[0]
    assert doc.dtype == np.int64 and lab.shape == (1,)
    assert len(T.Imikolov(window_size=5)[0]) == 5
    assert len(T.Movielens()[0]) == 8
    assert len(T.Conll05st()[0]) == 9
    src, trg, nxt = T.WMT16()[0]
    assert (trg[1:] == nxt[:-1]).all()


# ----------------------------------------------------------------------------- inference / onnx
def test_inference_predictor_matches_layer(tmp_path):
    from paddle_hackathon_amd.static import InputSpec
    net = paddle.nn.Sequential(paddle.nn.Linear(8, 16), paddle.nn.GELU(), paddle.nn.Linear(16, 3))
    path = str(tmp_path / "inference")
    paddle.jit.save(net, path, input_spec=[InputSpec([None, 8], "float32", "x")])
    cfg = paddle.inference.Config(path + ".pdmodel", path + ".pdiparams")
    pred = paddle.inference.create_predictor(cfg)
    x = np.random.rand(5, 8).astype("float32")
    h = pred.get_input_handle(pred.get_input_names()[0])
    h.reshape([5, 8])
    h.copy_from_cpu(x)
    pred.run()
    out = pred.get_output_handle(pred.get_output_names()[0]).copy_to_cpu()
    np.testing.assert_allclose(out, net(paddle.to_tensor(x)).numpy(), rtol=1e-5, atol=1e-6)
    pool = paddle.inference.PredictorPool(cfg, 2)
    assert pool.retrive(1).get_input_names() == pred.get_input_names()
    cfg2 = paddle.inference.Config(str(tmp_path))
    assert paddle.inference.create_predictor(cfg2).get_input_names() == ["x"]


def test_onnx_export(tmp_path):
    from paddle_hackathon_amd.static import InputSpec
    net = paddle.nn.Sequential(paddle.nn.Linear(8, 16), paddle.nn.ReLU(), paddle.nn.Linear(16, 3))
    p = paddle.onnx.export(net, str(tmp_path / "m"), input_spec=[InputSpec([None, 8], "float32", "x")],
                           opset_version=11)
    data = open(p, "rb").read()
    assert len(data) > 8 * 16 * 4 and b"x" in data
    # params are restored after export
    assert not net[0].weight.stop_gradient


def test_legacy_reader_and_dataset():
    r = paddle.batch(lambda: iter(range(10)), 4)
    assert [len(b) for b in r()] == [4, 4, 2]
    from paddle_hackathon_amd import reader
    assert list(reader.firstn(lambda: iter(range(10)), 3)()) == [0, 1, 2]
    assert sorted(reader.shuffle(lambda: iter(range(10)), 4)()) == list(range(10))
    comp = reader.compose(lambda: iter([1, 2]), lambda: iter([(3, 4), (5, 6)]))
    assert list(comp()) == [(1, 3, 4), (2, 5, 6)]
    img, lab = next(paddle.dataset.mnist.train()())
    assert img.shape == (784,) and -1.0 <= img.min() and img.max() <= 1.0
    x, y = next(paddle.dataset.uci_housing.train()())
    assert x.shape == (13,)


def test_device_and_utils():
    assert "cpu" in paddle.device.get_all_device_type()
    assert paddle.device.is_compiled_with_rocm()
    paddle.utils.require_version("0.0.1")
    with pytest.raises(ImportError):
        paddle.utils.try_import("definitely_not_a_module_xyz")

    @paddle.utils.deprecated(update_to="paddle.new", since="0.1", level=1)
    def old():
        return 1
    with pytest.warns(DeprecationWarning):
        assert old() == 1
    x = paddle.to_tensor([1.0, 2.0])
    y = paddle.utils.dlpack.from_dlpack(paddle.utils.dlpack.to_dlpack(x))
    np.testing.assert_array_equal(x.numpy(), y.numpy())
    paddle.utils.run_check()
    paddle.set_printoptions(precision=2)
    s = str(paddle.to_tensor([1.23456]))
    assert "1.23" in s and "1.2346" not in s
    paddle.set_printoptions(precision=8)
    paddle.check_shape([2, -1])
    with pytest.raises(ValueError):
        paddle.check_shape([2, -3])


def test_fft_signal_vs_numpy():
    x = np.random.rand(4, 16).astype("float32")
    t = paddle.to_tensor(x)
    np.testing.assert_allclose(paddle.fft.fft(t).numpy(), np.fft.fft(x), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(paddle.fft.rfft2(t, norm="ortho").numpy(), np.fft.rfft2(x, norm="ortho"), rtol=1e-4,
                               atol=1e-4)
    np.testing.assert_allclose(paddle.fft.irfft(paddle.fft.rfft(t)).numpy(), x, atol=1e-5)
    np.testing.assert_allclose(paddle.fft.fftshift(t).numpy(), np.fft.fftshift(x), atol=0)
    np.testing.assert_allclose(paddle.fft.fftfreq(8, 0.5).numpy(), np.fft.fftfreq(8, 0.5), rtol=1e-6)
    sig = paddle.to_tensor(np.random.rand(2, 512).astype("float32"))
    spec = paddle.signal.stft(sig, 64, hop_length=16, window=paddle.to_tensor(np.hanning(64).astype("float32")))
    rec = paddle.signal.istft(spec, 64, hop_length=16, window=paddle.to_tensor(np.hanning(64).astype("float32")),
                              length=512)
    np.testing.assert_allclose(rec.numpy()[:, 64:-64], sig.numpy()[:, 64:-64], atol=1e-4)
