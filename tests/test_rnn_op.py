"""The reference ``rnn`` op (rnn_op.cc; python/paddle/nn/layer/rnn.py:1008-1056): ``nn.SimpleRNN /
LSTM / GRU`` and ``nn.RNN(cell)`` run as ONE op that records in static Programs, saves as the
reference ``rnn`` op type (with ``fill_constant_batch_size_like`` initial states), and round-trips
through save_inference_model / ``to_static`` + ``jit.save``. CPU numerics against the per-cell
path (torch fused cells) and an explicit step loop for variable-length batches."""
import os

import numpy as np
import pytest
import torch

import paddle_hackathon_amd as paddle
from paddle_hackathon_amd.ops import rnn as R

CASES = [(paddle.nn.LSTM, {}), (paddle.nn.GRU, {}), (paddle.nn.SimpleRNN, {}),
         (paddle.nn.SimpleRNN, {"activation": "relu"})]


@pytest.mark.parametrize("cls,kw", CASES)
@pytest.mark.parametrize("direction", ["forward", "bidirect"])
def test_op_path_matches_cell_path_with_grads(cls, kw, direction):
    paddle.seed(1)
    m = cls(6, 8, num_layers=2, direction=direction, **kw)
    x = paddle.to_tensor(np.random.RandomState(0).randn(3, 5, 6).astype("float32"), stop_gradient=False)
    y, _ = m(x)
    gy = [g.numpy() for g in paddle.grad(y.sum(), [x] + m.parameters())]
    y2, _ = m._cell_forward(x)
    gy2 = [g.numpy() for g in paddle.grad(y2.sum(), [x] + m.parameters())]
    np.testing.assert_allclose(y.numpy(), y2.numpy(), rtol=1e-5, atol=1e-6)
    for a, b in zip(gy, gy2):
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-6)


def test_weight_list_is_reference_order():
    m = paddle.nn.LSTM(4, 5, num_layers=2, direction="bidirect")
    ws = m._all_weights
    cells = [m[0].cell_fw, m[0].cell_bw, m[1].cell_fw, m[1].cell_bw]
    assert ws[:8] == [w for c in cells for w in (c.weight_ih, c.weight_hh)]
    assert ws[8:] == [b for c in cells for b in (c.bias_ih, c.bias_hh)]
    assert m.weight_ih_l1_reverse is m[1].cell_bw.weight_ih


@pytest.mark.parametrize("mode", ["LSTM", "GRU", "RNN_TANH"])
def test_sequence_length_masks_like_unpadded_rows(mode):
    cls = {"LSTM": paddle.nn.LSTM, "GRU": paddle.nn.GRU, "RNN_TANH": paddle.nn.SimpleRNN}[mode]
    paddle.seed(2)
    m = cls(4, 6, direction="bidirect")
    rng = np.random.RandomState(3)
    x = rng.randn(3, 7, 4).astype("float32")
    lens = np.array([7, 4, 2], "int64")
    y, st = m(paddle.to_tensor(x), sequence_length=paddle.to_tensor(lens))
    h = (st[0] if mode == "LSTM" else st).numpy()
    for b in range(3):
        L = lens[b]
        yb, stb = m(paddle.to_tensor(x[b:b + 1, :L]))
        hb = (stb[0] if mode == "LSTM" else stb).numpy()
        np.testing.assert_allclose(y.numpy()[b, :L], yb.numpy()[0], rtol=1e-5, atol=1e-6)
        assert np.all(y.numpy()[b, L:] == 0)
        np.testing.assert_allclose(h[:, b], hb[:, 0], rtol=1e-5, atol=1e-6)


def _net():
    class Net(paddle.nn.Layer):
        def __init__(self):
            super().__init__()
            self.lstm = paddle.nn.LSTM(8, 16, num_layers=2, direction="bidirect")
            self.gru = paddle.nn.GRU(32, 12)
            self.fc = paddle.nn.Linear(12, 3)

        def forward(self, x):
            y, _ = self.lstm(x)
            z, _ = self.gru(y)
            return self.fc(z[:, -1])
    return Net()


def test_static_program_records_one_rnn_op_and_round_trips(tmp_path):
    paddle.seed(0)
    net = _net()
    xs = np.random.RandomState(0).rand(4, 6, 8).astype("float32")
    ref = net(paddle.to_tensor(xs)).numpy()
    paddle.enable_static()
    try:
        main, startup = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, startup):
            x = paddle.static.data("x", [-1, 6, 8], "float32")
            out = net(x)
            assert list(out.shape) == [-1, 3]
        types = [op.type.rsplit(".", 1)[-1] for op in main.global_block().ops]
        assert types.count("rnn_op") == 2
        exe = paddle.static.Executor()
        o, = exe.run(main, feed={"x": xs}, fetch_list=[out])
        np.testing.assert_allclose(o, ref, rtol=1e-5, atol=1e-6)
        prefix = str(tmp_path / "m")
        paddle.static.save_inference_model(prefix, [x], [out], exe, program=main)
        from paddle_hackathon_amd.static import proto as pb
        desc = pb.ProgramDesc()
        with open(prefix + ".pdmodel", "rb") as f:
            desc.ParseFromString(f.read())
        saved = [op.type for op in desc.blocks[0].ops]
        assert saved.count("rnn") == 2 and "fill_constant_batch_size_like" in saved
        rnn_ops = [op for op in desc.blocks[0].ops if op.type == "rnn"]
        slots = {v.parameter: len(v.arguments) for v in rnn_ops[0].inputs}
        assert slots["WeightList"] == 16 and slots["PreState"] == 2
        assert {v.parameter for v in rnn_ops[0].outputs} == {"Out", "State", "Reserve", "DropoutState"}
        prog, feeds, fetches = paddle.static.load_inference_model(prefix, exe)
        r, = exe.run(prog, feed={feeds[0]: xs}, fetch_list=fetches)
        np.testing.assert_allclose(r, ref, rtol=1e-5, atol=1e-6)
    finally:
        paddle.disable_static()


def test_static_program_with_lstm_and_gru_trains():
    paddle.enable_static()
    try:
        paddle.seed(4)
        main, startup = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, startup):
            x = paddle.static.data("x", [-1, 6, 8], "float32")
            y, _ = paddle.nn.LSTM(8, 16)(x)
            z, _ = paddle.nn.GRU(16, 8, direction="bidirect")(y)
            out = paddle.nn.Linear(16, 3)(z[:, -1])
            lab = paddle.static.data("y", [-1, 1], "int64")
            loss = paddle.nn.functional.cross_entropy(out, lab)
            paddle.optimizer.Adam(0.01).minimize(loss)
        exe = paddle.static.Executor()
        exe.run(startup)
        rng = np.random.RandomState(5)
        xs, ys = rng.rand(8, 6, 8).astype("float32"), rng.randint(0, 3, [8, 1]).astype("int64")
        ls = [float(np.asarray(exe.run(main, feed={"x": xs, "y": ys}, fetch_list=[loss])[0]).reshape(-1)[0])
              for _ in range(25)]
        assert ls[-1] < 0.5 * ls[0], ls
    finally:
        paddle.disable_static()


def test_to_static_jit_save_lstm_classifier_with_lengths(tmp_path):
    class Cls(paddle.nn.Layer):
        def __init__(self):
            super().__init__()
            self.emb = paddle.nn.Embedding(50, 8)
            self.lstm = paddle.nn.LSTM(8, 16, direction="bidirect")
            self.fc = paddle.nn.Linear(32, 2)

        def forward(self, ids, lens):
            y, (h, c) = self.lstm(self.emb(ids), sequence_length=lens)
            return self.fc(y.mean(1))
    paddle.seed(6)
    net = Cls()
    net.eval()
    rng = np.random.RandomState(7)
    ids, lens = rng.randint(0, 50, [4, 7]).astype("int64"), np.array([7, 5, 3, 6], "int64")
    ref = net(paddle.to_tensor(ids), paddle.to_tensor(lens)).numpy()
    st = paddle.jit.to_static(net, input_spec=[paddle.static.InputSpec([None, 7], "int64"),
                                               paddle.static.InputSpec([None], "int64")])
    np.testing.assert_allclose(st(paddle.to_tensor(ids), paddle.to_tensor(lens)).numpy(), ref, rtol=1e-5, atol=1e-6)
    paddle.jit.save(st, str(tmp_path / "cls"))
    ld = paddle.jit.load(str(tmp_path / "cls"))
    np.testing.assert_allclose(ld(paddle.to_tensor(ids), paddle.to_tensor(lens)).numpy(), ref, rtol=1e-5, atol=1e-6)


def test_rnn_wrapper_over_cells_records_in_static_programs():
    paddle.seed(8)

    class MyCell(paddle.nn.SimpleRNNCell):   # a user cell: the per-step loop
        pass
    mods = [paddle.nn.RNN(paddle.nn.LSTMCell(8, 16)), paddle.nn.RNN(paddle.nn.GRUCell(8, 16), is_reverse=True),
            paddle.nn.RNN(MyCell(8, 16))]
    xs = np.random.RandomState(9).rand(3, 5, 8).astype("float32")
    refs = [m(paddle.to_tensor(xs))[0].numpy() for m in mods]
    paddle.enable_static()
    try:
        main, startup = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, startup):
            x = paddle.static.data("x", [-1, 5, 8], "float32")
            outs = [m(x)[0] for m in mods]
        res = paddle.static.Executor().run(main, feed={"x": xs}, fetch_list=outs)
    finally:
        paddle.disable_static()
    for a, b in zip(res, refs):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)


def test_step_loop_oracle_matches_torch_kernels():
    """ops/rnn.py's explicit recurrence (the GPU tests' fp32 oracle) == torch's fused kernels"""
    g = torch.Generator().manual_seed(0)
    T, B, I, H = 5, 3, 4, 6
    for mode, G in ((0, 1), (1, 1), (2, 4), (3, 3)):
        x = torch.randn(T, B, I, generator=g)
        w_ih, w_hh = torch.randn(G * H, I, generator=g) * 0.3, torch.randn(G * H, H, generator=g) * 0.3
        b_ih, b_hh = torch.randn(G * H, generator=g) * 0.1, torch.randn(G * H, generator=g) * 0.1
        h0, c0 = torch.randn(B, H, generator=g), torch.randn(B, H, generator=g)
        for rev in (False, True):
            y1, h1, c1 = R._vf_layer(x, h0, c0, [w_ih, w_hh, b_ih, b_hh], mode, rev)
            gx = x @ w_ih.t() + b_ih
            y2, h2, c2 = R._recur_torch(gx, h0, c0, w_hh, b_hh, None, mode, rev)
            torch.testing.assert_close(y1, y2, rtol=1e-5, atol=1e-5)
            torch.testing.assert_close(h1, h2, rtol=1e-5, atol=1e-5)
            if mode == 2:
                torch.testing.assert_close(c1, c2, rtol=1e-5, atol=1e-5)
