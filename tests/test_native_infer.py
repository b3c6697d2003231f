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


_CLIENTS = {}


def _client(tmp_path):
    """the C++ client (tests/native_infer/infer_main.cpp) linked against libpha_infer.so, built from
    source into the test's tmp dir (once per source text and library path in a session)"""
    import hashlib
    src = os.path.join(HERE, "native_infer", "infer_main.cpp")
    libdir = os.path.dirname(lib_path())
    with open(src, "rb") as f:
        key = (hashlib.sha256(f.read()).hexdigest(), libdir)
    exe = _CLIENTS.get(key)
    if exe is None or not os.path.exists(exe):
        exe = str(tmp_path / "infer_main")
        inc = os.path.join(os.path.dirname(HERE), "paddle_hackathon_amd", "csrc", "infer")
        subprocess.run(["g++", "-O2", "-std=c++17", "-I", inc, src, "-o", exe, "-L", libdir, "-lpha_infer",
                        f"-Wl,-rpath,{libdir}"], check=True)
        _CLIENTS[key] = exe
    return exe


def _run_client(tmp_path, m, p, feeds, device):
    args = [_client(tmp_path), m, p, str(device), str(tmp_path / "out")]
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


def test_ir_passes_fold_conv_bn_and_match_unfused(tmp_path):
    """conv_bn_fuse_pass / conv_elementwise_add_fuse_pass at load (reference paddle_pass_builder.cc:108):
    ResNet-18's 20 conv + batch_norm pairs fold into filters + biases; results match the unfused
    program and the Python predictor"""
    name, m, p, feeds = _cases(tmp_path)[0]
    fused = NativePredictor(m, p, device=-1)
    plain = NativePredictor(m, p, device=-1, ir_optim=False)
    assert any(s.startswith("conv_bn_fuse_pass x20") for s in fused.applied_passes), fused.applied_passes
    assert plain.applied_passes == []
    a, b = fused.run(feeds), plain.run(feeds)
    for x, y in zip(a, b):
        np.testing.assert_allclose(x, y, rtol=1e-4, atol=1e-5)
    for x, y in zip(a, _python_predictor(m, p, feeds)):
        np.testing.assert_allclose(x, y, rtol=1e-4, atol=1e-5)


def _corrupt_params(tmp_path, p, edit):
    data = bytearray(open(p, "rb").read())
    edit(data)
    bad = str(tmp_path / "bad.pdiparams")
    with open(bad, "wb") as f:
        f.write(bytes(data))
    return bad


def test_malformed_params_stream_is_a_clean_error(tmp_path):
    import struct
    name, m, p, feeds = _cases(tmp_path)[2]

    def huge_lod(d):   # LoD level count of the first tensor
        d[4:12] = struct.pack("<Q", 1 << 40)

    def neg_desc(d):   # tensor desc size of the first tensor (no LoD levels in it)
        d[16:20] = struct.pack("<i", -5)
    for edit in (huge_lod, neg_desc, lambda d: d.__delitem__(slice(len(d) - 7, len(d)))):
        bad = _corrupt_params(tmp_path, p, edit)
        with pytest.raises(RuntimeError, match="params stream|trailing|truncated"):
            NativePredictor(m, bad, device=-1)


def _pool_threads(m, p, feeds, device, n=4, reps=3):
    import threading
    preds = [NativePredictor(m, p, device=device) for _ in range(n)]
    res, errs = [None] * n, []

    def work(i):
        try:
            for _ in range(reps):
                res[i] = preds[i].run(feeds)
        except Exception as e:   # noqa: BLE001
            errs.append(e)
    th = [threading.Thread(target=work, args=(i,)) for i in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    return res, preds


def test_predictor_pool_threads_host(tmp_path):
    name, m, p, feeds = _cases(tmp_path)[0]
    res, _ = _pool_threads(m, p, feeds, -1)
    for r in res[1:]:
        for a, b in zip(r, res[0]):
            np.testing.assert_array_equal(a, b)


@pytest.mark.gpu
def test_predictor_pool_threads_gpu_own_streams_and_pool(tmp_path):
    """four predictors (each its own stream and block pool) driven from four threads at once; a
    second run of a predictor allocates nothing new (pooled memory)"""
    import torch
    name, m, p, feeds = _cases(tmp_path)[0]
    res, preds = _pool_threads(m, p, feeds, 0)
    host = NativePredictor(m, p, device=-1).run(feeds)
    for r in res:
        for a, h in zip(r, host):
            np.testing.assert_allclose(a, h, rtol=2e-4, atol=2e-5)
    before = preds[0].pooled_bytes()
    assert before > 0
    preds[0].run(feeds)
    assert preds[0].pooled_bytes() == before
    torch.cuda.set_device(0)   # torch's current device changes nothing for the predictor
    preds[1].run(feeds)


@pytest.mark.gpu
def test_native_resnet50_latency_log(tmp_path):
    """not a gate: ResNet-50 batch-8 latency of the native GPU predictor (conv + BN folded) next to
    the Python predictor on the same files, for the log"""
    import time
    from paddle_hackathon_amd.vision.models import resnet50
    paddle.seed(0)
    m, p = _save(tmp_path, resnet50(), [InputSpec([None, 3, 224, 224], "float32", "x")], "r50")
    feeds = {"x": np.random.RandomState(0).randn(8, 3, 224, 224).astype("float32")}
    nat = NativePredictor(m, p, device=0)
    nat.run(feeds)
    t0 = time.perf_counter()
    for _ in range(5):
        out = nat.run(feeds)
    t_nat = (time.perf_counter() - t0) / 5
    cfg = inference.Config(m, p)
    cfg.enable_use_gpu(100, 0)
    pred = inference.create_predictor(cfg)
    h = pred.get_input_handle("x")
    h.copy_from_cpu(feeds["x"])
    pred.run()
    t0 = time.perf_counter()
    for _ in range(5):
        h.copy_from_cpu(feeds["x"])
        pred.run()
        ref = [pred.get_output_handle(n).copy_to_cpu() for n in pred.get_output_names()]
    t_py = (time.perf_counter() - t0) / 5
    np.testing.assert_allclose(out[0], ref[0], rtol=5e-2, atol=5e-2)
    print(f"\n[native-infer] ResNet-50 b8 fp32: native {t_nat * 1e3:.1f} ms ({nat.applied_passes}), "
          f"python predictor {t_py * 1e3:.1f} ms")


def _relmax(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-6))


@pytest.mark.gpu
def test_native_gpu_bf16_matches_fp32(tmp_path):
    """bf16 matrix products (NativePredictor(bf16=True) / PD_ConfigEnableMkldnnBfloat16: mul / matmul
    / fc and the im2col convolutions on libpha_kernels.so's MFMA GEMM) against the fp32 device path
    on the same files, within bf16 rounding"""
    for name, m, p, feeds in _cases(tmp_path):
        ref = NativePredictor(m, p, device=0).run(feeds)
        pred = NativePredictor(m, p, device=0, bf16=True)
        got = pred.run(feeds)
        for g, r in zip(got, ref):
            assert g.shape == r.shape
            assert _relmax(g, r) < 3e-2, (name, _relmax(g, r))
        again = pred.run(feeds)
        for g, a in zip(got, again):
            np.testing.assert_array_equal(g, a)


@pytest.mark.gpu
def test_native_bf16_latency_log(tmp_path):
    """not a gate: ResNet-50 batch 8 and a BERT-base-sized encoder (4 layers, batch 8 x seq 128) on
    the native GPU predictor, fp32 vs bf16 matrix products, for the log"""
    import time
    from paddle_hackathon_amd.vision.models import resnet50

    class Enc(nn.Layer):
        def __init__(self):
            super().__init__()
            self.enc = nn.TransformerEncoder(nn.TransformerEncoderLayer(768, 12, 3072, dropout=0.0,
                                                                        activation="gelu"), 4)

        def forward(self, x):
            return self.enc(x)
    paddle.seed(0)
    rs = np.random.RandomState(0)
    cases = [("ResNet-50 b8", _save(tmp_path, resnet50(), [InputSpec([None, 3, 224, 224], "float32", "x")], "r50"),
              {"x": rs.randn(8, 3, 224, 224).astype("float32")}),
             ("encoder-768x4 b8 s128", _save(tmp_path, Enc(), [InputSpec([None, 128, 768], "float32", "x")], "enc768"),
              {"x": rs.randn(8, 128, 768).astype("float32")})]
    for name, (m, p), feeds in cases:
        res = {}
        for bf in (False, True):
            pred = NativePredictor(m, p, device=0, bf16=bf)
            out = pred.run(feeds)
            t0 = time.perf_counter()
            for _ in range(5):
                out = pred.run(feeds)
            res[bf] = ((time.perf_counter() - t0) / 5, out)
        err = _relmax(res[True][1][0], res[False][1][0])
        print(f"\n[native-infer] {name}: fp32 {res[False][0] * 1e3:.2f} ms, bf16 {res[True][0] * 1e3:.2f} ms "
              f"(max |bf16 - fp32| / max |fp32| = {err:.2e})")
        assert err < 5e-2
