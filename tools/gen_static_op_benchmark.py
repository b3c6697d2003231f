"""Measure the static per-op benchmark table of paddle.cost_model on this GPU (MI355X):
forward and forward + backward time of each op at one config, through the framework's public
ops (the same kernels a program runs), CUDA-event timed, median of 20 after 5 warmups.

  python tools/gen_static_op_benchmark.py [out.json]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import paddle_hackathon_amd as paddle  # noqa: E402
import paddle_hackathon_amd.nn.functional as F  # noqa: E402


def _cfg(**shapes):
    return "".join(f"{k} (Variable) - dtype: {d}, shape: {list(s)}\n" for k, (d, s) in shapes.items())


def _time(fn, grad_of=None):
    ts = []
    for i in range(25):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        out = fn()
        if grad_of is not None:
            out.backward(grad_of(out))
        b.record()
        torch.cuda.synchronize()
        if i >= 5:
            ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def _t(shape, dtype="float32", grad=True, scale=1.0):
    t = paddle.to_tensor(torch.randn(*shape, device="cuda") * scale).astype(dtype)
    t.stop_gradient = not grad
    return t


def cases():
    f32 = "float32"
    x = lambda *s: _t(s)  # noqa: E731
    yield "abs", _cfg(x=(f32, [16, 128, 257, 257])), lambda a: paddle.abs(a), [x(16, 128, 257, 257)]
    yield "relu", _cfg(x=(f32, [16, 128, 257, 257])), lambda a: F.relu(a), [x(16, 128, 257, 257)]
    yield "sigmoid", _cfg(x=(f32, [16, 1024, 1024])), lambda a: F.sigmoid(a), [x(16, 1024, 1024)]
    yield "tanh", _cfg(x=(f32, [16, 1024, 1024])), lambda a: paddle.tanh(a), [x(16, 1024, 1024)]
    yield "exp", _cfg(x=(f32, [16, 1024, 1024])), lambda a: paddle.exp(a), [x(16, 1024, 1024)]
    yield "gelu", _cfg(x=(f32, [16, 1024, 4096])), lambda a: F.gelu(a), [x(16, 1024, 4096)]
    yield "elementwise_add", _cfg(x=(f32, [50, 128, 1000]), y=(f32, [50, 128, 1000])), \
        lambda a, b: a + b, [x(50, 128, 1000), x(50, 128, 1000)]
    yield "elementwise_mul", _cfg(x=(f32, [50, 128, 1000]), y=(f32, [128, 1000])), \
        lambda a, b: a * b, [x(50, 128, 1000), x(128, 1000)]
    yield "scale", _cfg(x=(f32, [16, 1024, 1024])), lambda a: paddle.scale(a, 2.0, 1.0), [x(16, 1024, 1024)]
    yield "matmul_v2", _cfg(x=(f32, [4096, 4096]), y=(f32, [4096, 4096])), lambda a, b: paddle.matmul(a, b), \
        [x(4096, 4096), x(4096, 4096)]
    yield "matmul_v2", _cfg(x=("bfloat16", [8192, 8192]), y=("bfloat16", [8192, 8192])), \
        lambda a, b: paddle.matmul(a, b), [_t([8192, 8192], "bfloat16"), _t([8192, 8192], "bfloat16")]
    yield "conv2d", _cfg(input=(f32, [16, 256, 56, 56]), filter=(f32, [256, 256, 3, 3])), \
        lambda a, w: F.conv2d(a, w, padding=1), [x(16, 256, 56, 56), _t([256, 256, 3, 3], scale=0.02)]
    yield "conv2d", _cfg(input=("bfloat16", [64, 256, 56, 56]), filter=("bfloat16", [256, 256, 3, 3])), \
        lambda a, w: F.conv2d(a, w, padding=1), [_t([64, 256, 56, 56], "bfloat16"),
                                                 _t([256, 256, 3, 3], "bfloat16", scale=0.02)]
    bn = paddle.nn.BatchNorm2D(256)
    yield "batch_norm", _cfg(x=(f32, [64, 256, 56, 56])), lambda a: bn(a), [x(64, 256, 56, 56)]
    ln = paddle.nn.LayerNorm(1024)
    yield "layer_norm", _cfg(x=(f32, [16, 1024, 1024])), lambda a: ln(a), [x(16, 1024, 1024)]
    yield "softmax", _cfg(x=(f32, [16, 16, 512, 512])), lambda a: F.softmax(a, -1), [x(16, 16, 512, 512)]
    yield "pool2d", _cfg(x=(f32, [64, 256, 56, 56])), lambda a: F.max_pool2d(a, 2), [x(64, 256, 56, 56)]
    yield "reduce_mean", _cfg(x=(f32, [16, 2048, 1024])), lambda a: paddle.mean(a, axis=-1), [x(16, 2048, 1024)]
    yield "reduce_sum", _cfg(x=(f32, [16, 2048, 1024])), lambda a: paddle.sum(a, axis=1), [x(16, 2048, 1024)]
    yield "transpose2", _cfg(x=(f32, [16, 512, 16, 64])), lambda a: paddle.transpose(a, [0, 2, 1, 3]), \
        [x(16, 512, 16, 64)]
    yield "concat", _cfg(x0=(f32, [16, 512, 1024]), x1=(f32, [16, 512, 1024])), \
        lambda a, b: paddle.concat([a, b], 1), [x(16, 512, 1024), x(16, 512, 1024)]
    emb = paddle.nn.Embedding(50304, 1024)
    ids = paddle.to_tensor(torch.randint(0, 50304, (16, 512), device="cuda"))
    yield "lookup_table_v2", _cfg(ids=("int64", [16, 512]), w=(f32, [50304, 1024])), lambda: emb(ids), []
    lab = paddle.to_tensor(torch.randint(0, 1000, (4096, 1), device="cuda"))
    yield "softmax_with_cross_entropy", _cfg(logits=(f32, [4096, 1000]), label=("int64", [4096, 1])), \
        lambda a: F.softmax_with_cross_entropy(a, lab), [x(4096, 1000)]
    yield "dropout", _cfg(x=(f32, [16, 1024, 1024])), lambda a: F.dropout(a, 0.1), [x(16, 1024, 1024)]


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "paddle_hackathon_amd", "cost_model",
        "static_op_benchmark_mi355x.json")
    paddle.set_device("gpu")
    dev = torch.cuda.get_device_name(0)
    rows = []
    counts = {}
    for op, cfg, fn, args in cases():
        def fwd():
            with paddle.no_grad():
                return fn(*args)
        tf = _time(fwd)
        tb = _time(lambda: fn(*args), grad_of=lambda o: paddle.ones_like(o))
        k = counts.get(op, 0)
        counts[op] = k + 1
        rows.append({"name": f"{op}_{k}", "op": op, "op_count": 1, "config": cfg, "device": dev,
                     "paddle_gpu_time": round(tf, 5), "paddle_gpu_time_backward": round(tb, 5)})
        print(f"{op:28s} fwd {tf:8.4f} ms  fwd+bwd {tb:8.4f} ms  {cfg.strip()}", flush=True)
    with open(out_path, "w") as f:
        json.dump(rows, f, indent=1)
    print("wrote", out_path)


if __name__ == "__main__":
    main()
