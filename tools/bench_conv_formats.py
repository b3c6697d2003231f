"""Training-step time of zoo CNNs by data format and conv implementation (one GPU, bf16 O2,
Momentum, eager): ResNet-50 NCHW (the default, kept channels-last in memory by the own kernels) vs
NHWC, and MobileNetV2 / ResNeXt-50 on the own direct grouped / depthwise kernels vs MIOpen
(PHA_CONV_IMPL=library).

  python tools/bench_conv_formats.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import paddle_hackathon_amd as paddle  # noqa: E402
from paddle_hackathon_amd.vision import models  # noqa: E402


def step_ms(name, fmt, batch, impl, steps=8, warmup=3, hw=224):
    os.environ["PHA_CONV_IMPL"] = impl
    paddle.seed(0)
    kw = {"data_format": fmt} if fmt == "NHWC" else {}
    model = paddle.amp.decorate(getattr(models, name)(**kw), level="O2", dtype="bfloat16")
    opt = paddle.optimizer.Momentum(learning_rate=0.01, momentum=0.9, parameters=model.parameters(),
                                    multi_precision=True)
    shape = (batch, hw, hw, 3) if fmt == "NHWC" else (batch, 3, hw, hw)
    x = paddle.to_tensor(torch.randn(*shape, device="cuda").bfloat16())
    y = paddle.to_tensor(torch.randint(0, 1000, (batch,), device="cuda"))

    def one():
        with paddle.amp.auto_cast(level="O2", dtype="bfloat16"):
            loss = paddle.nn.functional.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        opt.clear_grad(set_to_zero=False)

    for _ in range(warmup):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    paddle.set_device("gpu")
    rows = [("resnet50", "NHWC", 128, "hip"), ("resnet50", "NCHW", 128, "hip"), ("resnet50", "NCHW", 128, "library"),
            ("mobilenet_v2", "NCHW", 128, "hip"), ("mobilenet_v2", "NCHW", 128, "library"),
            ("resnext50_32x4d", "NCHW", 64, "hip"), ("resnext50_32x4d", "NCHW", 64, "library")]
    for name, fmt, b, impl in rows:
        ms = step_ms(name, fmt, b, impl)
        print(f"{name:16s} {fmt} batch {b:3d} conv={impl:7s}: {ms:7.1f} ms/step  {b / ms * 1e3:7.0f} img/s", flush=True)


if __name__ == "__main__":
    main()
