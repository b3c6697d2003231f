"""fp32 (Paddle's default dtype) training on the own kernels (three-term bf16 split, ops/conv_gemm.py
split3 / ops/gemm.py mm_f32) vs MIOpen / hipBLASLt fp32 (PHA_CONV_F32=library, PHA_MATMUL_F32=library):
ResNet-50 NCHW training steps and square fp32 GEMMs.

  python tools/bench_fp32.py
  python tools/bench_fp32.py resnet hip|library     (ResNet-50 only, one side)
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import paddle_hackathon_amd as paddle  # noqa: E402
from paddle_hackathon_amd.vision import models  # noqa: E402


def resnet_ms(impl, batch=64, steps=6, warmup=3):
    os.environ["PHA_CONV_F32"] = impl
    os.environ["PHA_MATMUL_F32"] = impl
    paddle.seed(0)
    model = models.resnet50()
    opt = paddle.optimizer.Momentum(learning_rate=0.01, momentum=0.9, parameters=model.parameters())
    x = paddle.to_tensor(torch.randn(batch, 3, 224, 224, device="cuda"))
    y = paddle.to_tensor(torch.randint(0, 1000, (batch,), device="cuda"))

    def one():
        loss = paddle.nn.functional.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        opt.clear_grad(set_to_zero=False)
        return loss
    for _ in range(warmup):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = one()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3, float(loss.item())


def gemm_tf(impl, n):
    from paddle_hackathon_amd.ops import gemm as G
    a = torch.randn(n, n, device="cuda")
    b = torch.randn(n, n, device="cuda")
    f = (lambda: G.mm_f32(a, b)) if impl == "hip" else (lambda: a @ b)
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        c = f()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 10
    ref = (a.double() @ b.double())
    err = ((c.double() - ref).abs().max() / ref.abs().max()).item()
    return 2 * n ** 3 / dt / 1e12, err


def main():
    paddle.set_device("gpu")
    if len(sys.argv) > 2 and sys.argv[1] == "resnet":   # one side only (for rocprofv3)
        ms, loss = resnet_ms(sys.argv[2])
        print(f"resnet50 fp32 NCHW batch 64 conv/matmul={sys.argv[2]}: {ms:7.1f} ms/step loss {loss:.4f}")
        return
    for n in (2048, 4096, 8192):
        for impl in ("hip", "library"):
            tf, err = gemm_tf(impl, n)
            print(f"fp32 GEMM {n}^3 {impl:7s}: {tf:7.1f} TF/s  max rel err {err:.1e}", flush=True)
    for impl in ("hip", "library"):
        ms, loss = resnet_ms(impl)
        print(f"resnet50 fp32 NCHW batch 64 conv/matmul={impl:7s}: {ms:7.1f} ms/step {64 / ms * 1e3:6.0f} img/s "
              f"loss {loss:.4f}", flush=True)


if __name__ == "__main__":
    main()
