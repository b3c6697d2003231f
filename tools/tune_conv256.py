"""Measure the own conv kernels' tile choices for the ResNet-50 training shapes (NHWC and NCHW, the
bench batch and the test batch) by timing, and write them to the committed table
(paddle_hackathon_amd/tuning/conv256_gfx950.json) that ops/conv_gemm.py reads — so every run and
every rank picks the same kernels.

  python tools/tune_conv256.py [--batch 256 ...]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import paddle_hackathon_amd as paddle  # noqa: E402
from paddle_hackathon_amd.ops import conv_gemm  # noqa: E402
from paddle_hackathon_amd.vision.models import resnet50  # noqa: E402


def run(batch, fmt):
    paddle.seed(0)
    kw = {"data_format": "NHWC"} if fmt == "NHWC" else {}
    model = paddle.amp.decorate(resnet50(**kw), level="O2", dtype="bfloat16")
    opt = paddle.optimizer.Momentum(learning_rate=0.1, momentum=0.9, parameters=model.parameters(),
                                    multi_precision=True)
    shape = (batch, 224, 224, 3) if fmt == "NHWC" else (batch, 3, 224, 224)
    x = paddle.to_tensor(torch.randn(*shape, device="cuda").bfloat16())
    y = paddle.to_tensor(torch.randint(0, 1000, (batch,), device="cuda"))
    for _ in range(2):
        with paddle.amp.auto_cast(level="O2", dtype="bfloat16"):
            loss = paddle.nn.functional.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        opt.clear_grad(set_to_zero=False)
    torch.cuda.synchronize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[256])
    ap.add_argument("--formats", nargs="+", default=["NHWC", "NCHW"])
    ap.add_argument("--out", default=conv_gemm.TUNING_TABLE)
    ap.add_argument("--retune-tn", action="store_true",
                    help="re-time only the weight-gradient / TN launches (tile x split-K), keep the other picks")
    ap.add_argument("--retune-all", action="store_true", help="re-time every launch of the run (conv and TN)")
    a = ap.parse_args()
    paddle.set_device("gpu")
    conv_gemm.set_timing_autotune(True)
    conv_gemm._retune_tn[0] = a.retune_tn or a.retune_all
    conv_gemm._retune_conv[0] = a.retune_all
    for b in a.batch:
        for f in a.formats:
            run(b, f)
            print(f"tuned ResNet-50 {f} batch {b}: {len(conv_gemm._tuned)} picks", flush=True)
    n = conv_gemm.dump_tuning(a.out)
    print(f"wrote {n} entries to {a.out}")


if __name__ == "__main__":
    main()
