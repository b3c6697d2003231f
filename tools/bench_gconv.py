"""ResNeXt-50 32x4d training steps (bf16 O2, NCHW, eager): grouped 3x3 convolutions on the grouped
implicit GEMM (PHA_GCONV_MFMA=1, ops/conv_gemm.py conv2d_nhwc256_grouped) vs the direct VALU kernels
(PHA_GCONV_MFMA=0) vs MIOpen (PHA_CONV_IMPL=library), alternated on one box.

  python tools/bench_gconv.py
  python tools/bench_gconv.py 1 hip     (one variant, e.g. under rocprofv3)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_conv_formats import step_ms  # noqa: E402
import paddle_hackathon_amd as paddle  # noqa: E402


def main():
    paddle.set_device("gpu")
    if len(sys.argv) > 1:   # one variant only (for rocprofv3): bench_gconv.py MFMA(0|1) IMPL(hip|library)
        os.environ["PHA_GCONV_MFMA"] = sys.argv[1]
        ms = step_ms("resnext50_32x4d", "NCHW", 64, sys.argv[2] if len(sys.argv) > 2 else "hip")
        print(f"resnext50_32x4d batch 64 gconv_mfma={sys.argv[1]}: {ms:7.1f} ms/step", flush=True)
        return
    for rep in range(2):
        for mfma, impl in (("1", "hip"), ("0", "hip"), ("1", "library")):
            os.environ["PHA_GCONV_MFMA"] = mfma
            ms = step_ms("resnext50_32x4d", "NCHW", 64, impl)
            print(f"resnext50_32x4d batch 64 conv={impl:7s} gconv_mfma={mfma}: {ms:7.1f} ms/step "
                  f"{64 / ms * 1e3:7.0f} img/s", flush=True)


if __name__ == "__main__":
    main()
