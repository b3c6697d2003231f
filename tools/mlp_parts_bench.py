"""The MLP's GELU-adjacent products at the GPT-3 1.3B shape (32768 tokens, H 2048, F 8192), sustained:
backward  d pre = (dY W2^T) * gelu'(pre) (+ d b1): library NT + HIP dGELU pass / gemm4w dGELU +
column-sum epilogue / own gemm4p NT + HIP pass; forward gelu(x W1 + b1) (+ pre): gemm4p GELU epilogue /
gemm4w NN GELU epilogue / library + HIP bias-GELU pass. python tools/mlp_parts_bench.py"""
import sys

import torch

sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import gemm as G, hip  # noqa: E402
from paddle_hackathon_amd.ops.conv_gemm import weight_t  # noqa: E402
from tools.g4p_sustain import sustain  # noqa: E402


def main():
    T, H, F = 32768, 2048, 8192
    torch.manual_seed(0)
    x = torch.randn(T, H, device="cuda").bfloat16()
    w1 = (torch.randn(H, F, device="cuda") * 0.02).bfloat16()
    b1 = (torch.randn(F, device="cuda") * 0.02).bfloat16()
    w2 = (torch.randn(F, H, device="cuda") * 0.02).bfloat16()
    gy = torch.randn(T, H, device="cuda").bfloat16()
    pre = torch.randn(T, F, device="cuda").bfloat16()
    w1t = weight_t(w1)

    def bwd_lib():
        ga = gy @ w2.t()
        return hip.bias_gelu_bwd(ga, pre, b1, True)

    def bwd_4w():
        g, part = G.gemm(gy, w2, False, False, act="dgelu", aux=pre, colsum=True)
        return g, G.colsum_finish(part, b1.dtype)

    def bwd_own():
        ga = G.gemm_p(gy, w2, False, False)
        return hip.bias_gelu_bwd(ga, pre, b1, True)

    def fwd_4p():
        return G.mm_nt_bias_gelu(x, w1t, b1)

    def fwd_4w():
        return G.nn(x, w1, bias=b1, act="gelu", aux_out=True)

    def fwd_lib():
        h = x @ w1
        return hip.bias_gelu_fwd(h, b1, True), h

    for name, f in (("bwd lib NT + dGELU pass", bwd_lib), ("bwd gemm4w dGELU+colsum epilogue", bwd_4w),
                    ("bwd gemm4p NT + dGELU pass", bwd_own), ("fwd gemm4p GELU epilogue", fwd_4p),
                    ("fwd gemm4w NN GELU epilogue", fwd_4w), ("fwd lib + bias-GELU pass", fwd_lib)):
        t = sustain(f)
        print(f"{name:34s} {t * 1e6:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
