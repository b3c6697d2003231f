"""gemm256 (or, with argument "8p", the 8-phase gemm8p) at M=N=K=8192 (bf16 random) for
rocprofv3 PMC passes."""
import sys
import torch
sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import conv_gemm  # noqa: E402
a = (torch.rand(8192, 8192, device="cuda") * 2 - 1).bfloat16()
b = (torch.rand(8192, 8192, device="cuda") * 2 - 1).bfloat16()
for _ in range(3):
    if "8p" in sys.argv[1:]:
        conv_gemm.gemm8p(a, b)
    else:
        conv_gemm.gemm256_nt(a, b)
torch.cuda.synchronize()
print("done")
