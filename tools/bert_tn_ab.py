"""BERT-base weight gradients (TN, K = B*S = 16,384 tokens, x^T dY + the bias column sums): the
persistent gemm4p TN kernel at every split-K factor (fp32 slabs + in-order reduce, column sums
from its B fragments) vs the gemm256 TN kernel family (128/256-wide tiles, autotuned tile x split)
+ the HIP column sum, vs hipBLASLt + column sum. python tools/bert_tn_ab.py"""
import os
import sys

import torch

sys.path.insert(0, ".")
os.environ.setdefault("PHA_CONV_TUNE", "1")
from paddle_hackathon_amd.ops import gemm as G  # noqa: E402
from paddle_hackathon_amd.ops import conv_gemm as CG  # noqa: E402
from paddle_hackathon_amd.ops import hip as H  # noqa: E402

K = int(os.environ.get("TOK", 16384))


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    tot = {}
    for name, M, N in (("qkv dW", 768, 2304), ("out dW", 768, 768), ("fc1 dW", 768, 3072), ("fc2 dW", 3072, 768)):
        x = torch.randn(K, M, device="cuda").bfloat16()
        dy = torch.randn(K, N, device="cuda").bfloat16()
        ref = (x.float().t() @ dy.float())
        res = {}
        for sp in (1, 2, 4, 8, 16):
            def own(sp=sp):
                c, part = G.gemm_p(x, dy, True, True, splits=sp, colsum=True)
                return c, G.colsum_rows_finish(part, torch.bfloat16)
            c, _ = own()
            err = ((c.float() - ref).norm() / ref.norm()).item()
            res[f"g4p s{sp}"] = (timeit(own), err)
        res[f"g4p auto(s{G._splits(M, N, K, x.device)})"] = (timeit(lambda: G.mm_tn_db(x, dy)), 0.0)

        def g256():
            return CG.gemm256_tn(x, dy), H.col_sum(dy, torch.bfloat16)
        c, _ = g256()
        res["g256 tuned"] = (timeit(g256), ((c.float() - ref).norm() / ref.norm()).item())
        res["lib"] = (timeit(lambda: (x.t() @ dy, H.col_sum(dy, torch.bfloat16))), 0.0)
        fl = 2.0 * M * N * K
        print(f"{name} {M}x{N}x{K}: " + "  ".join(f"{k} {v[0]:.1f}us/{fl / v[0] / 1e6:.0f}TF" + (f" e{v[1]:.1e}" if v[1] else "")
                                                  for k, v in res.items()), flush=True)
        print(f"   g256 pick: {CG._tuned.get(('tn', x.dtype, M, N, K))}", flush=True)
        for k, v in res.items():
            tot[k.split('(')[0]] = tot.get(k.split('(')[0], 0.0) + v[0]
    print("per layer sum: " + "  ".join(f"{k} {v:.0f}us" for k, v in tot.items()), flush=True)


if __name__ == "__main__":
    main()
