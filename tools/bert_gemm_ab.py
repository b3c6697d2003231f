"""BERT-base NT products (M = 32 x 512 tokens, H = 768): hipBLASLt vs the own persistent gemm4p
(256 x 256 tiles) vs gemm256_nt at every tile / BK (sustained timing, interleaved), to route the
768-wide products onto tiles that fill 256 CUs. python tools/bert_gemm_ab.py"""
import os
import sys
import time

import torch

sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import gemm as G  # noqa: E402
from paddle_hackathon_amd.ops import conv_gemm as CG  # noqa: E402

M = int(os.environ.get("BERT_M", 16384))
SHAPES = [("qkv fwd", 2304, 768), ("out fwd", 768, 768), ("fc1 fwd", 3072, 768), ("fc2 fwd", 768, 3072),
          ("qkv dX", 768, 2304), ("fc1 dX", 768, 3072), ("fc2 dX", 3072, 768)]


def timed(fn, secs=0.25):
    fn()
    torch.cuda.synchronize()
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < secs:
        for _ in range(10):
            fn()
        n += 10
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


def main():
    L, z = CG._L256(), CG._ptr(CG._zero_page(torch.device("cuda")))
    tot = {}
    for name, N, K in SHAPES:
        a = torch.randn(M, K, device="cuda").bfloat16()
        bt = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        st = torch.cuda.current_stream().cuda_stream

        def g256(tile, bk):
            def f():
                rc = L.pha_gemm256_nt(CG._DT[a.dtype], CG._ptr(a), CG._ptr(bt), CG._ptr(c), None, M, N, K, K, K, N, 0,
                                      z, tile, bk, torch.cuda.current_stream().cuda_stream)
                assert rc == 0
            return f
        var = {"lib": lambda: torch.matmul(a, bt.t(), out=c), "g4p": lambda: G.gemm_p(a, bt, out=c)}
        for t in range(6):
            for bk in (32, 64):
                var[f"g256_{t}_{bk}"] = g256(t, bk)
        ref = (a.float() @ bt.float().t())
        res = {}
        for _ in range(2):
            for k, f in var.items():
                res.setdefault(k, []).append(timed(f))
        for k, f in var.items():   # correctness of each variant
            c.zero_()
            f()
            torch.cuda.synchronize()
            err = ((c.float() - ref).norm() / ref.norm()).item()
            assert err < 1e-2, (name, k, err)
        best = {k: min(v) for k, v in res.items()}
        own = min((v, k) for k, v in best.items() if k != "lib")
        fl = 2.0 * M * N * K
        print(f"{name:8s} N={N:5d} K={K:5d}: lib {best['lib'] * 1e6:7.1f}us ({fl / best['lib'] / 1e12:5.0f}TF)  "
              f"g4p {best['g4p'] * 1e6:7.1f}us  best own {own[1]} {own[0] * 1e6:7.1f}us ({fl / own[0] / 1e12:5.0f}TF)  "
              f"own/lib {own[0] / best['lib']:.3f}", flush=True)
        tot["lib"] = tot.get("lib", 0) + best["lib"]
        tot["own"] = tot.get("own", 0) + own[0]
    print(f"sum per layer: lib {tot['lib'] * 1e6:.0f}us own-best {tot['own'] * 1e6:.0f}us", flush=True)


if __name__ == "__main__":
    main()
