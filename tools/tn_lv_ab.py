"""Weight gradients (TN, K = 98,304 tokens: GPT-3 1.3B at micro-batch 48) with the bias column sums
(mm_tn_db), gemm4p schedule variant LV 0 (shipped) vs 8 (PIN) vs 40 (PIN + SPREAD DMA placement),
interleaved rounds after a sustained warm-up; results must be bitwise equal.
python tools/tn_lv_ab.py"""
import os
import sys
import time

import torch

sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import gemm as G  # noqa: E402

T = int(os.environ.get("TOK", 98304))


def main():
    tot = {}
    for name, M, N in (("qkv dW", 2048, 6144), ("fc1 dW", 2048, 8192), ("fc2 dW", 8192, 2048), ("bert qkv dW", 768, 2304)):
        K = T if not name.startswith("bert") else 16384
        x = torch.randn(K, M, device="cuda").bfloat16()
        dy = torch.randn(K, N, device="cuda").bfloat16()
        outs = {}

        def run(lv):
            os.environ["PHA_G4P_TN_LV"] = str(lv)
            return G.mm_tn_db(x, dy)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 1.0:
            run(0)
            torch.cuda.synchronize()
        res = {}
        for _ in range(3):
            for lv in (0, 8, 40):
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                for _ in range(5):
                    run(lv)
                torch.cuda.synchronize()
                res.setdefault(lv, []).append((time.perf_counter() - t1) / 5)
        for lv in (0, 8, 40):
            outs[lv] = run(lv)
        eq = all(torch.equal(outs[lv][0], outs[0][0]) and torch.equal(outs[lv][1], outs[0][1]) for lv in (8, 40))
        fl = 2.0 * M * N * K
        print(f"{name} {M}x{N}x{K}: " + "  ".join(f"lv{lv} {min(v) * 1e6:.0f}us/{fl / min(v) / 1e12:.0f}TF" for lv, v in res.items())
              + f"  bitwise_equal={eq}", flush=True)
        for lv, v in res.items():
            tot[lv] = tot.get(lv, 0.0) + min(v)
        del x, dy
    print("sum: " + "  ".join(f"lv{lv} {v * 1e6:.0f}us" for lv, v in tot.items()), flush=True)


if __name__ == "__main__":
    main()
