"""Sustained-load NT GEMM timing (power / clock steady state, as inside a training step): each
variant runs back to back for ~1.5 s on model-like data (weights N(0, 0.02), unit-variance
activations); the reported time is the mean of the last second. Own gemm4p (LV 0 / 8) vs hipBLASLt.
python tools/g4p_sustain.py"""
import os
import sys
import time

import torch

sys.path.insert(0, ".")
from paddle_hackathon_amd.ops import gemm as G  # noqa: E402

T = 32768


SECS = float(os.environ.get("SUSTAIN_SECS", "1.5"))
SHAPES = os.environ.get("SHAPES")


def sustain(fn, secs=SECS, tail=None):
    tail = secs * 2 / 3 if tail is None else tail
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < secs - tail:
        fn()
        n += 1
        if n % 8 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    m = 0
    while time.perf_counter() - t1 < tail:
        for _ in range(8):
            fn()
        m += 8
        torch.cuda.synchronize()
    return (time.perf_counter() - t1) / m


def main():
    tot = {}
    for name, N, K in (("fc2 fwd", 2048, 8192), ("qkv dX", 2048, 6144), ("qkv fwd", 6144, 2048),
                       ("out fwd", 2048, 2048), ("fc2 dX", 8192, 2048)):
        if SHAPES and name not in SHAPES.split(","):
            continue
        x = torch.randn(T, K, device="cuda").bfloat16()
        wt = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
        b = torch.randn(N, device="cuda") * 0.02
        fl = 2.0 * T * N * K
        lvs = os.environ.get("LVS", "0,8").split(",")
        var = {}
        for lv in lvs:
            if lv == "adeep":   # no-bias kernel: compared with the no-bias two-buffer build and x @ w^T
                var["lv8nb"] = lambda: G.gemm_p(x, wt, epi_extra=G.EPI_EARLY | (8 << 17))
                var["adeep"] = lambda: G.gemm_p(x, wt, epi_extra=G.EPI_EARLY | G.EPI_ADEEP)
                var["libnb"] = lambda: x @ wt.t()
                continue
            epi = G.EPI_EARLY | (G.EPI_RING if lv == "ring" else int(lv) << 17)
            var["ring" if lv == "ring" else f"lv{lv}"] = (lambda epi=epi: G.gemm_p(x, wt, bias=b, epi_extra=epi))
        var["lib"] = lambda: torch.addmm(b.bfloat16(), x, wt.t())
        res = {}
        for rep in range(2):
            for k, fn in var.items():
                res.setdefault(k, []).append(sustain(fn))
        med = {k: min(v) for k, v in res.items()}
        for k, v in med.items():
            tot[k] = tot.get(k, 0.0) + v
        print(f"NT {name} {T}x{N}x{K}: " + "  ".join(f"{k} {med[k] * 1e6:.0f}us/{fl / med[k] / 1e12:.0f}TF"
                                                    for k in var), flush=True)
    print("sum: " + "  ".join(f"{k} {v * 1e3:.2f}ms" for k, v in tot.items()), flush=True)


if __name__ == "__main__":
    main()
