"""Fit the per-rank peak HBM that tools/mem_rehearsal.py measured at two reduced depths,
peak(L) = a + b * L for every rank of a layout, and extrapolate to the model's full depth.
Verdict per layout: the worst rank's extrapolated reserved memory plus an RCCL allowance must
leave >= 15 % of an MI355X's 288 GB free.

python tools/mem_fit.py gpurun_out/mem_r6.jsonl"""
import json
import sys
from collections import defaultdict

HBM_GB = 288.0
RCCL_GB = 2.0       # RCCL channel buffers + proxy FIFOs for <= 7 peers (NCCL_BUFFSIZE 4 MiB x channels), rounded up
FULL = {"gpt3-1.3b": 24, "gpt3-13b": 40}


def main(path):
    runs = defaultdict(dict)
    for line in open(path):
        line = line.strip()
        if not line.startswith("{"):
            continue
        r = json.loads(line)
        key = (r["model"], r["layout"], r["micro_batch"], r["recompute"], r["world"])
        runs[key][r["layers"]] = r["ranks"]
    ok_all = True
    print(f"{'model':10s} {'layout':22s} {'mb':>3s} {'rc':>3s}  depths   worst-rank alloc / reserved at full depth"
          f"  + RCCL {RCCL_GB:.0f} GB  headroom")
    for (model, layout, mb, rc, world), by_l in sorted(runs.items()):
        if len(by_l) < 2:
            print(f"{model:10s} {layout:22s} only one depth measured: {sorted(by_l)}")
            ok_all = False
            continue
        l0, l1 = sorted(by_l)[:2]
        full = FULL.get(model)
        worst = (0.0, 0.0)
        for r0, r1 in zip(sorted(by_l[l0], key=lambda r: r["rank"]), sorted(by_l[l1], key=lambda r: r["rank"])):
            ext = []
            for k in ("peak_gb", "reserved_gb"):
                b = (r1[k] - r0[k]) / (l1 - l0)
                ext.append(r0[k] + b * (full - l0))
            worst = max(worst, tuple(ext), key=lambda e: max(e))
        need = max(worst) + RCCL_GB   # the larger of the two fits (reserved grows slower at small L)
        head = 1.0 - need / HBM_GB
        ok = head >= 0.15
        ok_all &= ok
        print(f"{model:10s} {layout:22s} {mb:3d} {'y' if rc else 'n':>3s}  L={l0},{l1}->{full:<3d} "
              f"{worst[0]:7.1f} / {worst[1]:7.1f} GB      {need:7.1f} GB   {100 * head:5.1f} %  {'OK' if ok else 'OVER'}")
    print("all layouts keep >= 15 % headroom" if ok_all else "some layout misses the 15 % headroom")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
