"""Where the GPT-3 1.3B step's torch-native kernels come from: two training steps under
torch.profiler with Python stacks; for every non-own kernel class (fills, copies, reductions, cat,
memsets) print its device time per step and the top framework call sites that launched it.
python tools/gpt_torch_kernels.py [micro_batch]"""
import collections
import sys

import torch

sys.path.insert(0, ".")


def main():
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.models.gpt_train import GPTTrainer, Layout
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    S = 2048
    paddle.set_device("gpu:0")
    paddle.seed(1234)
    tr = GPTTrainer("gpt3-1.3b", Layout(world=1, tp=1, pp=1, sharding_stage=0, micro_batches=1), 0, lr=1e-4,
                    amp=True, clip=1.0, cfg_overrides={"max_position_embeddings": S})
    ids = torch.randint(0, tr.cfg.vocab_size, (B, S + 1), device="cuda")
    inp, lab = paddle.Tensor(ids[:, :-1].contiguous()), paddle.Tensor(ids[:, 1:].contiguous())
    for _ in range(2):
        tr.step(inp, lab)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    steps = 2
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for _ in range(steps):
            tr.step(inp, lab)
        torch.cuda.synchronize()
    own = ("pha::", "anonymous namespace", "Cijk", "gemm", "fa_", "ln_", "adam", "bias_gelu", "col_", "softmax_ce",
           "transpose16", "embedding", "splitk")
    per_kernel = collections.defaultdict(float)
    sites = collections.defaultdict(lambda: collections.Counter())
    events = prof.events()
    by_id = {e.id: e for e in events}
    for e in events:
        if e.device_type.name != "CUDA" and getattr(e, "device_type", None) is not None and str(e.device_type) != "DeviceType.CUDA":
            continue
        name = e.name
        if any(o in name for o in own):
            continue
        per_kernel[name[:90]] += e.device_time_total if hasattr(e, "device_time_total") else e.cuda_time_total
    # CPU ops with their stacks -> the kernels they launched
    for e in events:
        if str(e.device_type) == "DeviceType.CUDA":
            continue
        kids = [k for k in getattr(e, "kernels", [])]
        if not kids or not e.stack:
            continue
        frames = [f for f in e.stack if "paddle_hackathon_amd" in f and "torch/" not in f][:3]
        for k in kids:
            if any(o in k.name for o in own):
                continue
            sites[k.name[:90]][" <- ".join(frames) or e.name] += k.duration / steps
    tot = sum(per_kernel.values()) / steps
    print(f"torch-native device time {tot / 1e3:.2f} ms/step")
    for name, t in sorted(per_kernel.items(), key=lambda x: -x[1])[:14]:
        print(f"{t / steps / 1e3:8.3f} ms/step  {name}")
        for site, us in sites[name].most_common(4):
            print(f"      {us / 1e3:7.3f}  {site[:220]}")


if __name__ == "__main__":
    main()
