"""Which aten ops (and shapes) launch the GPT-3 1.3B step's torch-native kernels: two profiled
training steps, CPU ops grouped by input shape, sorted by the device time of the kernels they
launched. python tools/gpt_aten_ops.py [micro_batch]"""
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
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        for _ in range(steps):
            tr.step(inp, lab)
        torch.cuda.synchronize()
    rows = []
    for e in prof.key_averages(group_by_input_shape=True):
        if not e.key.startswith("aten::"):
            continue
        dev = getattr(e, "self_device_time_total", None)
        if dev is None:
            dev = e.self_cuda_time_total
        if dev <= 0:
            continue
        rows.append((dev / steps, e.count / steps, e.key, str(e.input_shapes)[:150]))
    rows.sort(reverse=True)
    print(f"aten self device time {sum(r[0] for r in rows) / 1e3:.2f} ms/step")
    for us, n, k, shp in rows[:40]:
        print(f"{us / 1e3:8.3f} ms/step {n:6.1f}/step  {k:28s} {shp}")


if __name__ == "__main__":
    main()
