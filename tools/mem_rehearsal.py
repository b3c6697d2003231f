"""Per-rank peak HBM of the BASELINE multi-GPU layouts, rehearsed on ONE MI355X: every rank of an
N-rank torchrun job (gloo collectives, PHA_DIST_BACKEND=gloo) lives on cuda:0 and runs the real
GPTTrainer step of bench.py (fleet topology, TP / PP / sharding, DP reducer buckets, AdamW fp32
master) at a reduced depth L; torch.cuda.max_memory_allocated is per process, so each rank's peak
is its own. Two depths give peak(L) = a + b L per rank, extrapolated to the model's full depth
and compared with the 288 GB of an MI355X (the target keeps >= 15 % headroom).

torchrun --nproc-per-node N tools/mem_rehearsal.py --model gpt3-1.3b --tp 4 --layers 2 --micro-batch 16
(run by tools/gpu_r6_mem.sh; not for the real multi-GPU job, which the driver runs)"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt3-1.3b")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--pp", type=int, default=1)
    ap.add_argument("--sharding-stage", type=int, default=0)
    ap.add_argument("--layers", type=int, required=True)
    ap.add_argument("--micro-batch", type=int, required=True)
    ap.add_argument("--seq-len", type=int, default=2048)
    ap.add_argument("--recompute", action="store_true")
    a = ap.parse_args()
    os.environ.setdefault("PHA_DIST_BACKEND", "gloo")
    import torch
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd import distributed as dist
    from paddle_hackathon_amd.models.gpt_train import GPTTrainer, Layout
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        dist.init_parallel_env()
    rank = dist.get_rank()
    gpu = torch.cuda.is_available()
    if gpu:
        torch.cuda.set_device(0)
    paddle.set_device("gpu:0" if gpu else "cpu")
    paddle.seed(1234 + rank)
    lo = Layout(world=world, tp=a.tp, pp=a.pp, sharding_stage=a.sharding_stage,
                micro_batches=2 * a.pp if a.pp > 1 else 1)
    tr = GPTTrainer(a.model, lo, rank, lr=1e-4, amp=True, clip=1.0,
                    cfg_overrides={"num_layers": a.layers, "max_position_embeddings": max(2048, a.seq_len),
                                   "recompute": a.recompute})
    B, S = a.micro_batch, a.seq_len
    dev = "cuda" if gpu else "cpu"
    g = torch.Generator(device=dev)
    g.manual_seed(tr.data_rank())
    ids = paddle.to_tensor(torch.randint(0, tr.cfg.vocab_size, (B, S + 1), device=dev, generator=g))
    inp, lab = paddle.Tensor(ids[:, :-1]._t.contiguous()), paddle.Tensor(ids[:, 1:]._t.contiguous())
    for _ in range(2):
        loss = tr.step(inp, lab)
    if gpu:
        torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated() / 2 ** 30 if gpu else 0.0
    res = {"rank": rank, "peak_gb": round(peak, 2),
           "reserved_gb": round(torch.cuda.max_memory_reserved() / 2 ** 30, 2) if gpu else 0.0,
           "loss": round(float(loss.item()), 4)}
    import torch.distributed as td
    allr = [None] * world
    if world > 1:
        td.all_gather_object(allr, res)
    else:
        allr = [res]
    if rank == 0:
        print(json.dumps({"model": a.model, "layout": lo.name(), "world": world, "layers": a.layers,
                          "micro_batch": B, "recompute": a.recompute, "ranks": allr}), flush=True)
    if world > 1:
        td.barrier()


if __name__ == "__main__":
    main()
