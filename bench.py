#!/usr/bin/env python
"""Headline benchmark: GPT-3 1.3B pre-training tokens/sec under fleet data parallelism
(BASELINE.json: "samples/sec/GPU ResNet-50 bf16 + tokens/sec GPT-3-1.3B fleet DP at 1/2/4/8 MI355X").

    python bench.py --gpus N --steps K --warmup W            # N>1: spawns N ranks itself
    torchrun --nproc-per-node N bench.py --gpus N ...         # or the driver's launcher

With ``--gpus N > 1`` and no ``WORLD_SIZE`` in the environment the script starts N worker
processes of itself (one per GPU, RCCL rendezvous on 127.0.0.1) through the in-tree launcher
before anything touches the GPU, and exits with the job's code. Under a launcher, ``WORLD_SIZE``
must equal ``--gpus`` or the script exits non-zero.

Each step = forward + backward + AdamW update (fp32 master weights) of the full
24-layer GPT-3 1.3B (hidden 2048, 16 heads, ffn 8192, vocab 50304, seq 2048) in
bf16 on synthetic token ids; weak scaling (micro-batch per GPU fixed).
The other half of BASELINE's metric, ResNet-50 bf16 samples/sec (batch 256 per GPU, NHWC,
Momentum), runs on the same ranks right after the GPT timing and is reported inside the same JSON
line (``config.resnet50_samples_per_sec``, whole job; ``--no-resnet`` skips it). A single-rank job
replays that step as one hipGraph and also times it eagerly (``config.resnet50_eager_samples_per_sec``),
the mode multi-rank jobs use, so the eager numbers form a like-for-like 1 -> N curve;
``--model resnet50`` measures only that config.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

BASELINE_METRIC = "samples/sec/GPU ResNet-50 bf16 + tokens/sec GPT-3-1.3B fleet DP at 1/2/4/8 MI355X"


def _args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="gpt3-1.3b")
    ap.add_argument("--micro-batch", type=int, default=None,
                    help="per-GPU batch (default: GPT 48 x 2048 tokens, BERT 32, ResNet 256); GPT micro-batch 16 "
                         "measured +7.6 %% tokens/s over 8, 32 +1.3 %% over 16, 48 +0.5 %% over 32 on one MI355X "
                         "(bigger GEMMs, the optimizer and the gradient all-reduce amortised over more tokens; "
                         "183 GB of the 288 GB HBM at 48 — 64 adds another +0.5 %% at 237 GB, too little headroom "
                         "for the multi-rank buffers; profiles/gpt3_micro_batch_r5.txt); ResNet 512 measured "
                         "slower than 256")
    ap.add_argument("--seq-len", type=int, default=2048)
    ap.add_argument("--recompute", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--tp", type=int, default=1, help="GPT tensor-parallel degree (dp = gpus / (tp * pp))")
    ap.add_argument("--pp", type=int, default=1, help="GPT pipeline-parallel degree (1F1B over RCCL p2p)")
    ap.add_argument("--micro-batches", type=int, default=None,
                    help="pipeline: micro-batches per step (default: 2 * pp); the per-GPU batch is cut into them")
    ap.add_argument("--sharding-stage", type=int, default=0, choices=[0, 1, 2, 3],
                    help="GPT: group-sharded data parallelism over the gpus / (tp * pp) data ranks (1: optimizer "
                         "state, 2: + gradients, 3: + parameters); composes with --pp (BASELINE config 5: "
                         "--model gpt3-13b --pp 2 --sharding-stage 3 --recompute on 8 GPUs)")
    ap.add_argument("--gemm-tuning", default="off", choices=["db", "tune", "off"],
                    help="off (default): the library heuristics for the products the static policy leaves on "
                         "hipBLASLt; db: load the in-tree TunableOp solution database (within noise of off: "
                         "124.4 / 123.4k vs 124.2 / 122.9k tokens/s alternating on one box, "
                         "profiles/gemm_tuning_db_ab_r5.txt); tune: benchmark solutions and write the database")
    ap.add_argument("--gemm-tuning-file", default=None, help="database path (default: the in-tree one)")
    ap.add_argument("--gemm-tuning-ms", type=int, default=15, help="tune: time budget per GEMM shape")
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="replay the whole training step (fwd + bwd + optimizer) as one hipGraph "
                         "(paddle.device.cuda.graphs.wrap_cuda_graph). auto: BERT on a single rank (its eager "
                         "step is host-bound: graphed 1,242-1,275 vs eager 1,236 samples/s), ResNet-50 eager "
                         "(eager measured ahead of the graph in every alternating pair: 9,086 / 9,077, 9,077 / "
                         "9,012, 9,123 / 9,082 img/s); on: graph (multi-rank: builds the model and reducer on "
                         "the capture stream and captures the RCCL all-reduce — unverified across ranks, one "
                         "GPU per test box); off: eager")
    ap.add_argument("--force-dp", action="store_true",
                    help="ResNet-50: wrap the model in DataParallel (RCCL reducer) even on one rank — checks the "
                         "graph-captured all-reduce path on a single GPU")
    ap.add_argument("--no-resnet", action="store_true",
                    help="GPT-3 1.3B run: skip the ResNet-50 half of the headline metric (by default it runs after "
                         "the GPT timing, same --steps/--warmup, and lands in config.resnet50_*)")
    return ap.parse_args()


def _self_launch(a):
    """--gpus N without a launcher: run N ranks of this script (children, not exec: the parent never
    initialises the GPU) and return the job's exit code."""
    from paddle_hackathon_amd.parallel.spawn import launch
    import torch
    n_dev = torch.cuda.device_count()   # does not initialise HIP on this image
    if n_dev < a.gpus:
        print(f"[bench] --gpus {a.gpus} but only {n_dev} GPU(s) visible", file=sys.stderr, flush=True)
        return 2
    return launch(["--nproc_per_node", str(a.gpus), os.path.abspath(__file__)] + sys.argv[1:])


def main():
    a = _args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        sys.exit(_self_launch(a))
    # only when a multi-rank ResNet step captures its RCCL all-reduce into the hipGraph (--graph on)
    # must the NCCL watchdog stop polling events of captured work (torch's documented setting for
    # graphed DDP); everywhere else it stays on, so an RCCL fault or desync aborts instead of hanging
    if int(env_world or 1) > 1 and a.graph == "on" and a.warmup >= 2 and \
            os.environ.get("PHA_DIST_BACKEND", "nccl") == "nccl":
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "0")
    if env_world is not None and int(env_world) != a.gpus:
        print(f"[bench] WORLD_SIZE={env_world} disagrees with --gpus {a.gpus}", file=sys.stderr, flush=True)
        sys.exit(2)
    import torch
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd import distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        dist.init_parallel_env()
    rank = dist.get_rank()
    # ranks beyond the visible GPUs share them (only the one-GPU multi-rank rehearsal, PHA_DIST_BACKEND=gloo)
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count()))
    paddle.set_device(f"gpu:{torch.cuda.current_device()}")
    paddle.seed(1234 + rank)
    if a.gemm_tuning != "off":
        from paddle_hackathon_amd.incubate import autotune
        n = autotune.enable_gemm_tuning(tune=(a.gemm_tuning == "tune"), filename=a.gemm_tuning_file,
                                        max_tuning_ms=a.gemm_tuning_ms)
        if rank == 0:
            print(f"[bench] gemm tuning={a.gemm_tuning} entries={n}", file=sys.stderr, flush=True)

    if a.model.startswith("resnet"):
        return bench_resnet(a, paddle, dist, world, rank)
    if a.model.startswith("bert"):
        return bench_bert(a, paddle, dist, world, rank)

    from paddle_hackathon_amd.models.gpt_train import GPTTrainer, Layout
    tp, pp = max(1, a.tp), max(1, a.pp)
    if world % (tp * pp):
        raise SystemExit(f"--tp {tp} x --pp {pp} must divide the world size {world}")
    B, S = _gpt_micro_batch(a, torch, world, rank), a.seq_len
    lo = Layout(world=world, tp=tp, pp=pp, sharding_stage=a.sharding_stage,
                micro_batches=(a.micro_batches or 2 * pp) if pp > 1 else 1)
    if pp > 1 and B % lo.micro_batches:
        raise SystemExit(f"--micro-batch {B} must be a multiple of --micro-batches {lo.micro_batches}")
    tr = GPTTrainer(a.model, lo, rank, lr=1e-4, amp=True, clip=1.0,
                    cfg_overrides={"max_position_embeddings": max(2048, S), "recompute": a.recompute})
    cfg = tr.cfg
    model = tr.model
    dp = lo.data_ranks
    gen = torch.Generator(device="cuda")
    # tensor / pipeline peers see the same tokens: seed by data rank
    gen.manual_seed(tr.data_rank())
    ids = paddle.to_tensor(torch.randint(0, cfg.vocab_size, (B, S + 1), device="cuda", generator=gen))
    inp, lab = ids[:, :-1], ids[:, 1:]
    inp = paddle.Tensor(inp._t.contiguous())
    lab = paddle.Tensor(lab._t.contiguous())

    def step():
        return tr.step(inp, lab)

    for i in range(a.warmup):
        tw = time.perf_counter()
        loss = step()
        torch.cuda.synchronize()
        if rank == 0:
            print(f"[bench] warmup {i} loss={float(loss.item()):.4f} {time.perf_counter() - tw:.3f}s", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device="cuda")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    ms = elapsed / a.steps * 1000.0
    tokens = B * S * dp * a.steps
    value = tokens / elapsed
    if rank == 0:
        n_params = tr.n_params
        out = {
            "metric": ("tokens/sec GPT-3-1.3B fleet DP (bf16, whole job)" if a.model == "gpt3-1.3b" else
                       f"tokens/sec {a.model} (bf16, whole job)"),
            "baseline_metric": BASELINE_METRIC,
            "value": round(value, 2), "unit": "tokens/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16", "data": "synthetic (random token ids), random-init weights",
            "config": {"model": "GPT-3-1.3B" if a.model == "gpt3-1.3b" else a.model, "global_batch": B * dp,
                       "seq_len": S, "parallelism": lo.name(), "micro_batch_per_gpu": B,
                       "n_params": n_params,
                       "optimizer": "AdamW fp32-master", "final_loss": round(float(loss.item()), 4),
                       "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2 ** 30, 1)},
        }
    if a.model == "gpt3-1.3b" and not a.no_resnet:
        # the second half of BASELINE's metric: ResNet-50 samples/s on the same ranks
        final_loss = float(loss.item())
        del model, tr, loss, ids, inp, lab, step
        import gc
        gc.collect()
        torch.cuda.empty_cache()
        r = bench_resnet(a, paddle, dist, world, rank, emit=False)
        r_eager = r
        if r["config"]["hip_graph"]:
            # the same step timed eagerly too, so a 1 -> N curve of the eager numbers compares like
            # with like (multi-rank jobs time ResNet eagerly unless --graph on)
            gc.collect()
            torch.cuda.empty_cache()
            r_eager = bench_resnet(argparse.Namespace(**{**vars(a), "graph": "off"}), paddle, dist, world, rank,
                                   emit=False)
        if rank == 0:
            out["config"]["final_loss"] = round(final_loss, 4)
            out["config"].update({"resnet50_samples_per_sec": r["value"],
                                  "resnet50_samples_per_sec_per_gpu": r["config"]["samples_per_sec_per_gpu"],
                                  "resnet50_ms_per_step": r["ms_per_step"],
                                  "resnet50_global_batch": r["config"]["global_batch"],
                                  "resnet50_hip_graph": r["config"]["hip_graph"],
                                  "resnet50_eager_samples_per_sec": r_eager["value"],
                                  "resnet50_eager_samples_per_sec_per_gpu":
                                      r_eager["config"]["samples_per_sec_per_gpu"]})
    if rank == 0:
        print(json.dumps(out), flush=True)


def _timed(a, step, world, rank, dist):
    import torch
    for i in range(a.warmup):
        tw = time.perf_counter()
        loss = step()
        torch.cuda.synchronize()
        if rank == 0:
            print(f"[bench] warmup {i} loss={float(loss.item()):.4f} {time.perf_counter() - tw:.3f}s", file=sys.stderr,
                  flush=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device="cuda")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, loss


def bench_bert(a, paddle, dist, world, rank):
    """BERT-base pre-training (MLM 15 % masked positions + NSP), seq 512, bf16 O2, AdamW. Replayed as
    one hipGraph under the same policy as ResNet (--graph): the eager step is host-bound (Python
    issue time ~ GPU time, profiles/bert_host_prof_r6.log); dropout masks stay fresh per replay
    through the kernels' device seed word (ops/hip.dropout_seed), Adam reads lr / beta powers from
    device scalars."""
    import torch
    cap_stream = torch.cuda.Stream() if _bert_graphed(a, world) else torch.cuda.current_stream()
    with torch.cuda.stream(cap_stream):
        return _bench_bert(a, paddle, dist, world, rank, cap_stream)


def _bench_bert(a, paddle, dist, world, rank, cap_stream):
    import torch
    from paddle_hackathon_amd.models import bert_config, BertForPretraining, BertPretrainingCriterion
    S = a.seq_len if a.seq_len != 2048 else 512
    B = a.micro_batch or 32
    cfg = bert_config(a.model if a.model in ("bert-base", "bert-large", "bert-tiny") else "bert-base",
                      max_position_embeddings=max(512, S))
    model = BertForPretraining(cfg)
    crit = BertPretrainingCriterion(cfg.vocab_size)
    model = paddle.amp.decorate(model, level="O2", dtype="bfloat16")
    opt = paddle.optimizer.AdamW(learning_rate=1e-4, weight_decay=0.01, parameters=model.parameters(),
                                 multi_precision=True)
    if world > 1:
        strategy = dist.fleet.DistributedStrategy()
        strategy.hybrid_configs = {"dp_degree": world, "mp_degree": 1, "pp_degree": 1}
        dist.fleet.init(is_collective=True, strategy=strategy)
        model = dist.fleet.distributed_model(model)
        opt = dist.fleet.distributed_optimizer(opt)
    g = torch.Generator(device="cuda")
    g.manual_seed(rank)
    ids = paddle.to_tensor(torch.randint(0, cfg.vocab_size, (B, S), device="cuda", generator=g))
    tt = paddle.to_tensor((torch.arange(S, device="cuda") >= S // 2).long().expand(B, S).contiguous())
    n_mask = max(1, int(0.15 * S))
    mpos = paddle.to_tensor((torch.randperm(S, device="cuda", generator=g)[:n_mask].unsqueeze(0)
                             + S * torch.arange(B, device="cuda").unsqueeze(1)).reshape(-1))
    mlab = paddle.to_tensor(torch.randint(0, cfg.vocab_size, (B * n_mask,), device="cuda", generator=g))
    nlab = paddle.to_tensor(torch.randint(0, 2, (B,), device="cuda", generator=g))

    def step():
        with paddle.amp.auto_cast(level="O2", dtype="bfloat16"):
            mlm, nsp = model(ids, tt, masked_positions=mpos)
        loss = crit(mlm, nsp, mlab, nlab)
        loss.backward()
        opt.step()
        opt.clear_grad(set_to_zero=False)
        return loss

    graphed = _bert_graphed(a, world)
    if graphed:
        from paddle_hackathon_amd.device.cuda.graphs import wrap_cuda_graph
        step = wrap_cuda_graph(step)
        step._stream = cap_stream
    elapsed, loss = _timed(a, step, world, rank, dist)
    value = B * world * a.steps / elapsed
    if rank == 0:
        print(json.dumps({
            "metric": "samples/sec BERT-base pretraining bf16 (whole job)", "baseline_metric": BASELINE_METRIC,
            "value": round(value, 2), "unit": "samples/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1000, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16", "data": "synthetic token ids / masks, random-init weights",
            "config": {"model": "BERT-base" if cfg.hidden_size == 768 else a.model, "global_batch": B * world,
                       "seq_len": S, "parallelism": f"dp{world}", "tokens_per_sec": round(value * S, 1),
                       "final_loss": round(float(loss.item()), 4), "hip_graph": bool(graphed)}}), flush=True)


def _graphed(a, world, auto):
    """whether a step is replayed as one hipGraph (see --graph); ``auto``: the model's default on
    a single rank"""
    if a.warmup < 2 or a.graph == "off":
        return False
    from paddle_hackathon_amd.parallel import collective
    if world > 1 and collective.get_backend() != "nccl":
        return False   # host (gloo) collectives cannot be captured
    return a.graph == "on" or (auto and world == 1)


def _resnet_graphed(a, world):
    return _graphed(a, world, auto=False)


def _bert_graphed(a, world):
    return _graphed(a, world, auto=True)


def _gpt_micro_batch(a, torch, world, rank):
    """per-GPU micro-batch: --micro-batch, else 2 for the larger GPTs, else 48 for GPT-3 1.3B
    (182.9 GB peak) when every rank has the free HBM for it — stepping down to 32 (128.5 GB) or 16
    (74 GB) otherwise, so a card with less free memory than an MI355X's 288 GB runs instead of
    failing; ranks agree on the smallest free memory, so they all pick the same size"""
    if a.micro_batch:
        return a.micro_batch
    if a.model != "gpt3-1.3b":
        return 2
    if max(1, a.tp) > 1 or max(1, a.pp) > 1 or a.sharding_stage or a.recompute:
        return 16   # the free-memory thresholds below were measured for the plain DP layout only
    free_gb = torch.cuda.mem_get_info()[0] / 2 ** 30
    # ranks that share one device (a gloo rehearsal on one GPU) each get their share of it
    per_dev = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")) // max(1, torch.cuda.device_count()))
    free_gb /= per_dev
    if world > 1:
        import torch.distributed as td
        t = torch.tensor([free_gb], dtype=torch.float64,
                         device="cuda" if td.get_backend() == "nccl" else "cpu")
        td.all_reduce(t, op=td.ReduceOp.MIN)
        free_gb = float(t.item())
    for mb, need_gb in ((48, 200), (32, 145), (16, 90)):
        if free_gb >= need_gb:
            break
    if mb != 48 and rank == 0:
        print(f"[bench] {free_gb:.0f} GB free HBM: GPT micro-batch {mb} instead of 48", file=sys.stderr, flush=True)
    return mb


def bench_resnet(a, paddle, dist, world, rank, emit=True):
    import torch
    # model, reducer hooks and every step run on one stream: the capture stream when graphed
    cap_stream = torch.cuda.Stream() if _resnet_graphed(a, world) else torch.cuda.current_stream()
    with torch.cuda.stream(cap_stream):
        return _bench_resnet(a, paddle, dist, world, rank, emit, cap_stream)


def _bench_resnet(a, paddle, dist, world, rank, emit, cap_stream):
    import torch
    from paddle_hackathon_amd.vision.models import resnet50
    model = resnet50(data_format="NHWC")
    model = paddle.amp.decorate(model, level="O2", dtype="bfloat16")
    opt = paddle.optimizer.Momentum(learning_rate=0.1, momentum=0.9, parameters=model.parameters(),
                                    weight_decay=paddle.regularizer.L2Decay(1e-4), multi_precision=True)
    if world > 1 or a.force_dp:
        if world == 1 and not torch.distributed.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29555")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
            dist.init_parallel_env()
        model = paddle.DataParallel(model)
    B = (a.micro_batch if a.model.startswith("resnet") else None) or 256
    x = paddle.to_tensor(torch.randn(B, 224, 224, 3, device="cuda").to(torch.bfloat16))
    y = paddle.to_tensor(torch.randint(0, 1000, (B,), device="cuda"))

    def step():
        with paddle.amp.auto_cast(level="O2", dtype="bfloat16"):
            out = model(x)
        loss = paddle.nn.functional.cross_entropy(out, y)
        loss.backward()
        opt.step()
        opt.clear_grad(set_to_zero=False)
        return loss

    graphed = _resnet_graphed(a, world)
    if graphed:
        # warmup call 1 runs eagerly (GEMM picks, allocator growth), call 2 captures and replays:
        # every timed step is one replay of the full forward + backward + optimizer kernels, on the
        # stream the model and reducer were built on (autograd's AccumulateGrad nodes then match
        # the capture stream)
        from paddle_hackathon_amd.device.cuda.graphs import wrap_cuda_graph
        step = wrap_cuda_graph(step)
        step._stream = cap_stream
    elapsed, loss = _timed(a, step, world, rank, dist)
    value = B * world * a.steps / elapsed
    res = {
            "metric": "samples/sec ResNet-50 bf16 (whole job)", "baseline_metric": BASELINE_METRIC,
            "value": round(value, 2), "unit": "samples/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1000, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16", "data": "synthetic ImageNet-shaped, random-init weights",
            "config": {"model": "ResNet-50", "global_batch": B * world, "seq_len": None, "parallelism": f"dp{world}",
                       "layout": "NHWC", "samples_per_sec_per_gpu": round(value / world, 2),
                       "hip_graph": bool(graphed), "data_parallel_reducer": bool(world > 1 or a.force_dp)}}
    if emit and rank == 0:
        print(json.dumps(res), flush=True)
    return res


if __name__ == "__main__":
    main()
