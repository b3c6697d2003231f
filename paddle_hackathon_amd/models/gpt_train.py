"""The GPT pre-training step as bench.py times it, for every fleet layout BASELINE.json names:
data parallel, tensor parallel (DP x TP), pipeline parallel (1F1B, optionally x TP) and sharding
(stage 1 / 2 / 3, alone or under pipeline parallel) — one construction path shared by the
benchmark and by the gloo parity tests (tests/test_bench_layouts.py), so what the 8-GPU scaling
run measures is what the CPU tests check against single-process training.

Reference layouts: python/paddle/distributed/fleet/base/topology.py (dp x mp x pp x sharding
groups), meta_parallel/pipeline_parallel.py (1F1B), meta_parallel/sharding/
group_sharded_stage{2,3}.py, fleetx GPT configs.

Rank roles: tensor-parallel and pipeline peers see the same tokens; data-parallel and sharding
ranks see different ones (both split the batch), so ``data_ranks = dp * sharding``.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

_LEVEL = {1: "os", 2: "os_g", 3: "p_g_os"}


@dataclass
class Layout:
    world: int = 1
    tp: int = 1
    pp: int = 1
    sharding_stage: int = 0     # 0: no sharding; 1/2/3: group-sharded over all data ranks
    micro_batches: int = 1      # pipeline accumulate_steps

    @property
    def data_ranks(self):
        return self.world // (self.tp * self.pp)

    @property
    def dp(self):
        return 1 if self.sharding_stage else self.data_ranks

    @property
    def sharding(self):
        return self.data_ranks if self.sharding_stage else 1

    def name(self):
        s = f"dp{self.dp}"
        if self.tp > 1:
            s += f"_tp{self.tp}"
        if self.pp > 1:
            s += f"_pp{self.pp}"
        if self.sharding_stage:
            s += f"_sharding{self.sharding}-stage{self.sharding_stage}"
        return s


def _tp_slice(state, model, rank, tp):
    """the slices of a full state dict that tensor-parallel rank ``rank`` of ``tp`` holds: each
    tensor whose shape differs from the model's parameter is split along the differing dim"""
    import numpy as np
    params = dict(model.named_parameters())
    out = {}
    for name, v in state.items():
        p = params.get(name)
        v = np.asarray(v)
        if p is None or tuple(p.shape) == v.shape:
            out[name] = v
            continue
        d = [i for i in range(v.ndim) if v.shape[i] != p.shape[i]][0]
        out[name] = np.ascontiguousarray(np.split(v, tp, axis=d)[rank % tp])
    return out


class GPTTrainer:
    """``step(inp, lab) -> loss`` for one rank of the layout (inp / lab: this rank's token block,
    [batch, seq] int64; with pipeline parallelism the batch is cut into ``micro_batches``)."""

    def __init__(self, model_name, layout: Layout, rank=0, lr=1e-4, amp=True, clip=1.0, cfg_overrides=None,
                 state=None, optimizer="adamw"):
        import paddle_hackathon_amd as paddle
        from paddle_hackathon_amd import distributed as dist
        from paddle_hackathon_amd.models import gpt_config, GPTForPretraining, GPTForPretrainingPipe
        lo = layout
        if lo.world % (lo.tp * lo.pp):
            raise SystemExit(f"tp {lo.tp} x pp {lo.pp} must divide the world size {lo.world}")
        self.layout, self.rank = lo, rank
        hcg = None
        if lo.world > 1:
            strategy = dist.fleet.DistributedStrategy()
            strategy.hybrid_configs = {"dp_degree": lo.dp, "mp_degree": lo.tp, "pp_degree": lo.pp,
                                       "sharding_degree": lo.sharding}
            if lo.pp > 1:
                strategy.pipeline_configs = {"micro_batch_size": 1, "accumulate_steps": lo.micro_batches}
            dist.fleet.init(is_collective=True, strategy=strategy)
            hcg = dist.fleet.get_hybrid_communicate_group()
            self.strategy = strategy
        cfg = gpt_config(model_name, tensor_parallel_degree=lo.tp, **(cfg_overrides or {}))
        self.cfg = cfg
        if lo.pp > 1:
            model = GPTForPretrainingPipe(cfg, topology=hcg.topology())
            if state is not None:
                model.set_state_dict_from_gpt(state)
        else:
            model = GPTForPretraining(cfg)
            if state is not None:
                if lo.tp > 1:   # a full (single-card) state: this rank's tensor-parallel slices
                    state = _tp_slice(state, model, hcg.get_model_parallel_rank(), lo.tp)
                model.set_state_dict({k: paddle.to_tensor(v) for k, v in state.items()})
        if amp:
            model = paddle.amp.decorate(model, level="O2", dtype="bfloat16")
        self.inner = model
        gc = paddle.nn.ClipGradByGlobalNorm(clip) if clip else None
        if optimizer == "adamw":
            opt = paddle.optimizer.AdamW(learning_rate=lr, beta1=0.9, beta2=0.95, weight_decay=0.1,
                                         parameters=model.parameters(), grad_clip=gc, multi_precision=amp)
        else:
            opt = paddle.optimizer.SGD(learning_rate=lr, parameters=model.parameters(), grad_clip=gc)
        self.n_params = sum(p._t.numel() for p in model.parameters())
        if lo.sharding_stage and lo.sharding > 1:
            from paddle_hackathon_amd.parallel.sharding import group_sharded_parallel
            keep = getattr(model, "shared_parameters", lambda: [])()
            # stage 3 shards parameters of >= segment elements (PHA_STAGE3_SEGMENT; the tests force
            # the tiny models' blocks to shard too)
            seg = int(os.environ.get("PHA_STAGE3_SEGMENT", str(2 ** 20)))
            m2, opt, _ = group_sharded_parallel(model, opt, _LEVEL[lo.sharding_stage], segment_size=seg,
                                                group=hcg.get_sharding_parallel_group(), replicate=keep)
            if lo.pp == 1:
                model = m2
            else:
                # the global-norm clip spans the pipeline stages too (hybrid check group)
                clip_obj = getattr(opt, "_grad_clip", None)
                cg = hcg.get_check_parallel_group()
                if clip_obj is not None and cg is not None and cg.nranks > 1:
                    clip_obj._check_group = cg.pg
                    clip_obj._mp_degree = lo.tp
        if lo.pp > 1:
            model = dist.fleet.distributed_model(model)
        elif lo.world > 1 and not lo.sharding_stage:
            model = dist.fleet.distributed_model(model)
            opt = dist.fleet.distributed_optimizer(opt)
        self.model, self.opt = model, opt

    def data_rank(self):
        """index of this rank's token block among the data ranks (dp x sharding)"""
        lo = self.layout
        if lo.world == 1:
            return 0
        from paddle_hackathon_amd import distributed as dist
        hcg = dist.fleet.get_hybrid_communicate_group()
        d = hcg.get_data_parallel_rank() if lo.dp > 1 else 0
        s = hcg.get_sharding_parallel_rank() if lo.sharding > 1 else 0
        return d * lo.sharding + s

    def step(self, inp, lab):
        if self.layout.pp > 1:
            return self.model.train_batch([inp, lab], self.opt)
        loss = self.model(inp, lab)
        loss.backward()
        self.opt.step()
        self.opt.clear_grad(set_to_zero=False)
        return loss
