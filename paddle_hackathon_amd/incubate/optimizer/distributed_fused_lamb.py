"""``incubate.optimizer.DistributedFusedLamb`` (reference: python/paddle/incubate/optimizer/
distributed_fused_lamb.py, paddle/fluid/operators/optimizers/distributed_fused_lamb_op.cu).

LAMB over ONE flat fp32 buffer of all parameters (each parameter's slot aligned to
``alignment`` elements), with the optimizer state sharded over the data-parallel ranks:

  1. gradients are fused into the flat buffer (gradient_accumulation_steps > 1: accumulated there,
     the update runs every k-th step) and REDUCE-SCATTERED over RCCL — each rank receives the
     summed gradient of its 1/N shard (divided by N unless ``is_grad_scaled_by_nranks``);
  2. the global gradient norm is one all-reduce of the shards' squared sums (``grad_clip`` =
     ClipGradByGlobalNorm: scale = clip / max(norm, clip); ``clip_after_allreduce`` False clips
     the local gradients before the reduce);
  3. each rank updates its shard of the fp32 master weights with the moments of that shard only
     (1/N of the optimizer memory per rank); the per-parameter trust ratios ||w|| / ||r|| need
     sums over parameters that straddle shards: per-parameter partial sums (index_add over the
     shard's element -> parameter map) are all-reduced as one [2, n_params] tensor;
  4. the updated shards are ALL-GATHERED and copied back into the parameters.

One reduce-scatter, two small all-reduces and one all-gather per step — on xGMI the two large
collectives are bandwidth-optimal rings over the flat buffer. On the GPU steps 2-3 are three HIP
kernels (csrc/kernels/lamb.hip: gradient square sum; clip + moments + direction + per-parameter
norm sums; trust-ratio update), the clip scale and trust ratios staying on the device. Single-process it is exactly
``optimizer.Lamb`` (tests/test_distributed_fused_lamb.py checks 2 gloo ranks against it). Works in
dygraph and in static programs (the static optimizer op steps the optimizer)."""
from __future__ import annotations

import torch
import torch.distributed as dist

from ...framework.core import _wrap
from ...optimizer.optimizer import Lamb

__all__ = ["DistributedFusedLamb"]


class DistributedFusedLamb(Lamb):
    def __init__(self, learning_rate=0.001, lamb_weight_decay=0.01, beta1=0.9, beta2=0.999, epsilon=1e-6,
                 parameters=None, grad_clip=None, exclude_from_weight_decay_fn=None, clip_after_allreduce=True,
                 is_grad_scaled_by_nranks=True, alignment=128, use_master_param_norm=True, gradient_accumulation_steps=1,
                 use_master_acc_grad=True, nproc_per_node=None, name=None):
        from ...nn.clip import ClipGradByGlobalNorm
        super().__init__(learning_rate=learning_rate, lamb_weight_decay=lamb_weight_decay, beta1=beta1, beta2=beta2,
                         epsilon=epsilon, parameters=parameters, grad_clip=None,
                         exclude_from_weight_decay_fn=exclude_from_weight_decay_fn, name=name)
        if grad_clip is not None and not isinstance(grad_clip, ClipGradByGlobalNorm):
            raise TypeError("Only ClipGradByGlobalNorm is supported in DistributedFusedLamb")
        self._max_global_grad_norm = grad_clip.clip_norm if grad_clip is not None else -1.0
        self._clip_after_allreduce = clip_after_allreduce
        self._is_grad_scaled_by_nranks = is_grad_scaled_by_nranks
        self._alignment = max(int(alignment or 1), 1)
        self._use_master_param_norm = use_master_param_norm
        if gradient_accumulation_steps < 1:
            raise ValueError("gradient_accumulation_steps must be >= 1")
        self._gradient_accumulation_steps = int(gradient_accumulation_steps)
        self._nproc_per_node = nproc_per_node
        self._flat = None     # layout + state, built on the first step
        self._acc_count = 0

    # ---------------------------------------------------------------------------------- layout
    def _group(self):
        if dist.is_available() and dist.is_initialized():
            return dist.get_world_size(), dist.get_rank()
        return 1, 0

    def _build(self, params):
        world, rank = self._group()
        dev = params[0]._t.device
        offs, off = [], 0
        for p in params:
            offs.append(off)
            n = p._t.numel()
            off += -(-n // self._alignment) * self._alignment
        quantum = self._alignment * world
        total = -(-off // quantum) * quantum
        shard = total // world
        lo = rank * shard
        pid = torch.full((total,), len(params), dtype=torch.long, device=dev)   # padding -> dummy slot
        master = torch.zeros(total, dtype=torch.float32, device=dev)
        for i, (p, o) in enumerate(zip(params, offs)):
            n = p._t.numel()
            pid[o:o + n] = i
            m = self._master(p)
            master[o:o + n] = (m._t if m is not None else p._t).detach().reshape(-1).float()
        wd = torch.tensor([0.0 if (self._exclude is not None and self._exclude(p)) else float(self._wd)
                           for p in params] + [0.0], dtype=torch.float32, device=dev)
        lr_ratio = torch.tensor([self._lr_ratio(p, self._param_groups[0]) for p in params] + [1.0],
                                dtype=torch.float32, device=dev)
        self._flat = dict(params=list(params), ids=[id(p) for p in params], offs=offs, total=total, shard=shard,
                          pid32=pid[lo:lo + shard].to(torch.int32).contiguous(), lr_ratio=lr_ratio,
                          lo=lo, world=world, rank=rank, pid=pid[lo:lo + shard].contiguous(),
                          master=master[lo:lo + shard].clone(), m1=torch.zeros(shard, device=dev),
                          m2=torch.zeros(shard, device=dev), wd=wd,
                          acc=torch.zeros(total, dtype=torch.float32, device=dev)
                          if self._gradient_accumulation_steps > 1 else None,
                          b1p=1.0, b2p=1.0)
        # a state_dict set before the first step (the usual resume order) was only parked
        self._load_pending()

    # ---------------------------------------------------------------------------------- step
    def step(self):
        pgs = [(p, g) for p, g, _ in self._collect()]
        if not pgs:
            return
        params = [p for p, _ in pgs]
        if self._flat is None or self._flat["ids"] != [id(p) for p in params]:
            self._build(params)
        F = self._flat
        dev = F["master"].device
        flat_g = torch.zeros(F["total"], dtype=torch.float32, device=dev)
        for (p, g), o in zip(pgs, F["offs"]):
            flat_g[o:o + g._t.numel()] = g._t.detach().reshape(-1).float()
        if F["acc"] is not None:   # gradient accumulation: update on every k-th step only
            F["acc"].add_(flat_g)
            self._acc_count += 1
            if self._acc_count % self._gradient_accumulation_steps:
                return
            flat_g = F["acc"] / self._gradient_accumulation_steps
            F["acc"].zero_()
        world = F["world"]
        clip = self._max_global_grad_norm
        if clip > 0 and not self._clip_after_allreduce:
            n = flat_g.square().sum().sqrt()
            flat_g = flat_g * (clip / torch.maximum(n, torch.tensor(clip, device=dev)))
        if world > 1:
            g = torch.empty(F["shard"], dtype=torch.float32, device=dev)
            dist.reduce_scatter_tensor(g, flat_g)
            if not self._is_grad_scaled_by_nranks:
                g.div_(world)
        else:
            g = flat_g
        if self._fused_ok(dev):
            self._fused_update(F, g, world, clip)
        else:
            self._torch_update(F, g, world, clip)
        if world > 1:
            full = torch.empty(F["total"], dtype=torch.float32, device=dev)
            dist.all_gather_into_tensor(full, F["master"])
        else:
            full = F["master"]
        with torch.no_grad():
            for p, o in zip(F["params"], F["offs"]):
                n = p._t.numel()
                v = full[o:o + n].view(p._t.shape)
                m = self._master(p)
                if m is not None:
                    m._t.copy_(v)
                p._t.copy_(v.to(p._t.dtype))
        self._step_count += 1

    @staticmethod
    def _fused_ok(dev):
        from ...ops import _lib
        return dev.type == "cuda" and _lib.native_available()

    def _fused_update(self, F, g, world, clip):
        """steps 2-3 as the lamb.hip kernels (clip scale, trust ratios and lr stay on the device)"""
        from ctypes import c_float, c_int, c_long, c_void_p
        from ...ops import _lib
        L = _lib._load()
        if not getattr(L, "_lamb_sig", False):
            P = c_void_p
            L.pha_lamb_sq.argtypes = [P, c_long, P, P, P]
            L.pha_lamb_moment.argtypes = [P, P, P, P, P, P, P, c_int, c_long] + [c_float] * 7 + [P, P]
            L.pha_lamb_apply.argtypes = [P, P, P, P, P, c_int, c_long, c_float, P, P]
            L._lamb_sig = True
        dev = g.device
        st = c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        ptr = lambda t: c_void_p(0 if t is None else t.data_ptr())   # noqa: E731
        n = F["shard"]
        g = g.contiguous()
        gsq = None
        if clip > 0 and self._clip_after_allreduce:
            part = torch.empty(8192, dtype=torch.float32, device=dev)
            gsq = torch.empty(1, dtype=torch.float32, device=dev)
            rc = L.pha_lamb_sq(ptr(g), n, ptr(part), ptr(gsq), st)
            if rc:
                raise RuntimeError(f"pha_lamb_sq failed ({rc})")
            if world > 1:
                dist.all_reduce(gsq)
        b1, b2 = self._beta1, self._beta2
        F["b1p"] *= b1
        F["b2p"] *= b2
        npar = len(F["params"]) + 1
        norms = torch.zeros(2, npar, dtype=torch.float32, device=dev)
        rc = L.pha_lamb_moment(ptr(g), ptr(F["m1"]), ptr(F["m2"]), ptr(F["master"]), ptr(F["pid32"]), ptr(F["wd"]),
                               ptr(norms), npar, n, b1, b2, 1 - F["b1p"], 1 - F["b2p"], self._epsilon, 1.0,
                               clip if gsq is not None else 0.0, ptr(gsq), st)
        if rc:
            raise RuntimeError(f"pha_lamb_moment failed ({rc})")
        if world > 1:
            dist.all_reduce(norms)
        rc = L.pha_lamb_apply(ptr(F["master"]), ptr(g), ptr(F["pid32"]), ptr(norms), ptr(F["lr_ratio"]), npar, n,
                              float(self.get_lr()), None, st)
        if rc:
            raise RuntimeError(f"pha_lamb_apply failed ({rc})")

    def _torch_update(self, F, g, world, clip):
        dev = g.device
        if clip > 0 and self._clip_after_allreduce:
            sq = g.square().sum().reshape(1)
            if world > 1:
                dist.all_reduce(sq)
            n = sq.sqrt()
            g = g * (clip / torch.maximum(n, torch.tensor(clip, device=dev)))
        b1, b2 = self._beta1, self._beta2
        F["b1p"] *= b1
        F["b2p"] *= b2
        m1, m2, w, pid = F["m1"], F["m2"], F["master"], F["pid"]
        m1.mul_(b1).add_(g, alpha=1 - b1)
        m2.mul_(b2).addcmul_(g, g, value=1 - b2)
        r = (m1 / (1 - F["b1p"])) / ((m2 / (1 - F["b2p"])).sqrt() + self._epsilon) + F["wd"][pid] * w
        npar = len(F["params"]) + 1
        norms = torch.zeros(2, npar, dtype=torch.float32, device=dev)
        norms[0].index_add_(0, pid, w * w)
        norms[1].index_add_(0, pid, r * r)
        if world > 1:
            dist.all_reduce(norms)
        wn, rn = norms[0].sqrt(), norms[1].sqrt()
        trust = torch.where((wn > 0) & (rn > 0), wn / rn.clamp_min(1e-30), torch.ones_like(wn))
        lr = float(self.get_lr())
        w.sub_(lr * (F["lr_ratio"] * trust)[pid] * r)

    # ---------------------------------------------------------------------------------- state
    def state_dict(self):
        sd = {}
        if self._flat is not None:
            F = self._flat
            r = F["rank"]
            sd = {f"dfl_moment1_shard{r}": _wrap(F["m1"]), f"dfl_moment2_shard{r}": _wrap(F["m2"]),
                  f"dfl_master_shard{r}": _wrap(F["master"]), "dfl_beta_pows": [F["b1p"], F["b2p"]],
                  "dfl_step": self._step_count}
        if hasattr(self._learning_rate, "state_dict"):
            sd["LR_Scheduler"] = self._learning_rate.state_dict()
        return sd

    def set_state_dict(self, state_dict):
        if "LR_Scheduler" in state_dict and hasattr(self._learning_rate, "set_state_dict"):
            self._learning_rate.set_state_dict(state_dict["LR_Scheduler"])
        self._pending_state = state_dict
        if self._flat is not None:
            self._load_pending()

    def _load_pending(self):
        st = getattr(self, "_pending_state", None)
        if not st or self._flat is None:
            return
        F = self._flat
        r = F["rank"]
        for k, name in (("m1", "moment1"), ("m2", "moment2"), ("master", "master")):
            v = st.get(f"dfl_{name}_shard{r}")
            if v is not None:
                F[k].copy_(v._t if hasattr(v, "_t") else torch.as_tensor(v))
        if "dfl_beta_pows" in st:
            F["b1p"], F["b2p"] = st["dfl_beta_pows"]
        self._step_count = st.get("dfl_step", self._step_count)
        self._pending_state = None
